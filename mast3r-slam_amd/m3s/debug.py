"""Debug entry points of the GN op (C ABI ``m3s_gn_build_system``).

``build_system_gpu`` runs one accumulate + assemble pass on the GPU and returns the dense
normal equations (H, b) in f64 -- the system the reference's SparseBlock builds
(gn_kernels.cu:71-113) -- optionally for one edge shard only (the multi-GPU path sums
these over ranks with RCCL).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

import mast3r_slam_backends as mb

MODES = {"points": mb.GN_POINTS, "rays": mb.GN_RAYS, "calib": mb.GN_CALIB}


def make_args(g, mode, L, Twc, edge_range=None, max_iter=1, delta=0.0, comm=None, dev="cuda",
              ws=None, dx=None, local=None):
    """Fill an ``m3s_gn_args`` for a synth.Graph-like object (tensors moved to ``dev``).
    ``local`` = (idx, valid, Q) already sliced to ``edge_range``."""
    c = lambda t: t.to(dev).contiguous()
    E = g.ii.shape[0]
    lo, hi = edge_range if edge_range is not None else (0, E)
    if local is None:
        idx, valid, Q = c(g.idx[lo:hi]), c(g.valid[lo:hi]), c(g.Q[lo:hi])
    else:
        idx, valid, Q = local
    keep = [c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), idx, valid, Q, c(g.K)]
    N, HW = g.Xs.shape[0], g.Xs.shape[1]
    a = mb.GNArgs()
    a.mode = MODES[mode]
    a.Twc = Twc.data_ptr()
    a.Xs, a.Cs, a.ii, a.jj = (t.data_ptr() for t in keep[:4])
    a.idx, a.valid, a.Q = idx.data_ptr(), valid.data_ptr(), Q.data_ptr()
    a.N, a.HW, a.E_total, a.E_local, a.edge_offset = N, HW, E, hi - lo, lo
    if mode == "rays":
        a.sigma0, a.sigma1 = L["sigma_ray"], L["sigma_dist"]
    elif mode == "calib":
        a.sigma0, a.sigma1 = L["sigma_pixel"], L["sigma_depth"]
    else:
        a.sigma0, a.sigma1 = L["sigma_point"], 0.0
    a.C_thresh, a.Q_thresh = L["C_conf"], L["Q_conf"]
    a.K = keep[7].data_ptr()
    a.height, a.width = g.H, g.W
    a.pixel_border, a.z_eps = L["pixel_border"], L["depth_eps"]
    a.max_iter, a.delta_thresh = max_iter, delta
    if dx is None:
        dx = torch.zeros((max(N - 1, 0), 7), device=dev)
    keep.append(dx)
    a.dx = dx.data_ptr()
    nbytes = mb.lib.m3s_gn_workspace_bytes(a.mode, N, HW, E, hi - lo)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    keep.append(ws)
    a.ws, a.ws_bytes = ws.data_ptr(), nbytes
    a.comm = comm
    a.order = mb._gn_order[0]
    a.contract = mb._gn_contract[0]
    a.stream = torch.cuda.current_stream(torch.device(dev)).cuda_stream
    return a, keep


def build_system_gpu(g, mode, L, edge_range=None):
    Twc = g.Twc.cuda().contiguous()
    a, keep = make_args(g, mode, L, Twc, edge_range=edge_range)
    n = 7 * (g.Xs.shape[0] - 1)
    H = np.zeros((n, n), np.float64)
    b = np.zeros((n,), np.float64)
    rc = mb.lib.m3s_gn_build_system(ctypes.byref(a), H.ctypes.data_as(ctypes.c_void_p),
                                    b.ctypes.data_as(ctypes.c_void_p))
    mb._raise(rc, "gn_build_system")
    del keep
    return H, b


def edge_hessians_gpu(g, mode, L, edge_range=None):
    """One reference-order accumulate pass (gn_refacc.hip): the reference align kernels'
    outputs Hs [4, E, 7, 7] and gs [2, E, 7] (f32) for the current poses."""
    Twc = g.Twc.cuda().contiguous()
    a, keep = make_args(g, mode, L, Twc, edge_range=edge_range)
    E = a.E_local
    Hs = np.zeros((4, E, 7, 7), np.float32)
    gs = np.zeros((2, E, 7), np.float32)
    rc = mb.lib.m3s_gn_edge_hessians(ctypes.byref(a), Hs.ctypes.data_as(ctypes.c_void_p),
                                     gs.ctypes.data_as(ctypes.c_void_p))
    mb._raise(rc, "gn_edge_hessians")
    del keep
    return Hs, gs
