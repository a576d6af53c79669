"""Edge-sharded multi-GPU Gauss-Newton (one process per GPU, RCCL over xGMI).

Partitioning: the 2E directed edges are split into contiguous,
count-balanced ranges, one per rank.  Poses / point maps / confidences of all keyframes
are replicated; idx / valid / Q live only on the owning rank.  Every GN iteration each rank
accumulates its edges into the compact block-sparse system (28 f64 per 7x7 block + 7 per
pose gradient), ONE RCCL sum all-reduce combines them (~0.3-0.9 MB at 1024 edges), and
every rank runs the same deterministic solve + retraction, so poses stay bitwise identical
without a broadcast.

The RCCL communicator is created by the backend library (``m3s_comm_init``) from a unique
id that rank 0 broadcasts through ``torch.distributed`` (gloo or nccl process group).
``HostComm`` plugs a ``torch.distributed`` all_reduce (e.g. gloo) into the same seam
(``m3s_comm_init_host``): the op's sharded path then runs unchanged with several processes on
one GPU -- the test hook for the exchange (tests/test_gpu_dist.py).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

import mast3r_slam_backends as mb


def shard_range(n_edges: int, world: int, rank: int):
    """Contiguous balanced range [lo, hi) of directed edges owned by ``rank``."""
    base, rem = divmod(n_edges, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def comm_size(comm) -> int:
    """Ranks the communicator spans, as its transport reports them (RCCL: ncclCommCount)."""
    n = ctypes.c_int(0)
    mb._raise(mb.lib.m3s_comm_size(comm.handle, ctypes.byref(n)), "comm size")
    return n.value


class RcclComm:
    """Backend-owned RCCL communicator for the op's per-iteration exchange (an all-gather of the
    ranks' f64 per-edge records; M3S_GN_GATHER=0: the all-reduce of the assembled systems)."""

    def __init__(self, rank: int, world: int, group=None, device=None):
        idb = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            buf = (ctypes.c_char * 128)()
            mb._raise(mb.lib.m3s_comm_get_unique_id(ctypes.cast(buf, ctypes.c_void_p)), "comm id")
            idb = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        if dist.get_backend(group) == "nccl":
            t = idb.to(device or torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(t, 0, group=group)
            idb = t.cpu()
        else:
            dist.broadcast(idb, 0, group=group)
        raw = (ctypes.c_char * 128).from_buffer_copy(bytes(idb.tolist()))
        h = ctypes.c_void_p()
        mb._raise(mb.lib.m3s_comm_init(ctypes.cast(raw, ctypes.c_void_p), world, rank, ctypes.byref(h)),
                  "comm init")
        self.handle = h
        self.rank, self.world = rank, world

    def close(self):
        if self.handle:
            mb.lib.m3s_comm_destroy(self.handle)
            self.handle = None


class HostComm:
    """Host-callback communicator: each iteration the library hands the staged compact
    system (f64, host memory) to ``dist.all_reduce(SUM)`` over ``group``."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.calls = 0

        def _allreduce(user, buf, count):
            try:
                t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)))
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                self.calls += 1
                return 0
            except Exception:  # noqa: BLE001 -- reported as an m3s error code
                return 1

        self._fn = mb.HOST_ALLREDUCE_FN(_allreduce)  # keep the trampoline alive
        h = ctypes.c_void_p()
        mb._raise(mb.lib.m3s_comm_init_host(self._fn, None, self.world, self.rank, ctypes.byref(h)),
                  "comm init (host)")
        self.handle = h

    def close(self):
        if self.handle:
            mb.lib.m3s_comm_destroy(self.handle)
            self.handle = None


def two_way_range(fwd, bwd, lo, hi):
    """The rank's directed edges [lo, hi) of a two-way edge store -- forward edges 0..E-1, then
    the same pairs backward (global_opt.py:104-110 order) -- as (first, second) halves of
    (idx, valid, Q) views, without concatenating: ``fwd`` / ``bwd`` are (idx, valid, Q) of the
    E forward / backward edges.  Returns (first, second_or_None)."""
    E = fwd[0].shape[0]
    a_lo, a_hi = min(lo, E), min(hi, E)
    b_lo, b_hi = max(lo, E) - E, max(hi, E) - E
    first = tuple(t[a_lo:a_hi] for t in fwd)
    second = tuple(t[b_lo:b_hi] for t in bwd)
    if a_hi == a_lo:
        return second, None
    if b_hi == b_lo:
        return first, None
    return first, second


def gauss_newton_sharded(mode, Twc, Xs, Cs, ii, jj, idx_local, valid_local, Q_local, edge_offset,
                         comm: RcclComm | HostComm | None, max_iter, delta_thresh,
                         second_half=None, **p):
    """Sharded variant of gauss_newton_{rays,calib,points}: ``ii``/``jj`` hold ALL directed
    edges, ``idx_local``/``valid_local``/``Q_local`` the rank's range starting at
    ``edge_offset`` (optionally continued by ``second_half``, see two_way_range).  Twc is
    updated in place identically on every rank."""
    mode_id = {"points": mb.GN_POINTS, "rays": mb.GN_RAYS, "calib": mb.GN_CALIB}[mode]
    if mode == "rays":
        s0, s1 = p["sigma_ray"], p["sigma_dist"]
    elif mode == "calib":
        s0, s1 = p["sigma_pixel"], p["sigma_depth"]
    else:
        s0, s1 = p["sigma_point"], 0.0
    return mb._run_gn(
        mode_id, Twc, Xs, Cs, ii, jj, idx_local, valid_local, Q_local, max_iter, delta_thresh,
        s0, s1, p.get("C_conf", 0.0), p.get("Q_conf", 1.5), K=p.get("K"),
        height=p.get("height", 0), width=p.get("width", 0), pixel_border=p.get("pixel_border", 0),
        z_eps=p.get("depth_eps", 0.0), comm=(comm.handle if comm is not None else None),
        edge_offset=edge_offset, edge_total=ii.shape[0], second_half=second_half,
    )
