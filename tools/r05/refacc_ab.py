"""A/B of reference-order accumulate builds (gn_refacc.hip, M3S_GN_ORDER=reference): saves the
per-edge Hs / gs of small rays / calib / points graphs in each contraction convention and of the
full cfg3 calib graph, for a bitwise comparison between libraries (M3S_BACKEND_LIB), and times
the reference-order op on cfg3 (10 iterations, events around each call).

    python tools/r05/refacc_ab.py OUT.npz  ->  OUT.npz + one JSON line of timings
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mast3r-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.debug import edge_hessians_gpu  # noqa: E402
from m3s.geometry import constrain_points_to_ray  # noqa: E402

L = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, sigma_point=0.05,
         C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)


def graph(mode, cfg=None, H=48, W=64, seed=5):
    g = synth.make_graph(cfg if cfg else dict(N=6, E=8), H=H, W=W, seed=seed)
    if mode == "calib":
        g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    return g


out = {}
mb.set_gn_order("reference")
for conv in ("nvcc", "nvcc_right", "off"):
    mb.set_gn_contract(conv)
    for mode in ("rays", "calib", "points"):
        g = graph(mode)
        g.valid[1, 10:90] = False
        g.Q[2, :40] = 1.0
        Hs, gs = edge_hessians_gpu(g, mode, L)
        out[f"{conv}_{mode}_Hs"], out[f"{conv}_{mode}_gs"] = Hs, gs
mb.set_gn_contract("nvcc")
g = graph("calib", cfg="cfg3", H=384, W=512, seed=None)
out["cfg3_Hs"], out["cfg3_gs"] = edge_hessians_gpu(g, "calib", L)

c = lambda t: t.cuda()
args = [c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q), g.H, g.W,
        L["pixel_border"], L["depth_eps"], L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], 10, 0.0]
ms = []
for rep in range(4):
    Twc = g.Twc.clone().cuda()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    mb.gauss_newton_calib(Twc, *args)
    e1.record()
    torch.cuda.synchronize()
    if rep:
        ms.append(e0.elapsed_time(e1))
out["cfg3_Twc_10it"] = Twc.cpu().numpy()
np.savez(sys.argv[1], **out)
print(json.dumps({"lib": os.environ.get("M3S_BACKEND_LIB", "default"), "cfg3_ref_order_ms_per_call": ms,
                  "pair_iters_per_s": 256 * 10 / (min(ms) * 1e-3)}), flush=True)
