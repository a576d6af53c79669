"""Host-side overhead of one GN op call (cfg3): wall time of the call vs GPU time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.geometry import constrain_points_to_ray  # noqa: E402

g = synth.make_graph("cfg3", device="cuda")
Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
for it in range(4):
    Twc = g.Twc.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mb.gauss_newton_calib(Twc, Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W, -10, 1e-6,
                          1.0, 10.0, 0.0, 1.5, 10, 0.0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"call {it}: enqueue {1e3 * (t1 - t0):.2f} ms, total {1e3 * (t2 - t0):.2f} ms", flush=True)
