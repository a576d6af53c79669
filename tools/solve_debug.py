"""One GN call with M3S_SOLVE_DEBUG=1 on a BASELINE config: prints the elimination plan (rounds,
core size) and the solve's in-kernel phase clocks (stderr)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
os.environ.setdefault("M3S_SOLVE_DEBUG", "1")
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
g = synth.make_graph(cfg, H=48, W=64, device=dev)
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # calls (kernel statistics under rocprofv3)
for _ in range(reps):
    Twc = g.Twc.clone()
    mb.gauss_newton_rays(Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, 0.003, 10.0, 0.0, 1.5, iters, 0.0)
torch.cuda.synchronize()
print("ok", cfg)
