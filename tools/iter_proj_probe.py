"""Runs iter_proj at 512x384, B=8 (base.yaml matching parameters, the bench's synthetic pair) a
few times, for PMC profiling (tools/pmc_iter_proj.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.config import config as cfg0  # noqa: E402
from m3s.matching import prep_for_iter_proj  # noqa: E402

dev = torch.device("cuda", 0)
mc = cfg0["matching"]
mp = synth.make_match_pair(B=int(os.environ.get("B", "8")), H=384, W=512, seed=11, device=dev)
rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
for _ in range(int(os.environ.get("REPS", "5"))):
    mb.iter_proj(rays, pts, p_init, mc["max_iter"], mc["lambda_init"], mc["convergence_thresh"])
torch.cuda.synchronize()
print("done")
