"""Runs refine_matches at 512x384 (B=8, base.yaml radius 3 / dilation 5) a few times, for PMC
profiling of the matching kernels (tools/pmc_refine.sh).  VARIANT=1|2|3 runs a measurement-only
variant (mast3r_slam_backends.variants) instead of the product kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "8"))
mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device=dev)
W = 512
p1 = torch.stack((mp.idx_init % W, mp.idx_init // W), -1).long()
D11 = mp.D11.half()
D21 = mp.D21.view(B, 384 * 512, -1).half()
kind = int(os.environ.get("VARIANT", "0"))
for _ in range(int(os.environ.get("REPS", "5"))):
    if kind:
        from mast3r_slam_backends import variants
        variants.refine_matches_variant(kind, D11, D21, p1, 3, 5)
    else:
        mb.refine_matches(D11, D21, p1, 3, 5)
torch.cuda.synchronize()
print("done")
