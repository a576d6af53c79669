"""A/B of refine_matches builds (M3S_BACKEND_LIB selects the library): B=1 and B=8 kernel time
of refine_matches and the fused match op at 512x384, plus a checksum of the refined indices so
builds can be checked for identical outputs.  One JSON line per run."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.config import config as cfg0  # noqa: E402
from m3s.matching import match_iterative_proj, prep_for_iter_proj  # noqa: E402

dev = torch.device("cuda", 0)
mc = cfg0["matching"]
out = {"lib": os.environ.get("M3S_BACKEND_LIB", "default"), "tag": sys.argv[1] if len(sys.argv) > 1 else ""}
reps = 20
for B in (1, 8):
    mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device=dev)
    rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
    b, h, w = mp.X21.shape[:3]
    D11 = mp.D11.half()
    D21 = mp.D21.view(b, h * w, -1).half()
    p1, _ = mb.iter_proj(rays, pts, p_init, mc["max_iter"], mc["lambda_init"], mc["convergence_thresh"])
    p1 = p1.long()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_rf = t_op = 0.0
    for r in range(reps + 3):
        ev[0].record()
        (pr,) = mb.refine_matches(D11, D21, p1, mc["radius"], mc["dilation_max"])
        ev[1].record()
        idx, valid = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init)
        ev[2].record()
        torch.cuda.synchronize()
        if r >= 3:
            t_rf += ev[0].elapsed_time(ev[1]) / reps
            t_op += ev[1].elapsed_time(ev[2]) / reps
    h = hashlib.sha1(pr.cpu().numpy().tobytes() + idx.cpu().numpy().tobytes()).hexdigest()[:16]
    out[f"B{B}"] = {"refine_ms": t_rf, "match_op_ms": t_op, "sha": h}
print(json.dumps(out), flush=True)
