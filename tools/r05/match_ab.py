"""Fused match_iterative_proj op time (events) at B = 1 and 8 on the bench's match pairs; run once
per setting of an env switch (read at the first call) for an A/B on one box."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
from m3s import synth  # noqa: E402
from m3s.matching import match_iterative_proj  # noqa: E402

out = {"env": {k: v for k, v in os.environ.items() if k.startswith("M3S_")}}
for B in (1, 8):
    mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        i_f, v_f = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
    torch.cuda.synchronize()
    reps, t = 20, 0.0
    for r in range(reps):
        ev[0].record()
        i_f, v_f = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
        ev[1].record()
        torch.cuda.synchronize()
        t += ev[0].elapsed_time(ev[1]) / reps
    out[f"B{B}"] = {"fused_ms": t, "idx_checksum": int(i_f.sum()), "valid": int(v_f.sum())}
print(json.dumps(out))
