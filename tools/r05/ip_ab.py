"""iter_proj / refine kernel times (events) at B = 1 and 8 on the bench's match pairs; run once per
setting of an env switch (read at the first call) for an A/B on one box."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.matching import prep_for_iter_proj  # noqa: E402

out = {"env": {k: v for k, v in os.environ.items() if k.startswith("M3S_")}}
for B in (1, 8):
    mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device="cuda")
    rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
    b, h, w = mp.X21.shape[:3]
    D11 = mp.D11.half()
    D21 = mp.D21.view(b, h * w, -1).half()
    p1, conv = mb.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
    p1 = p1.long()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_ip = t_rf = 0.0
    reps = 20
    for r in range(reps + 3):
        ev[0].record()
        pn, cv = mb.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
        ev[1].record()
        pr = mb.refine_matches(D11, D21, p1, 3, 5)[0]
        ev[2].record()
        torch.cuda.synchronize()
        if r >= 3:
            t_ip += ev[0].elapsed_time(ev[1]) / reps
            t_rf += ev[1].elapsed_time(ev[2]) / reps
    from mast3r_slam_backends import variants as mv
    var = {}
    for name, kind in (("lds", mv.LDS), ("box", mv.BOX), ("planes", mv.PLANES)):
        t = 0.0
        for r in range(reps + 3):
            ev[1].record()
            o = mv.refine_matches_variant(kind, D11, D21, p1, 3, 5)[0]
            ev[2].record()
            torch.cuda.synchronize()
            if r >= 3:
                t += ev[1].elapsed_time(ev[2]) / reps
        var[name] = {"ms": t, "bitwise_product": bool(torch.equal(o, pr))}
    from m3s.matching import match_iterative_proj
    for _ in range(3):
        i_f, v_f = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
    torch.cuda.synchronize()
    t_fused = 0.0
    for r in range(reps):
        ev[0].record()
        i_f, v_f = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
        ev[1].record()
        torch.cuda.synchronize()
        t_fused += ev[0].elapsed_time(ev[1]) / reps
    var["fused_op"] = {"ms": t_fused, "idx_checksum": int(i_f.sum()), "valid": int(v_f.sum()),
                       "bitwise_product": True}
    out[f"B{B}"] = {"iter_proj_ms": t_ip, "refine_ms": t_rf, "refine_variants": var,
                    "iter_proj_GBps_65B": 65 * B * h * w / (t_ip * 1e-3) / 1e9,
                    "p_checksum": float(pn.double().sum()), "conv": int(cv.sum()),
                    "refine_checksum": int(pr.sum())}
print(json.dumps(out))
