"""Times the lattice-bucket MFMA refine variant (and the product kernel) at 512x384 on the bench's
matching data; M3S_VARIANTS_LIB selects a diagnostics build of libm3s_variants.so."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from mast3r_slam_backends import variants as mv  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.matching import prep_for_iter_proj  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "1"))
mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device=dev)
rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
p1, _ = mb.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
p1 = p1.long()
D11 = mp.D11.half()
D21 = mp.D21.view(B, 384 * 512, -1).half()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def t_ms(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


mv.variant_stats(True)
(lat,) = mv.refine_matches_variant(mv.LATTICE, D11, D21, p1, 3, 5)
resc, tot = mv.variant_stats(False)
(ref,) = mb.refine_matches(D11, D21, p1, 3, 5)
print(json.dumps({"lib": os.path.basename(mv.library_path), "B": B,
                  "lattice_ms": t_ms(lambda: mv.refine_matches_variant(mv.LATTICE, D11, D21, p1, 3, 5)),
                  "product_ms": t_ms(lambda: mb.refine_matches(D11, D21, p1, 3, 5)),
                  "equal": bool(torch.equal(lat, ref)), "rescored": resc / max(tot, 1), "mfma": mv.mfma_issued()}))
