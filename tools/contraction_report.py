"""How much the FMA-contraction convention moves the matching results.

The reference extension is built by nvcc -O3 (setup.py:29-37: --fmad=true), so the float
arithmetic of iter_proj (matching_kernels.cu:172-256) is FMA-contracted; rounds 1-2 pinned
contraction OFF.  This runs the CPU oracle's whole matching pipeline (the reference glue's host
arithmetic, iter_proj, p.long(), occlusion test, fp16 refine, u + W v) under each convention on
the bench's synthetic 512x384 pairs (B = 8, identity and warm start) and counts, between every two
conventions, the differing
  * iter_proj p_new floats (of 2 B H W),
  * truncated pre-refine pixels p.long() (of B H W),
  * final match indices and valid flags (of B H W).
The oracle is test infrastructure; this tool is a measurement, not part of the product.

usage: python tools/contraction_report.py [--out profiles/r03_contraction_matching.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_contraction_matching.json"))
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--H", type=int, default=384)
    ap.add_argument("--W", type=int, default=512)
    args = ap.parse_args()

    from m3s import synth
    from m3s.config import config as cfg0
    from oracle import oracle as O

    c = cfg0["matching"]
    mp = synth.make_match_pair(B=args.B, H=args.H, W=args.W, seed=11)  # bench.py's matching pairs
    X11, X21, D11, D21 = (t.numpy() for t in (mp.X11, mp.X21, mp.D11, mp.D21))
    n = args.B * args.H * args.W
    report = {"shape": [args.B, args.H, args.W], "pixels": n, "seed": 11,
              "conventions": list(O.CONTRACT), "starts": {}}
    for start, init in (("identity", None), ("warm", mp.idx_init.numpy())):
        res = {}
        t0 = time.time()
        for cm in O.CONTRACT:
            idx, valid, p_new, p_pre = O.match_iterative_proj(
                X11, X21, D11, D21, init, c["max_iter"], c["lambda_init"], c["convergence_thresh"],
                c["dist_thresh"], c["radius"], c["dilation_max"], contract=cm, return_pre=True)
            res[cm] = (idx, valid, p_new, p_pre)
        pairs = {}
        for a, b in itertools.combinations(O.CONTRACT, 2):
            ia, va, pa, la = res[a]
            ib, vb, pb, lb = res[b]
            dp = np.abs(pa.astype(np.float64) - pb.astype(np.float64))
            pairs[f"{a}_vs_{b}"] = {
                "p_new_floats_differ": int((pa.view(np.uint32) != pb.view(np.uint32)).sum()),
                "p_new_max_abs_diff_px": float(dp.max()),
                "p_long_pixels_differ": int((la != lb).any(-1).sum()),
                "final_idx_differ": int((ia != ib).sum()),
                "valid_differ": int((va != vb).sum()),
            }
        report["starts"][start] = pairs
        print(start, f"{time.time() - t0:.1f} s", json.dumps(pairs, indent=1), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(report, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
