"""How much the FMA-contraction convention moves the GN results.

The reference's align kernels are built by nvcc -O3 (setup.py:29-37: --fmad=true), so
`hij[l] += w*Jx[n]*Jx[m]` (gn_kernels.cu:616/1005/1081/1437-1487) is one fma per term and the
residual / Sim3 arithmetic is contracted too; rounds 1-2 pinned contraction OFF.  This runs the
CPU oracle (the reference backend restated, test infrastructure) on the bench graphs -- cfg3
(gauss_newton_calib, 256 pair edges) and cfg4 (gauss_newton_rays, 1024 pair edges) at 512x384 --
under each convention and reports, between every two conventions,
  * the per-edge Hs / gs of one accumulate pass (the reference kernels' output tensors): max
    difference in ulps of each 7x7 block's largest entry, and the fraction of entries that differ;
  * the poses after 1 and after 10 iterations: max relative difference;
and, for scale, each convention's distance from the same float terms summed in double.

usage: python tools/contraction_report_gn.py [--configs cfg3,cfg4] [--out ...]
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

LOCAL = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0, Q_conf=1.5,
             pixel_border=-10, depth_eps=1e-6)


def _ulp(a, b, axes):
    scale = np.maximum(np.abs(b).max(axis=axes, keepdims=True), np.float32(1e-30)).astype(np.float32)
    return float((np.abs(a.astype(np.float64) - b) / np.spacing(scale)).max())


def _rel(a, b):
    return float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg3,cfg4")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_contraction_gn.json"))
    args = ap.parse_args()

    from m3s import synth
    from m3s.geometry import constrain_points_to_ray
    from oracle import oracle as O

    report = {"conventions": list(O.CONTRACT), "configs": {}}
    for cfg in args.configs.split(","):
        spec = synth.CONFIGS[cfg]
        mode = spec["mode"]
        g = synth.make_graph(cfg)
        if mode == "calib":
            g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
        arrs = [t.numpy() for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]

        def params(n):
            if mode == "calib":
                return O.make_params("calib", LOCAL["sigma_pixel"], LOCAL["sigma_depth"], LOCAL["C_conf"],
                                     LOCAL["Q_conf"], K=g.K.numpy(), height=g.H, width=g.W,
                                     pixel_border=LOCAL["pixel_border"], z_eps=LOCAL["depth_eps"],
                                     max_iter=n, delta_thresh=0.0)
            return O.make_params("rays", LOCAL["sigma_ray"], LOCAL["sigma_dist"], LOCAL["C_conf"], LOCAL["Q_conf"],
                                 max_iter=n, delta_thresh=0.0)

        ie, je, _ = O.remap(arrs[3], arrs[4])
        res = {}
        t0 = time.time()
        for cm in O.CONTRACT:
            with O.contract(cm):
                Hs, gs = O.gn_align(params(1), arrs[0], arrs[1], arrs[2], ie, je, arrs[5], arrs[6], arrs[7])
                T1, _, _ = O.gauss_newton(params(1), *arrs)
                TN, _, _ = O.gauss_newton(params(args.iters), *arrs)
                with O.exact_sums():
                    T1x, _, _ = O.gauss_newton(params(1), *arrs)
            res[cm] = (Hs, gs, T1, TN, T1x)
            print(cfg, cm, f"{time.time() - t0:.0f} s", flush=True)
        pairs = {}
        for a, b in itertools.combinations(O.CONTRACT, 2):
            Ha, ga, T1a, TNa, _ = res[a]
            Hb, gb, T1b, TNb, _ = res[b]
            pairs[f"{a}_vs_{b}"] = {
                "Hs_max_ulp_of_block_max": _ulp(Ha, Hb, (-2, -1)),
                "Hs_entries_differ_frac": float((Ha != Hb).mean()),
                "gs_max_ulp_of_vector_max": _ulp(ga, gb, (-1,)),
                "poses_1iter_max_rel": _rel(T1a, T1b),
                f"poses_{args.iters}iter_max_rel": _rel(TNa, TNb),
            }
        report["configs"][cfg] = {
            "mode": mode, "edges": spec["E"], "keyframes": spec["N"], "iters": args.iters, "pairs": pairs,
            "poses_1iter_max_rel_vs_exact_sums": {cm: _rel(res[cm][2], res[cm][4]) for cm in O.CONTRACT},
        }
        print(cfg, json.dumps(report["configs"][cfg], indent=1), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(report, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
