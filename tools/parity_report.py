#!/usr/bin/env python
"""Parity report of the GN op on the headline graph (cfg3, calib) -- DESIGN.md §2.

Prints one JSON object:
  * oracle self-check: the reference's float order vs the same float terms summed exactly
    (1 and 10 iterations);
  * the fast path (default) vs the oracle after 1 and 10 iterations (and vs the exact sums);
  * the reference-order path (M3S_GN_ORDER_REFERENCE) vs the oracle: per-edge Hs / gs in ulp,
    poses after 1 and 10 iterations;
  * the cost in accuracy of each formula deviation the fast path used / uses, measured by
    substituting it into the reference-order path (env M3S_GN_REF_VARIANT bits), where the
    reference's own rounding is reproduced and any formula change shows up undiluted;
  * wall time of one 10-iteration call in both orders.
Test infrastructure (loads the oracle); run on the GPU box: python tools/parity_report.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402
from m3s.debug import edge_hessians_gpu  # noqa: E402
from m3s.geometry import constrain_points_to_ray  # noqa: E402
from oracle import oracle as O  # noqa: E402

L = dict(sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)


def rel(a, b):
    return float(np.abs(a - b).max() / np.abs(b).max())


def main():
    g = synth.make_graph("cfg3")
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    dev = torch.device("cuda", 0)
    G = {k: getattr(g, k).to(dev) for k in ("Xs", "Cs", "K", "ii", "jj", "idx", "valid", "Q")}

    def gpu(iters, order="fast", variant=0):
        os.environ["M3S_GN_REF_VARIANT"] = str(variant)
        prev = mb.set_gn_order(order)
        T = g.Twc.clone().to(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mb.gauss_newton_calib(T, G["Xs"], G["Cs"], G["K"], G["ii"], G["jj"], G["idx"], G["valid"], G["Q"],
                              g.H, g.W, L["pixel_border"], L["depth_eps"], L["sigma_pixel"],
                              L["sigma_depth"], L["C_conf"], L["Q_conf"], iters, 0.0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        mb.set_gn_order(prev)
        os.environ["M3S_GN_REF_VARIANT"] = "0"
        return T.cpu().numpy(), dt

    arrs = [t.numpy() for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]

    def oracle(iters, exact=False):
        P = O.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"],
                          K=g.K.numpy(), height=g.H, width=g.W, pixel_border=L["pixel_border"],
                          z_eps=L["depth_eps"], max_iter=iters, delta_thresh=0.0)
        if exact:
            with O.exact_sums():
                return O.gauss_newton(P, *arrs)[0]
        return O.gauss_newton(P, *arrs)[0]

    out = {"graph": "cfg3 calib: 128 keyframes, 512 directed edges, 384x512", "metric": "max|a-b| / max|b| over Twc"}
    To1, Tx1 = oracle(1), oracle(1, True)
    To10, Tx10 = oracle(10), oracle(10, True)
    out["oracle_reference_order_vs_exact_sums"] = {"1iter": rel(To1, Tx1), "10iter": rel(To10, Tx10)}
    for _ in range(2):  # warm-up (first-call planning, module load)
        gpu(10)
        gpu(10, "reference")
    Tf1, _ = gpu(1)
    Tf10, tf = gpu(10)
    Tr1, _ = gpu(1, "reference")
    Tr10, tr = gpu(10, "reference")
    out["fast_vs_oracle"] = {"1iter": rel(Tf1, To1), "10iter": rel(Tf10, To10),
                             "1iter_vs_exact_sums": rel(Tf1, Tx1), "10iter_vs_exact_sums": rel(Tf10, Tx10)}
    out["reference_order_vs_oracle"] = {"1iter": rel(Tr1, To1), "10iter": rel(Tr10, To10)}

    # the reference kernels' outputs themselves
    prev = mb.set_gn_order("reference")
    Hs_g, gs_g = edge_hessians_gpu(g, "calib", L | {"sigma_ray": 0, "sigma_dist": 0, "sigma_point": 0})
    mb.set_gn_order(prev)
    ie, je, _ = O.remap(arrs[3], arrs[4])
    P1 = O.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], K=g.K.numpy(),
                       height=g.H, width=g.W, pixel_border=L["pixel_border"], z_eps=L["depth_eps"], max_iter=1)
    Hs_o, gs_o = O.gn_align(P1, arrs[0], arrs[1], arrs[2], ie, je, arrs[5], arrs[6], arrs[7])
    sc = np.abs(Hs_o).max(axis=(-2, -1), keepdims=True).astype(np.float32)
    gsc = np.abs(gs_o).max(axis=-1, keepdims=True).astype(np.float32)
    out["reference_order_edge_hessians_vs_oracle"] = {
        "Hs_max_err_ulp_of_block_max": float((np.abs(Hs_g.astype(np.float64) - Hs_o) / np.spacing(sc)).max()),
        "gs_max_err_ulp_of_vector_max": float((np.abs(gs_g.astype(np.float64) - gs_o) / np.spacing(gsc)).max()),
        "Hs_bitwise_equal_fraction": float((Hs_g == Hs_o).mean()),
        "gs_bitwise_equal_fraction": float((gs_g == gs_o).mean()),
    }
    names = {1: "log_ratio (ln2*log2(zj*rcp(zi)))", 2: "v_rcp_f32 for 1/x", 4: "huber min(1, 1.345*rcp|r|)",
             7: "all three"}
    out["formula_deviation_cost_under_reference_order_1iter"] = {
        names[v]: rel(gpu(1, "reference", v)[0], To1) for v in (1, 2, 4, 7)}
    out["call_ms_10iter"] = {"fast": tf * 1e3, "reference_order": tr * 1e3}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
