"""GN fast-path accuracy probe: the op's poses against the CPU oracle (the reference's fp32 order,
FMA-contracted) and against the same float terms summed in double ("exact"), on
  * cfg4 topology at 48x64, rays, 3 and 1 iterations (tests/test_gpu_dist.py's graph),
  * cfg4 at 512x384, rays, 1 iteration,
  * cfg3 at 512x384, calib (ray-constrained points), 1 iteration.
One-iteration cases also compare the step dx itself (poses after one step carry the float Sim(3)
exponential's amplification of the log-scale step).
Run once per library build (M3S_BACKEND_LIB selects a variant); prints one JSON line.
Measurement tool (loads the oracle as the checker); not part of the product.

usage: M3S_BACKEND_LIB=... python tools/accuracy_probe.py [--tag name]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

L = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0, Q_conf=1.5,
         pixel_border=-10, depth_eps=1e-6)


def rel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / np.abs(b).max())


def system_split(name, g, mode, P, cache_dir, dx_op, dx_oracle):
    """Where the first step's error comes from: the op's normal equations (H, b) against the
    oracle's (reference order) and the exactly summed ones, entry-wise (relative to the largest
    entry), and the step dx solved from each mix of H and b -- whether H's or b's rounding moves
    the update."""
    from m3s.debug import build_system_gpu
    from oracle import oracle as O

    H_g, b_g = build_system_gpu(g, mode, L)
    cache = os.path.join(cache_dir, f"m3s_accprobe_sys_{name}.npz")
    arrs = [t.numpy() for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]
    if os.path.exists(cache):
        z = np.load(cache)
        H_o, b_o, H_x, b_x = z["H_o"], z["b_o"], z["H_x"], z["b_x"]
    else:
        H_o, b_o = O.gn_build_system(P, *arrs)
        with O.exact_sums():
            H_x, b_x = O.gn_build_system(P, *arrs)
        np.savez(cache, H_o=H_o, b_o=b_o, H_x=H_x, b_x=b_x)
    ent = lambda A, B: float(np.abs(A - B).max() / np.abs(B).max())
    dx = lambda H, b: -np.linalg.solve(H, b)  # dx = -A.solve() (the reference's sign)
    d_x = dx(H_x, b_x)
    rd = lambda d: float(np.abs(d - d_x).max() / np.abs(d_x).max())
    return {"H_vs_exact": ent(H_g, H_x), "b_vs_exact": ent(b_g, b_x),
            "H_oracle_vs_exact": ent(H_o, H_x), "b_oracle_vs_exact": ent(b_o, b_x),
            "dx_max_abs": float(np.abs(d_x).max()),
            "dx_rel": {"op_own_solve": rd(dx_op.reshape(-1)[:d_x.size]), "oracle_own_solve": rd(dx_oracle.reshape(-1)[:d_x.size]),
                       "gpu": rd(dx(H_g, b_g)), "oracle": rd(dx(H_o, b_o)),
                       "gpu_H_exact_b": rd(dx(H_g, b_x)), "exact_H_gpu_b": rd(dx(H_x, b_g)),
                       "oracle_H_exact_b": rd(dx(H_o, b_x)), "exact_H_oracle_b": rd(dx(H_x, b_o))},
            "cond_H": float(np.linalg.cond(H_x))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("M3S_BACKEND_LIB", "default")))
    ap.add_argument("--cache", default="/tmp", help="directory for the oracle's poses (shared across variants)")
    ap.add_argument("--system", action="store_true", help="also split the first step's error (H vs b)")
    ap.add_argument("--dump", default=None, help="directory for the poses / steps (npz per graph)")
    args = ap.parse_args()
    import mast3r_slam_backends as mb
    from m3s import synth
    from m3s.geometry import constrain_points_to_ray
    from oracle import oracle as O

    out = {"tag": args.tag}
    for name, cfg, H, W, seed, mode, iters in (("cfg4_48x64_3it", "cfg4", 48, 64, 7, "rays", 3),
                                               ("cfg4_48x64_1it", "cfg4", 48, 64, 7, "rays", 1),
                                               ("cfg4_full_1it", "cfg4", 384, 512, None, "rays", 1),
                                               ("cfg3_full_1it", "cfg3", 384, 512, None, "calib", 1)):
        g = synth.make_graph(cfg, H=H, W=W, seed=seed)
        if mode == "calib":
            g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
        c = lambda t: t.cuda()
        Twc = c(g.Twc)
        if mode == "rays":
            (dx_op,) = mb.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                                 L["sigma_ray"], L["sigma_dist"], L["C_conf"], L["Q_conf"], iters, 0.0)
            P = O.make_params("rays", L["sigma_ray"], L["sigma_dist"], L["C_conf"], L["Q_conf"], max_iter=iters,
                              delta_thresh=0.0)
        else:
            (dx_op,) = mb.gauss_newton_calib(Twc, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                                  g.H, g.W, L["pixel_border"], L["depth_eps"], L["sigma_pixel"], L["sigma_depth"],
                                  L["C_conf"], L["Q_conf"], iters, 0.0)
            P = O.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], K=g.K.numpy(),
                              height=g.H, width=g.W, pixel_border=L["pixel_border"], z_eps=L["depth_eps"],
                              max_iter=iters, delta_thresh=0.0)
        torch.cuda.synchronize()
        T = Twc.cpu().numpy()
        cache = os.path.join(args.cache, f"m3s_accprobe_{name}.npz")
        if os.path.exists(cache):
            z = np.load(cache)
            T_o, T_x, dx_o, dx_x = z["T_o"], z["T_x"], z["dx_o"], z["dx_x"]
        else:
            arrs = [t.numpy() for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]
            T_o, dx_o, _ = O.gauss_newton(P, *arrs)
            with O.exact_sums():
                T_x, dx_x, _ = O.gauss_newton(P, *arrs)
            np.savez(cache, T_o=T_o, T_x=T_x, dx_o=dx_o, dx_x=dx_x)
        out[name] = {"vs_exact": rel(T, T_x), "vs_oracle": rel(T, T_o), "sigma_oracle_vs_exact": rel(T_o, T_x)}
        if iters == 1:  # the step itself (accumulate + solve), relative to max |dx|
            out[name]["step_vs_exact"] = rel(dx_op.cpu().numpy(), dx_x)
            out[name]["step_oracle_vs_exact"] = rel(dx_o, dx_x)
        if args.dump:
            np.savez(os.path.join(args.dump, f"accprobe_{args.tag}_{name}.npz"), T=T, dx_op=dx_op.cpu().numpy(),
                     T_o=T_o, T_x=T_x, dx_o=dx_o, T0=g.Twc.numpy())
        if iters == 1 and args.system:
            out[name]["system"] = system_split(name, g, mode, P, args.cache, dx_op.cpu().numpy(), dx_o)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
