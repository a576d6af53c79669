"""Generate the GN residual-model golden fixtures from the REFERENCE Python (dev container only).

Run from the repo root:  python tests/golden/make_residual_golden.py
Writes tests/golden/residual_golden.npz (inputs + reference outputs, small shapes).

The backend's align kernels (gn_kernels.cu:813-1138 rays, :1231-1543 calib) evaluate, per
directed point-edge, the same residual model the reference's Python front end states in
torch: the ray + distance residual ``point_to_ray_dist`` and the pixel + log-depth projection
``project_calib`` (geometry.py:17-34, 60-104), each whitened by sqrt(q)/sigma and re-weighted
with ``huber`` (nonlinear_optimizer.py:28-33).  This script evaluates THOSE reference
functions, run as written in float32 torch on CPU, on the oracle's per-point inputs after the
relative pose is applied (X_j in frame i = T_ij X_j, from oracle.gn_residuals, so the Sim3
group math is the oracle's own; it is pinned separately by the KATs), and stores:

  * rays : err = point_to_ray_dist(T_ij X_j) - point_to_ray_dist(X_i)                (4)
  * calib: err = project_calib(T_ij X_j)[u, v, log z] - (u_target, v_target, log z_i) (3)
           valid = project_calib's valid & z_i > z_eps & the match / Q / C tests
  * w    = huber(sqrt_w * err) * sqrt_w^2,  sqrt_w = (1/sigma) sqrt(q) on valid points

tests/test_oracle_kat.py::test_oracle_residuals_match_reference_python compares the oracle's
kernel restatement with them (validity exactly; values to a few ulps of the operands -- the
kernels and the torch front end round differently, e.g. fx*(x/z)+cx vs (fx*x+cx*z)/z).

The reference is read from /root/reference at generation time only; nothing under tests/
imports it at run time, and no reference source is copied.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

from oracle import oracle as O  # noqa: E402

LOCAL = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0,
             Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)  # base.yaml:35-50


def install_stubs():
    lt = types.ModuleType("lietorch")

    class Sim3:  # only a type annotation on this path (geometry.act_Sim3)
        pass

    lt.Sim3 = Sim3
    sys.modules["lietorch"] = lt
    sys.path.insert(0, REF)


def main():
    install_stubs()
    from mast3r_slam import geometry as rgeo
    from mast3r_slam import nonlinear_optimizer as rnl

    from m3s import synth
    from m3s.geometry import constrain_points_to_ray

    out = {}
    for mode in ("rays", "calib"):
        g = synth.make_graph(dict(N=4, E=4), H=16, W=24, seed=17)
        if mode == "calib":
            g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
        # edge cases: a low-Q span, unmatched points, a point behind the camera (calib z test)
        g.Q[0, :40] = 1.2
        g.valid[1, 100:160] = False
        g.Xs[2, 200:205, 2] = -0.5
        L = LOCAL
        if mode == "rays":
            P = O.make_params("rays", L["sigma_ray"], L["sigma_dist"], L["C_conf"], L["Q_conf"])
        else:
            P = O.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"],
                              K=g.K.numpy(), height=g.H, width=g.W, pixel_border=L["pixel_border"],
                              z_eps=L["depth_eps"])
        ie, je, _ = O.remap(g.ii.numpy(), g.jj.numpy())
        Xjc, err_o, w_o, valid_o = O.gn_residuals(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), ie,
                                                  je, g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
        E, HW = g.idx.shape
        vm = g.valid[..., 0]
        ind = torch.where(vm, g.idx, torch.zeros_like(g.idx))
        Xi = torch.stack([g.Xs[int(ie[e])][ind[e]] for e in range(E)])            # [E,HW,3]
        ci = torch.stack([g.Cs[int(ie[e]), :, 0][ind[e]] for e in range(E)])       # [E,HW]
        cj = torch.stack([g.Cs[int(je[e]), :, 0] for e in range(E)])               # [E,HW]
        q = g.Q[..., 0]
        X = torch.from_numpy(Xjc)
        base_valid = vm & (q > L["Q_conf"]) & (ci > L["C_conf"]) & (cj > L["C_conf"])
        if mode == "rays":
            a, b = rgeo.point_to_ray_dist(X), rgeo.point_to_ray_dist(Xi)          # geometry.py:17-34
            err = a - b
            valid = base_valid
            s_inv = torch.tensor([1.0 / L["sigma_ray"]] * 3 + [1.0 / L["sigma_dist"]], dtype=torch.float32)
        else:
            pz, valid_p = rgeo.project_calib(X, g.K, (g.H, g.W), border=L["pixel_border"],
                                             z_eps=L["depth_eps"])                 # geometry.py:60-104
            target = torch.stack(((ind % g.W).float(), (ind // g.W).float(), torch.log(Xi[..., 2])), -1)
            a, b = pz, target
            err = a - b
            valid = base_valid & valid_p[..., 0] & (Xi[..., 2] > L["depth_eps"])
            s_inv = torch.tensor([1.0 / L["sigma_pixel"]] * 2 + [1.0 / L["sigma_depth"]], dtype=torch.float32)
        sqrt_w = torch.where(valid[..., None], s_inv * torch.sqrt(q)[..., None], torch.zeros(()))
        w = rnl.huber(sqrt_w * err) * sqrt_w * sqrt_w                              # nonlinear_optimizer.py:28-33
        R = err.shape[-1]
        # the same weight formula on the ORACLE's residuals: pins the weighting on identical
        # inputs (the residuals themselves differ by the two formulations' cancellation)
        err_o_t = torch.from_numpy(np.ascontiguousarray(err_o[..., :R]))
        w_on_o = rnl.huber(sqrt_w * err_o_t) * sqrt_w * sqrt_w
        out.update({
            f"{mode}_Twc": g.Twc.numpy(), f"{mode}_Xs": g.Xs.numpy(), f"{mode}_Cs": g.Cs.numpy(),
            f"{mode}_ii": g.ii.numpy(), f"{mode}_jj": g.jj.numpy(), f"{mode}_idx": g.idx.numpy(),
            f"{mode}_valid": g.valid.numpy(), f"{mode}_Q": g.Q.numpy(), f"{mode}_K": g.K.numpy(),
            f"{mode}_hw": np.array([g.H, g.W]),
            f"{mode}_Xj_Ci": Xjc,                        # the input the reference functions saw
            f"{mode}_err_ref": err.numpy().astype(np.float32),
            # magnitude of the two terms the reference subtracts (the cancellation scale)
            f"{mode}_err_scale": torch.maximum(a.abs(), b.abs()).numpy().astype(np.float32),
            f"{mode}_w_ref_on_oracle_err": w_on_o.numpy().astype(np.float32),
            f"{mode}_w_ref": w.numpy().astype(np.float32),
            f"{mode}_validity_ref": valid.numpy(),
            f"{mode}_rows": np.array(R),
        })
        # a report of the agreement at generation time (the test re-checks it)
        ok = valid.numpy()
        d_err = np.abs(err.numpy() - err_o[..., :R])[ok].max()
        d_w = np.abs(w.numpy() - w_o[..., :R])[ok].max()
        print(f"{mode}: {int(ok.sum())} valid of {ok.size}; validity equal: "
              f"{np.array_equal(ok, valid_o)}; max |err diff| {d_err:.3g}, max |w diff| {d_w:.3g}")
    path = os.path.join(HERE, "residual_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    main()
