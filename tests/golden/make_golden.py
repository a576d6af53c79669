"""Generate the glue-level golden fixtures from the REFERENCE Python (dev container only).

Run from the repo root:  python tests/golden/make_golden.py
Writes tests/golden/glue_golden.npz (inputs + reference outputs, small shapes).

What is pinned (reference file:line):
  * img_gradient                       mast3r_slam/image.py:5-38
  * prep_for_iter_proj                 mast3r_slam/matching.py:25-49
  * match_iterative_proj post-process  mast3r_slam/matching.py:52-90, driven through a
    stub `mast3r_slam_backends` whose iter_proj/refine_matches are the CPU ORACLE
    (so the fixture pins the reference glue: p.long(), occlusion test on the pre-refine
    pixels, .half() descriptors, u + W*v) -- once per FMA-contraction convention of the
    oracle's iter_proj: match_<start>_idx/valid under the reference build's (nvcc, the
    default), match_<start>_<conv>_idx/valid for every convention (off, nvcc, nvcc_right)
  * constrain_points_to_ray            mast3r_slam/geometry.py:37-42, 107-123
  * FactorGraph.solve_GN_rays / _calib  mast3r_slam/global_opt.py:104-213: the exact
    positional argument tuple handed to the op and the update_T_WCs write-back,
    captured with stub `lietorch` / frames / backend.

The reference is read from /root/reference at generation time only; nothing under
tests/ imports it at run time, and no reference source is copied.
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


# ---------------------------------------------------------------- stubs for absent deps
class _Sim3:
    """Minimal lietorch.Sim3 stand-in: only `.data` and indexing are used on the path."""

    def __init__(self, data):
        self.data = data

    def __getitem__(self, k):
        return _Sim3(self.data[k])

    @classmethod
    def Identity(cls, n, **kw):
        d = torch.zeros((n, 8))
        d[:, 6] = 1.0
        d[:, 7] = 1.0
        return cls(d)


captured = {}
_contract = ["nvcc"]  # the stub iter_proj's convention (oracle.CONTRACT)


def _stub_backend():
    m = types.ModuleType("mast3r_slam_backends")

    def iter_proj(rays, pts, p_init, max_iter, lam, thr):
        p, c = O.iter_proj(rays.numpy(), pts.numpy(), p_init.numpy(), max_iter, lam, thr,
                           contract=_contract[0])
        captured["iter_proj_in"] = (rays.clone(), pts.clone(), p_init.clone(), max_iter, lam, thr)
        return [torch.from_numpy(p), torch.from_numpy(c)]

    def refine_matches(D11, D21, p1, radius, dmax):
        captured["refine_in"] = (D11.clone(), D21.clone(), p1.clone(), radius, dmax)
        out = O.refine_matches(D11.numpy(), D21.numpy(), p1.numpy(), radius, dmax)
        return [torch.from_numpy(out)]

    def _gn(name):
        def f(*args):
            captured[name] = [a.clone() if isinstance(a, torch.Tensor) else a for a in args]
            return [None]

        return f

    m.iter_proj = iter_proj
    m.refine_matches = refine_matches
    m.gauss_newton_rays = _gn("gauss_newton_rays")
    m.gauss_newton_calib = _gn("gauss_newton_calib")
    m.gauss_newton_points = _gn("gauss_newton_points")
    return m


def install_stubs():
    lt = types.ModuleType("lietorch")
    lt.Sim3 = _Sim3
    sys.modules["lietorch"] = lt
    mu = types.ModuleType("mast3r_slam.mast3r_utils")
    mu.mast3r_match_symmetric = None
    mu.resize_img = None
    sys.modules["mast3r_slam.mast3r_utils"] = mu
    sys.modules["mast3r_slam_backends"] = _stub_backend()
    sys.path.insert(0, REF)


class _KF:
    def __init__(self, X, T, C, img):
        self.X_canon, self.T_WC, self.C, self.N, self.img = X, _Sim3(T), C, 2, img

    def get_average_conf(self):
        return self.C / self.N


class _Frames:
    def __init__(self, Xs, Ts, Cs, h, w):
        self.kfs = [_KF(Xs[k], Ts[k], Cs[k], torch.zeros(3, h, w)) for k in range(len(Xs))]

    def __getitem__(self, idx):
        return self.kfs[int(idx)]

    def update_T_WCs(self, T, idx):
        captured["update_T_WCs"] = (T.data.clone(), idx.clone())


def main():
    install_stubs()
    from mast3r_slam import config as rcfg  # reference config module
    from mast3r_slam import geometry as rgeo
    from mast3r_slam import global_opt as rgo
    from mast3r_slam import image as rimg
    from mast3r_slam import matching as rmatch

    rcfg.load_config(os.path.join(REF, "config", "base.yaml"))
    out = {}
    g = torch.Generator().manual_seed(1234)

    # img_gradient
    img = torch.randn((2, 3, 12, 16), generator=g)
    gx, gy = rimg.img_gradient(img)
    out.update(grad_in=img.numpy(), grad_gx=gx.numpy(), grad_gy=gy.numpy())

    # prep_for_iter_proj (identity and warm start)
    from m3s import synth

    mp = synth.make_match_pair(B=2, H=24, W=32, seed=5)
    rays, pts, p_init = rmatch.prep_for_iter_proj(mp.X11, mp.X21, None)
    out.update(X11=mp.X11.numpy(), X21=mp.X21.numpy(), D11=mp.D11.numpy(), D21=mp.D21.numpy(),
               idx_init=mp.idx_init.numpy(), prep_rays=rays.numpy(), prep_pts=pts.numpy(),
               prep_pinit=p_init.numpy())
    _, _, p_init_w = rmatch.prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
    out.update(prep_pinit_warm=p_init_w.numpy())

    # match_iterative_proj (reference glue + oracle kernels), per contraction convention
    for cm in O.CONTRACT:
        _contract[0] = cm
        for tag, init in (("id", None), ("warm", mp.idx_init)):
            idx, valid = rmatch.match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, init)
            out[f"match_{tag}_{cm}_idx"] = idx.numpy()
            out[f"match_{tag}_{cm}_valid"] = valid.numpy()
            out[f"match_{tag}_{cm}_p1_pre"] = captured["refine_in"][2].numpy()
            if cm == O.CONTRACT_DEFAULT:
                out[f"match_{tag}_idx"] = idx.numpy()
                out[f"match_{tag}_valid"] = valid.numpy()
                out[f"match_{tag}_p1_pre"] = captured["refine_in"][2].numpy()
    _contract[0] = O.CONTRACT_DEFAULT

    # constrain_points_to_ray
    Xs = torch.randn((3, 12 * 16, 3), generator=g).abs() + 0.5
    K = torch.tensor(synth.intrinsics(12, 16), dtype=torch.float32)
    out.update(cpr_Xs=Xs.numpy(), cpr_K=K.numpy(), cpr_out=rgeo.constrain_points_to_ray((12, 16), Xs, K).numpy())

    # FactorGraph.solve_GN_rays / solve_GN_calib argument capture
    gr = synth.make_graph(dict(N=4, E=4), H=12, W=16, seed=11)
    kf_ids = [3, 5, 8, 9]  # global keyframe ids (sparse, like a real run)
    Nk = 10
    Xall = torch.zeros((Nk, gr.HW, 3))
    Tall = torch.zeros((Nk, 1, 8))
    Call = torch.zeros((Nk, gr.HW, 1))
    for r, k in enumerate(kf_ids):
        Xall[k], Tall[k, 0], Call[k] = gr.Xs[r], gr.Twc[r], 2.0 * gr.Cs[r]
    frames = _Frames(Xall, Tall, Call, gr.H, gr.W)
    E = gr.ii.shape[0] // 2
    to_g = torch.tensor(kf_ids)
    for name, use_K in (("rays", None), ("calib", gr.K)):
        fg = rgo.FactorGraph(None, frames, K=use_K, device="cpu")
        fg.ii, fg.jj = to_g[gr.ii[:E]], to_g[gr.jj[:E]]
        fg.idx_ii2jj, fg.idx_jj2ii = gr.idx[:E], gr.idx[E:]
        fg.valid_match_j, fg.valid_match_i = gr.valid[:E], gr.valid[E:]
        fg.Q_ii2jj, fg.Q_jj2ii = gr.Q[:E], gr.Q[E:]
        (fg.solve_GN_rays if name == "rays" else fg.solve_GN_calib)()
        args = captured[f"gauss_newton_{name}"]
        for k, a in enumerate(args):
            out[f"fg_{name}_arg{k}"] = a.numpy() if isinstance(a, torch.Tensor) else np.array(a)
        out[f"fg_{name}_nargs"] = np.array(len(args))
        out[f"fg_{name}_upd_T"] = captured["update_T_WCs"][0].numpy()
        out[f"fg_{name}_upd_idx"] = captured["update_T_WCs"][1].numpy()
    out.update(fg_kf_ids=np.array(kf_ids), fg_graph_Xs=gr.Xs.numpy(), fg_graph_Twc=gr.Twc.numpy(),
               fg_graph_Cs=gr.Cs.numpy(), fg_graph_ii=gr.ii.numpy(), fg_graph_jj=gr.jj.numpy(),
               fg_graph_idx=gr.idx.numpy(), fg_graph_valid=gr.valid.numpy(), fg_graph_Q=gr.Q.numpy(),
               fg_graph_K=gr.K.numpy(), fg_graph_hw=np.array([gr.H, gr.W]))

    np.savez_compressed(os.path.join(HERE, "glue_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "glue_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
