"""Caller-side glue against fixtures produced by the
REFERENCE Python itself (tests/golden/make_golden.py, committed glue_golden.npz).

Runs on CPU: the product kernels are not involved here; the matching glue is driven
through a capture backend whose ops are the CPU oracle (test infrastructure), exactly as
the fixture generator drove the reference glue.
"""
import os
import types

import numpy as np
import pytest
import torch

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "glue_golden.npz"))


def T(k):
    return torch.from_numpy(GOLD[k])


def test_img_gradient_matches_reference():
    from m3s.image import img_gradient

    gx, gy = img_gradient(T("grad_in"))
    # same conv2d on the same device as the fixture generator: bitwise
    np.testing.assert_array_equal(gx.numpy(), GOLD["grad_gx"])
    np.testing.assert_array_equal(gy.numpy(), GOLD["grad_gy"])


def test_prep_for_iter_proj_matches_reference():
    from m3s.matching import prep_for_iter_proj

    rays, pts, p_init = prep_for_iter_proj(T("X11"), T("X21"), None)
    assert rays.shape == GOLD["prep_rays"].shape and rays.is_contiguous()
    np.testing.assert_array_equal(rays.numpy(), GOLD["prep_rays"])
    assert np.array_equal(pts.numpy(), GOLD["prep_pts"])
    assert np.array_equal(p_init.numpy(), GOLD["prep_pinit"]) and p_init.dtype == torch.float32
    _, _, p_w = prep_for_iter_proj(T("X11"), T("X21"), T("idx_init"))
    assert np.array_equal(p_w.numpy(), GOLD["prep_pinit_warm"])


def _oracle_backend(oracle):
    m = types.SimpleNamespace()

    def iter_proj(rays, pts, p_init, max_iter, lam, thr):
        p, c = oracle.iter_proj(rays.numpy(), pts.numpy(), p_init.numpy(), max_iter, lam, thr)
        return [torch.from_numpy(p), torch.from_numpy(c)]

    def refine_matches(D11, D21, p1, radius, dmax):
        m.refine_p1 = p1.clone()
        return [torch.from_numpy(oracle.refine_matches(D11.numpy(), D21.numpy(), p1.numpy(), radius, dmax))]

    m.iter_proj, m.refine_matches = iter_proj, refine_matches
    return m


@pytest.mark.parametrize("tag", ["id", "warm"])
def test_match_iterative_proj_glue_matches_reference(oracle, monkeypatch, tag):
    import m3s.matching as mm

    be = _oracle_backend(oracle)
    monkeypatch.setattr(mm, "mast3r_slam_backends", be)
    init = None if tag == "id" else T("idx_init")
    idx, valid = mm.match_iterative_proj(T("X11"), T("X21"), T("D11"), T("D21"), init)
    assert idx.dtype == torch.int64 and valid.dtype == torch.bool and valid.shape[-1] == 1
    # the pre-refine pixels reaching refine_matches (p.long() truncation) and the outputs:
    # identical inputs on the same device as the fixture generator => identical indices
    assert np.array_equal(be.refine_p1.numpy(), GOLD[f"match_{tag}_p1_pre"])
    assert np.array_equal(idx.numpy(), GOLD[f"match_{tag}_idx"])
    assert np.array_equal(valid.numpy(), GOLD[f"match_{tag}_valid"])


def test_constrain_points_to_ray_matches_reference():
    from m3s.geometry import constrain_points_to_ray

    out = constrain_points_to_ray((12, 16), T("cpr_Xs"), T("cpr_K"))
    assert np.array_equal(out.numpy(), GOLD["cpr_out"])


@pytest.mark.parametrize("name", ["rays", "calib"])
def test_factor_graph_hands_the_op_the_reference_arguments(name):
    """FactorGraph.solve_GN_* must pass the op exactly what the reference's does
    (global_opt.py:121-213): same positional tuple, dtypes, shapes, values, and the same
    update_T_WCs write-back."""
    from m3s.global_opt import FactorGraph, KeyframeStore

    kf_ids = GOLD["fg_kf_ids"].tolist()
    h, w = GOLD["fg_graph_hw"].tolist()
    store = KeyframeStore(10, h, w, device="cpu")
    store.size = 10
    Xs, Tw, Cs = T("fg_graph_Xs"), T("fg_graph_Twc"), T("fg_graph_Cs")
    for r, k in enumerate(kf_ids):
        store.X[k], store.T_WC[k, 0], store.C[k] = Xs[r], Tw[r], 2.0 * Cs[r]
    store.n_obs[:] = 2.0
    ii, jj = T("fg_graph_ii"), T("fg_graph_jj")
    E = ii.shape[0] // 2
    to_g = torch.tensor(kf_ids)
    K = T("fg_graph_K") if name == "calib" else None
    fg = FactorGraph(None, store, K=K, device="cpu")
    fg.ii, fg.jj = to_g[ii[:E]], to_g[jj[:E]]
    idx, valid, Q = T("fg_graph_idx"), T("fg_graph_valid"), T("fg_graph_Q")
    fg.idx_ii2jj, fg.idx_jj2ii = idx[:E], idx[E:]
    fg.valid_match_j, fg.valid_match_i = valid[:E], valid[E:]
    fg.Q_ii2jj, fg.Q_jj2ii = Q[:E], Q[E:]

    got = {}
    cap = types.SimpleNamespace()
    cap.gauss_newton_rays = lambda *a: got.setdefault("args", a) and [None]
    cap.gauss_newton_calib = lambda *a: got.setdefault("args", a) and [None]
    (fg.solve_GN_rays if name == "rays" else fg.solve_GN_calib)(backend=cap)
    args = got["args"]
    assert len(args) == int(GOLD[f"fg_{name}_nargs"])
    for k, a in enumerate(args):
        ref = GOLD[f"fg_{name}_arg{k}"]
        if isinstance(a, torch.Tensor):
            assert a.is_contiguous(), k
            assert a.dtype == torch.from_numpy(ref).dtype, (k, a.dtype, ref.dtype)
            assert tuple(a.shape) == ref.shape, (k, a.shape, ref.shape)
            assert np.array_equal(a.numpy(), ref), k
        else:
            assert type(a)(ref) == a and np.asarray(a).dtype.kind == ref.dtype.kind, (k, a, ref)
    # Twc is a view into the stacked pose tensor that is written back for ids[pin:]
    np.testing.assert_array_equal(store.T_WC[torch.tensor(kf_ids[1:])].numpy(), GOLD[f"fg_{name}_upd_T"])
    assert GOLD[f"fg_{name}_upd_idx"].tolist() == kf_ids[1:]


def test_oracle_match_glue_restatement_matches_reference(oracle):
    """The oracle's C restatement of the matching glue (oracle_match_prep / _post: the reference's
    host arithmetic -- fma-chain normalize, row-major fma conv taps, Python floor // and %) is
    bitwise the reference's prep_for_iter_proj output, and its whole pipeline (with the oracle's
    kernels) reproduces the reference's match_iterative_proj indices and flags.  This pins the
    checker of the fused HIP pipeline (test_gpu_matching.py)."""
    from m3s.config import config as cfg0

    rays, pts, p_init = oracle.match_prep(GOLD["X11"], GOLD["X21"], None)
    np.testing.assert_array_equal(rays, GOLD["prep_rays"])
    np.testing.assert_array_equal(pts, GOLD["prep_pts"])
    np.testing.assert_array_equal(p_init, GOLD["prep_pinit"])
    _, _, p_w = oracle.match_prep(GOLD["X11"], GOLD["X21"], GOLD["idx_init"])
    np.testing.assert_array_equal(p_w, GOLD["prep_pinit_warm"])
    c = cfg0["matching"]
    for tag, init in (("id", None), ("warm", GOLD["idx_init"])):
        idx, valid = oracle.match_iterative_proj(GOLD["X11"], GOLD["X21"], GOLD["D11"], GOLD["D21"], init,
                                                 c["max_iter"], c["lambda_init"], c["convergence_thresh"],
                                                 c["dist_thresh"], c["radius"], c["dilation_max"])
        np.testing.assert_array_equal(idx, GOLD[f"match_{tag}_idx"])
        np.testing.assert_array_equal(valid, GOLD[f"match_{tag}_valid"])
