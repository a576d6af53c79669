"""Keyframe point-map fusion (keyframe.hip via mast3r_slam_backends.pointmap_update and
m3s.frame.Frame.update_pointmap) against the reference's torch expressions
(frame.py:41-105): bit-exact for the per-point arithmetic on identical inputs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(HW=384 * 512, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn((HW, 3), generator=g)
    C = 1.0 + torch.rand((HW, 1), generator=g) * 5
    Xn = torch.randn((HW, 3), generator=g)
    Cn = 1.0 + torch.rand((HW, 1), generator=g) * 5
    return [t.to(DEV) for t in (X, C, Xn, Cn)]


def _T(seed=1):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(4, generator=g)
    q = q / q.norm()
    return torch.cat([torch.randn(3, generator=g) * 0.3, q, torch.tensor([1.1])]).to(DEV)


def _act(T, p):
    t, q, s = T[0:3], T[3:7], T[7]
    u, w = q[:3].expand_as(p), q[3]
    uv = 2.0 * torch.cross(u, p, dim=-1)
    return s * (p + w * uv + torch.cross(u, uv, dim=-1)) + t


def test_weighted_pointmap_bit_exact(backend):
    X, C, Xn, Cn = _inputs()
    ref_X = ((C * X) + (Cn * Xn)) / (C + Cn)  # frame.py:75
    ref_C = C + Cn  # frame.py:76
    backend.pointmap_update("weighted_pointmap", X, C, Xn, Cn)
    assert torch.equal(X, ref_X) and torch.equal(C, ref_C)


def test_indep_conf_and_recent_bit_exact(backend):
    X, C, Xn, Cn = _inputs(seed=3)
    m = Cn > C  # frame.py:70-72
    ref_X, ref_C = X.clone(), C.clone()
    ref_X[m.repeat(1, 3)] = Xn[m.repeat(1, 3)]
    ref_C[m] = Cn[m]
    backend.pointmap_update("indep_conf", X, C, Xn, Cn)
    assert torch.equal(X, ref_X) and torch.equal(C, ref_C)
    backend.pointmap_update("recent", X, C, Xn, Cn)
    assert torch.equal(X, Xn) and torch.equal(C, Cn)


def test_fused_transform(backend):
    X, C, Xn, Cn = _inputs(HW=4096, seed=5)
    T = _T()
    Xt = _act(T, Xn)
    ref_X = ((C * X) + (Cn * Xt)) / (C + Cn)
    X2, C2 = X.clone(), C.clone()
    backend.pointmap_update("weighted_pointmap", X2, C2, Xn, Cn, T)
    torch.testing.assert_close(X2, ref_X, rtol=0, atol=2e-6)
    # with the op's own transform the fusion is exact
    Xo = torch.empty_like(Xn)
    Co = torch.zeros_like(Cn)
    backend.pointmap_update("recent", Xo, Co, Xn, Cn, T)
    torch.testing.assert_close(Xo, Xt, rtol=0, atol=2e-6)
    assert torch.equal(X2, ((C * X) + (Cn * Xo)) / (C + Cn))


def test_frame_update_pointmap_modes():
    from m3s.config import config
    from m3s.frame import Frame

    X, C, Xn, Cn = _inputs(HW=2048, seed=7)
    cfg = {"tracking": dict(config["tracking"], filtering_mode="weighted_pointmap")}
    f = Frame(cfg=cfg)
    f.update_pointmap(X, C)
    assert f.N == 1 and torch.equal(f.X_canon, X)
    f.update_pointmap(Xn, Cn)
    assert f.N == 2 and f.N_updates == 2
    assert torch.equal(f.X_canon, ((C * X) + (Cn * Xn)) / (C + Cn))
    assert torch.equal(f.get_average_conf(), (C + Cn) / 2)
    cfg["tracking"]["filtering_mode"] = "best_score"
    g = Frame(cfg=cfg)
    g.update_pointmap(X, C)
    g.update_pointmap(Xn, Cn)
    better = torch.median(Cn) > torch.median(C)
    assert torch.equal(g.X_canon, Xn if better else X)
