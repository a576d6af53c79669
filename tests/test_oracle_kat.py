"""Known-answer tests that pin the CPU oracle itself.

The reference ships no golden vectors for its native ops, so the restatement is checked
against independent float64 mathematics:
  * Sim3 exp / retraction vs the exact integral form (scipy rotation, numeric quadrature);
  * the adjoint map vs its definition on the Lie algebra (finite differences);
  * every GN Jacobian row: H = J^T W J and g = J^T W r vs central finite differences of the
    residuals restated in float64 numpy;
  * noise-free graphs: GN converges to the generating poses;
  * iter_proj on an analytic ray field recovers the generating pixel;
  * refine_matches recovers planted descriptor peaks;
  * the dense LL^T solve vs numpy, and its failure semantics.
"""
import math

import numpy as np
import pytest
from scipy.spatial.transform import Rotation as Rot

from m3s import synth


def exp_sim3_exact(xi):
    tau, phi, sig = xi[:3], xi[3:6], xi[6]
    ts = np.linspace(0.0, 1.0, 4001)
    W = np.zeros((3, 3))
    for i, t in enumerate(ts):
        w = 0.5 if i in (0, len(ts) - 1) else 1.0
        W += w * math.exp(sig * t) * Rot.from_rotvec(phi * t).as_matrix()
    W /= len(ts) - 1
    return W @ tau, Rot.from_rotvec(phi).as_quat(), math.exp(sig)


def mat_of(pose):
    t, q, s = pose[:3].astype(np.float64), pose[3:7].astype(np.float64), float(pose[7])
    T = np.eye(4)
    T[:3, :3] = s * Rot.from_quat(q).as_matrix()
    T[:3, 3] = t
    return T


@pytest.mark.parametrize("scale", [1e-4, 0.05, 0.4])
def test_exp_sim3_matches_exact(oracle, scale):
    rng = np.random.default_rng(int(scale * 1e4))
    for _ in range(5):
        xi = (rng.standard_normal(7) * scale).astype(np.float32)
        t, q, s = oracle.exp_sim3(xi)
        te, qe, se = exp_sim3_exact(xi.astype(np.float64))
        if qe[3] < 0:
            qe = -qe
        assert np.abs(t - te).max() < 2e-6 + 1e-5 * np.abs(te).max()
        assert np.abs(q - qe).max() < 2e-6
        assert abs(s - se) < 2e-6 * se


def test_retraction_is_left_composition(oracle):
    rng = np.random.default_rng(1)
    pose = np.concatenate([rng.standard_normal(3), Rot.random(random_state=2).as_quat(), [1.3]]).astype(np.float32)
    xi = (rng.standard_normal(7) * 0.1).astype(np.float32)
    out = oracle.retr_sim3(xi, pose)
    te, qe, se = exp_sim3_exact(xi.astype(np.float64))
    D = np.eye(4)
    D[:3, :3] = se * Rot.from_quat(qe).as_matrix()
    D[:3, 3] = te
    np.testing.assert_allclose(mat_of(out), D @ mat_of(pose), atol=1e-5)


def test_adjoint_map_definition(oracle):
    """Y = X Adj(T)^{-1}: for a row vector X on the tangent at T_j's frame, the map the
    reference applies (gn_kernels.cu:277-297) equals X * d(T exp(d) T^-1 ...) -- checked by
    d/dxi [ log( T^{-1} exp(xi) T ) ] = Adj(T^{-1}) via finite differences of exp."""
    rng = np.random.default_rng(3)
    pose = np.concatenate([rng.standard_normal(3) * 0.5, Rot.random(random_state=4).as_quat(), [1.7]])
    Tm = mat_of(pose.astype(np.float32))

    def to_mat(xi):
        t, q, s = exp_sim3_exact(xi)
        M = np.eye(4)
        M[:3, :3] = s * Rot.from_quat(q).as_matrix()
        M[:3, 3] = t
        return M

    # Adj(T^{-1}) columns: T^{-1} exp(h e_k) T ~ exp(h * Adj(T^{-1}) e_k)
    h = 1e-5
    Ad = np.zeros((7, 7))
    Tinv = np.linalg.inv(Tm)
    for k in range(7):
        e = np.zeros(7)
        e[k] = h
        M = (Tinv @ to_mat(e) @ Tm - Tinv @ to_mat(-e) @ Tm) / (2 * h)
        # generator -> tangent (tau, phi, sigma)
        Ad[:3, k] = M[:3, 3]
        Ad[3:6, k] = [M[2, 1], M[0, 2], M[1, 0]]
        Ad[6, k] = np.trace(M[:3, :3]) / 3.0
    for _ in range(5):
        X = rng.standard_normal(7).astype(np.float32)
        Y = oracle.apply_sim3_adj_inv(pose.astype(np.float32), X)
        np.testing.assert_allclose(Y, X.astype(np.float64) @ Ad, rtol=1e-4, atol=1e-4)


# ------------------------------------------------------------------ Jacobians by FD


def residuals_f64(mode, Ti, Tj, Xi, Xj, K=None, W=None):
    """float64 restatement of the per-point residuals (gn_kernels.cu:924-947, 1360-1388, 564-570)."""
    Tij = np.linalg.inv(Ti) @ Tj
    P = Xj @ Tij[:3, :3].T + Tij[:3, 3]
    if mode == "rays":
        ni = np.linalg.norm(Xi, axis=1, keepdims=True)
        nj = np.linalg.norm(P, axis=1, keepdims=True)
        return np.concatenate([P / nj - Xi / ni, nj - ni], axis=1)
    if mode == "points":
        return P - Xi
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    u = fx * P[:, 0] / P[:, 2] + cx
    v = fy * P[:, 1] / P[:, 2] + cy
    return np.stack([u, v, np.log(P[:, 2]) - np.log(Xi[:, 2])], axis=1)


@pytest.mark.parametrize("mode", ["rays", "points", "calib"])
def test_hessian_is_JtWJ_by_finite_differences(oracle, mode):
    """One directed edge, all points valid, Huber inactive: the oracle's Hs/gs equal
    J^T W J and J^T W r with J from central differences of the float64 residuals w.r.t.
    left perturbations exp(d) T of the two poses."""
    rng = np.random.default_rng(7)
    HW = 64
    H_, W_ = 8, 8
    K = synth.intrinsics(H_, W_)
    Ti = np.concatenate([[0.0, 0.0, 0.0], [0, 0, 0, 1], [1.0]]).astype(np.float32)
    Tj = np.concatenate([[0.05, -0.02, 0.03], Rot.from_rotvec([0.02, -0.01, 0.03]).as_quat(), [1.05]]).astype(np.float32)
    Xj = np.stack([rng.uniform(-0.5, 0.5, HW), rng.uniform(-0.5, 0.5, HW), rng.uniform(2, 3, HW)], 1).astype(np.float32)
    Tij = np.linalg.inv(mat_of(Ti)) @ mat_of(Tj)
    P = Xj.astype(np.float64) @ Tij[:3, :3].T + Tij[:3, 3]
    Xi = (P + rng.normal(0, 1e-4, P.shape)).astype(np.float32)  # small residuals: Huber inactive
    if mode == "calib":
        Xi[:, 2] = P[:, 2] * np.exp(rng.normal(0, 1e-3, HW))
    Xs = np.stack([Xi, Xj]).astype(np.float32)  # row 0 = i, row 1 = j
    idx = np.arange(HW, dtype=np.int64)[None]
    valid = np.ones((1, HW, 1), np.uint8)
    Q = np.full((1, HW, 1), 2.0, np.float32)
    Cs = np.full((2, HW, 1), 2.0, np.float32)
    if mode == "calib":
        # the pixel target of point k is idx % W, idx / W: put the measured pixel there
        u = K[0, 0] * P[:, 0] / P[:, 2] + K[0, 2]
        v = K[1, 1] * P[:, 1] / P[:, 2] + K[1, 2]
        idx = (np.clip(np.round(v), 0, H_ - 1) * W_ + np.clip(np.round(u), 0, W_ - 1)).astype(np.int64)[None]
    sig = {"rays": (0.003, 10.0), "points": (0.05, 0.0), "calib": (1.0, 10.0)}[mode]
    Pp = oracle.make_params(mode, sig[0], sig[1], 0.0, 1.5, K=K, height=H_, width=W_, pixel_border=-10,
                            z_eps=1e-6)
    Twc = np.stack([Ti, Tj])
    Hs, gs = oracle.gn_align(Pp, Twc, Xs, Cs, np.array([0]), np.array([1]), idx, valid, Q)

    Mi, Mj = mat_of(Ti), mat_of(Tj)
    Xi64, Xj64 = Xs[0].astype(np.float64), Xs[1].astype(np.float64)
    targets = None
    if mode == "calib":
        targets = np.stack([idx[0] % W_, idx[0] // W_], 1).astype(np.float64)

    def res(Mi_, Mj_):
        r = residuals_f64(mode, Mi_, Mj_, Xi64[idx[0]], Xj64, K=K)
        if mode == "calib":
            r[:, :2] -= targets
        return r

    def exp_mat(d):
        t, q, s = exp_sim3_exact(d)
        M = np.eye(4)
        M[:3, :3] = s * Rot.from_quat(q).as_matrix()
        M[:3, 3] = t
        return M

    r0 = res(Mi, Mj)
    nres = r0.shape[1]
    J = np.zeros((HW, nres, 14))
    h = 1e-6
    for k in range(7):
        e = np.zeros(7)
        e[k] = h
        J[:, :, k] = (res(exp_mat(e) @ Mi, Mj) - res(exp_mat(-e) @ Mi, Mj)) / (2 * h)
        J[:, :, 7 + k] = (res(Mi, exp_mat(e) @ Mj) - res(Mi, exp_mat(-e) @ Mj)) / (2 * h)
    sq = math.sqrt(2.0)
    wv = {"rays": [1 / 0.003 ** 2] * 3 + [1 / 100.0], "points": [1 / 0.05 ** 2] * 3,
          "calib": [1.0, 1.0, 1 / 100.0]}[mode]
    wv = np.array(wv) * sq * sq
    Hd = np.einsum("pra,r,prb->ab", J, wv, J)
    gd = np.einsum("pra,r,pr->a", J, wv, r0)
    Ho = np.block([[Hs[0, 0], Hs[1, 0]], [Hs[2, 0], Hs[3, 0]]]).astype(np.float64)
    go = np.concatenate([gs[0, 0], gs[1, 0]]).astype(np.float64)
    np.testing.assert_allclose(Ho, Hd, rtol=2e-3, atol=2e-3 * np.abs(Hd).max())
    np.testing.assert_allclose(go, gd, rtol=5e-2, atol=5e-3 * max(np.abs(gd).max(), 1e-9))


@pytest.mark.parametrize("mode", ["rays", "points"])
def test_gn_converges_to_generating_poses(oracle, mode):
    g = synth.make_consistent_graph(N=5, H=24, W=32, seed=3)
    sig = {"rays": (0.003, 10.0), "points": (0.05, 0.0)}[mode]
    P = oracle.make_params(mode, sig[0], sig[1], 0.0, 1.5, max_iter=10, delta_thresh=0.0)
    T, dx, it = oracle.gauss_newton(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                                    g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
    assert it == 10
    assert np.abs(T - g.Twc_gt.numpy()).max() < 2e-5
    assert np.abs(g.Twc.numpy() - g.Twc_gt.numpy()).max() > 1e-3  # it did have to move


def test_calib_scale_only_known_answer(oracle):
    """Poses that differ only by scale map pixel grids onto each other exactly, so the
    calibrated projection + log-depth residuals vanish at the generating poses."""
    H, W, N = 16, 20, 3
    K = synth.intrinsics(H, W)
    rng = np.random.default_rng(5)
    z = rng.uniform(2, 3, H * W)
    v, u = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    base = np.stack([(u.ravel() - K[0, 2]) / K[0, 0] * z, (v.ravel() - K[1, 2]) / K[1, 1] * z, z], 1)
    scales = [1.0, 1.3, 0.8]
    gt = np.array([[0, 0, 0, 0, 0, 0, 1, s] for s in scales], np.float32)
    Xs = np.stack([base / s for s in scales]).astype(np.float32)
    init = gt.copy()
    init[1:, :3] += [[0.01, -0.02, 0.01], [-0.01, 0.01, 0.02]]
    init[1:, 7] *= [1.02, 0.97]
    q = Rot.from_rotvec([[0.01, 0.0, -0.01], [0.0, 0.01, 0.01]]).as_quat()
    init[1:, 3:7] = q
    und = [(0, 1), (1, 2), (0, 2)]
    ii = np.array([a for a, b in und] + [b for a, b in und])
    jj = np.array([b for a, b in und] + [a for a, b in und])
    E2 = len(ii)
    idx = np.tile(np.arange(H * W), (E2, 1)).astype(np.int64)
    valid = np.ones((E2, H * W, 1), np.uint8)
    Q = np.full((E2, H * W, 1), 3.0, np.float32)
    Cs = np.ones((N, H * W, 1), np.float32)
    P = oracle.make_params("calib", 1.0, 10.0, 0.0, 1.5, K=K, height=H, width=W, pixel_border=-10,
                           z_eps=1e-6, max_iter=15, delta_thresh=0.0)
    T, _, _ = oracle.gauss_newton(P, init, Xs, Cs, ii, jj, idx, valid, Q)
    assert np.abs(mat_of(T[1]) - mat_of(gt[1])).max() < 1e-4
    assert np.abs(mat_of(T[2]) - mat_of(gt[2])).max() < 1e-4


# ------------------------------------------------------------------ matching KATs


def test_iter_proj_recovers_analytic_pixel(oracle):
    """Ray image of a pinhole camera: the LM projection of a target ray converges to the
    generating sub-pixel location."""
    import torch

    from m3s.image import img_gradient

    H, W = 48, 64
    K = synth.intrinsics(H, W)
    v, u = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    d = np.stack([(u - K[0, 2]) / K[0, 0], (v - K[1, 2]) / K[1, 1], np.ones_like(u)], -1)
    rays = d / np.linalg.norm(d, axis=-1, keepdims=True)
    rt = torch.from_numpy(rays.astype(np.float32)).permute(2, 0, 1)[None]
    gx, gy = img_gradient(rt)
    img = torch.cat([rt, gx, gy], 1).permute(0, 2, 3, 1).contiguous().numpy()
    rng = np.random.default_rng(0)
    n = 200
    tu = rng.uniform(4, W - 5, n)
    tv = rng.uniform(4, H - 5, n)
    td = np.stack([(tu - K[0, 2]) / K[0, 0], (tv - K[1, 2]) / K[1, 1], np.ones(n)], -1)
    pts = (td / np.linalg.norm(td, axis=-1, keepdims=True)).astype(np.float32)[None]
    p0 = np.stack([np.round(tu) + rng.integers(-2, 3, n), np.round(tv) + rng.integers(-2, 3, n)], -1)
    p, conv = oracle.iter_proj(img, pts, p0[None].astype(np.float32), 10, 1e-8, 1e-6)
    err = np.hypot(p[0, :, 0] - tu, p[0, :, 1] - tv)
    assert np.median(err) < 0.05 and err.max() < 0.3
    assert conv.mean() > 0.9


def test_refine_recovers_planted_peaks(oracle):
    """Smooth descriptor field (as MASt3R's are); the query descriptor is an exact copy of
    the target pixel's, so the dilated coarse-to-fine search must end on the target."""
    mp = synth.make_match_pair(B=1, H=40, W=48, seed=2)
    H, W = 40, 48
    D11 = mp.D11.numpy()
    rng = np.random.default_rng(1)
    n = 300
    tu = rng.integers(3, W - 3, n)
    tv = rng.integers(3, H - 3, n)
    D21 = D11[0, tv, tu][None].copy()
    su = np.clip(tu + rng.integers(-3, 4, n), 0, W - 1)
    sv = np.clip(tv + rng.integers(-3, 4, n), 0, H - 1)
    p1 = np.stack([su, sv], -1)[None].astype(np.int64)
    out = oracle.refine_matches(D11.astype(np.float16), D21.astype(np.float16), p1, 3, 5)
    hit = (out[0, :, 0] == tu) & (out[0, :, 1] == tv)
    assert hit.mean() > 0.9, hit.mean()
    out32 = oracle.refine_matches(D11, D21, p1, 3, 5)
    assert ((out32[0, :, 0] == tu) & (out32[0, :, 1] == tv)).mean() > 0.9


def test_refine_order_and_strictness(oracle):
    """Equal scores: the first candidate in (u-offset outer, v-offset inner) order of the
    largest dilation wins, and later equal scores never replace it."""
    H = W = 40
    F = 24
    D11 = np.zeros((1, H, W, F), np.float16)
    D21 = np.zeros((1, 1, F), np.float16)
    D21[0, 0, 0] = 1.0
    # plant equal peaks at two dilation-5 window positions of a start at (20,20)
    for (u, v) in [(5, 20), (20, 5)]:  # offsets (-15,0) [i=0,j=3] and (0,-15) [i=3,j=0]
        D11[0, v, u, 0] = 0.5
    out = oracle.refine_matches(D11, D21, np.array([[[20, 20]]]), 3, 5)
    assert out[0, 0].tolist() == [5, 20]


def test_cholesky_solve_and_failure(oracle):
    rng = np.random.default_rng(0)
    A = rng.standard_normal((40, 40))
    H = A @ A.T + 40 * np.eye(40)
    b = rng.standard_normal(40)
    x, rc = oracle.cholesky_solve(H, b)
    assert rc == 0
    np.testing.assert_allclose(x, np.linalg.solve(H, b), rtol=1e-10, atol=1e-12)
    H2 = H.copy()
    H2[5, :] = 0
    H2[:, 5] = 0
    x2, rc2 = oracle.cholesky_solve(H2, b)
    assert rc2 == 1 and np.all(x2 == 0)


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_oracle_residuals_match_reference_python(oracle, mode):
    """The oracle's per-point residual model (the align kernels restated, gn_kernels.cu:905-978
    rays, :1346-1410 calib) against the reference's own Python statement of it, evaluated by
    tests/golden/make_residual_golden.py on the same points: point_to_ray_dist / project_calib
    (geometry.py:17-104) and huber (nonlinear_optimizer.py:28-33).
      * validity (match, Q, C, image border, depth) exactly;
      * residuals to 2 ulps of the operands' magnitude: the unit ray's (1) for the ray rows, the
        distance / log-depth terms, and |u| + cx (|v| + cy) for the pixel rows -- the kernel
        and the torch front end form u as fx*(x/z)+cx vs (fx*x+cx*z)/z and the norms
        differently, then cancel;
      * weights on identical residuals to 4 ulps (the kernel's huber divides k/|r| in double,
        torch multiplies by the reciprocal)."""
    import os

    O = oracle
    G = np.load(os.path.join(os.path.dirname(__file__), "golden", "residual_golden.npz"))
    g = lambda k: G[f"{mode}_{k}"]
    H, W = (int(v) for v in g("hw"))
    if mode == "rays":
        P = O.make_params("rays", 0.003, 10.0, 0.0, 1.5)
    else:
        P = O.make_params("calib", 1.0, 10.0, 0.0, 1.5, K=g("K"), height=H, width=W,
                          pixel_border=-10, z_eps=1e-6)
    ie, je, _ = O.remap(g("ii"), g("jj"))
    X, err, w, valid = O.gn_residuals(P, g("Twc"), g("Xs"), g("Cs"), ie, je, g("idx"), g("valid"), g("Q"))
    assert np.array_equal(X, g("Xj_Ci"))  # the fixture's reference functions saw these points
    ok = g("validity_ref")
    assert np.array_equal(valid, ok)
    assert 0.5 < ok.mean() < 1.0  # both valid and rejected points are covered
    R = int(g("rows"))
    scale = g("err_scale").copy()
    if mode == "rays":
        scale[..., :3] = 1.0
    else:
        K = g("K")
        scale[..., 0] += abs(K[0, 2])
        scale[..., 1] += abs(K[1, 2])
    d = np.abs(err[..., :R] - g("err_ref"))[ok]
    assert (d <= 2 * np.spacing(scale[ok])).all(), (d / np.spacing(scale[ok])).max()
    w_ref = g("w_ref_on_oracle_err")
    dw = np.abs(w[..., :R] - w_ref)
    assert (dw[ok] <= 4 * np.spacing(np.abs(w_ref[ok]))).all()
    assert np.all(w[..., :R][~ok] == 0) and np.all(w_ref[~ok] == 0)
    # both branches of huber (weight 1 and k/|r|) were exercised
    s_inv = np.float32(1.0 / (0.003 if mode == "rays" else 1.0))
    full = (s_inv * np.sqrt(g("Q")[..., 0])) ** 2
    down = w_ref[..., 0] < np.float32(0.999) * full
    assert down[ok].any() and (~down[ok]).any()
