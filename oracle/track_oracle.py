"""CPU oracle of the frame tracker's Sim3 Gauss-Newton (float64 numpy).

TEST INFRASTRUCTURE ONLY: imported by tests/, tests/golden/make_track_golden.py and bench.py's
cpu_baseline leg -- never by the product path (mast3r-slam_amd/).

Restates, line by line:
  * FrameTracker.opt_pose_ray_dist_sim3 / opt_pose_calib_sim3   tracker.py:173-266
  * FrameTracker.solve                                           tracker.py:156-171
  * check_convergence, huber                                     nonlinear_optimizer.py:5-33
  * point_to_ray_dist, act_Sim3, project_calib, skew_sym          geometry.py:5-104
  * the lietorch Sim3 group (act, inv, mul, Exp, retr = Exp(a) * X) used by them.
    lietorch (git dependency, no pinned revision, absent here) is restated from its published
    algorithm: tangent order (tau, phi, sigma), data (t, q xyzw, s); its Exp is the formula the
    reference backend inlines as expSim3 (gn_kernels.cu:323-390, incl. the as-written B) --
    parity of these group operations with lietorch itself is UNPINNED.

``Sim3T`` is a torch implementation of the same group for driving the REFERENCE tracker code
(tests/golden/make_track_golden.py), which imports lietorch.
"""
from __future__ import annotations

import math

import numpy as np

# ----------------------------------------------------------------------------- Sim3 (f64)


def quat_mul(a, b):
    ax, ay, az, aw = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    bx, by, bz, bw = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    return np.stack([
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by - ax * bz + ay * bw + az * bx,
        aw * bz + ax * by - ay * bx + az * bw,
        aw * bw - ax * bx - ay * by - az * bz,
    ], axis=-1)


def quat_rot(q, p):
    """R(q) p for unit q (xyzw), p [...,3]."""
    u = q[..., :3]
    w = q[..., 3:4]
    uv = 2.0 * np.cross(u, p)
    return p + w * uv + np.cross(u, uv)


def sim3_act(T, p):
    return T[..., 7:8] * quat_rot(T[..., 3:7], p) + T[..., 0:3]


def sim3_inv(T):
    s = 1.0 / T[..., 7:8]
    qi = T[..., 3:7] * np.array([-1.0, -1.0, -1.0, 1.0])
    t = -s * quat_rot(qi, T[..., 0:3])
    return np.concatenate([t, qi, s], axis=-1)


def sim3_mul(A, B):
    t = A[..., 0:3] + A[..., 7:8] * quat_rot(A[..., 3:7], B[..., 0:3])
    return np.concatenate([t, quat_mul(A[..., 3:7], B[..., 3:7]), A[..., 7:8] * B[..., 7:8]], axis=-1)


def sim3_exp(xi):
    """Exp of a tangent (tau, phi, sigma) -> data (t, q, s)  (expSim3, gn_kernels.cu:323-390)."""
    xi = np.asarray(xi, np.float64)
    tau, phi, sigma = xi[0:3], xi[3:6], float(xi[6])
    th2 = float(phi @ phi)
    th = math.sqrt(th2)
    if th2 < 1e-6:
        imag = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0
        real = 1.0 - th2 / 8.0 + th2 * th2 / 384.0
    else:
        imag = math.sin(0.5 * th) / th
        real = math.cos(0.5 * th)
    q = np.array([imag * phi[0], imag * phi[1], imag * phi[2], real])
    scale = math.exp(sigma)
    if abs(sigma) < 1e-6:
        C = 1.0
        if abs(th) < 1e-6:
            A, B = 0.5, 1.0 / 6.0
        else:
            A = (1.0 - math.cos(th)) / th2
            B = (th - math.sin(th)) / (th2 * th)
    else:
        C = (scale - 1.0) / sigma
        if abs(th) < 1e-6:
            s2 = sigma * sigma
            A = ((sigma - 1.0) * scale + 1.0) / s2
            B = (scale * 0.5 * s2 + scale - 1.0 - sigma * scale) / (s2 * sigma)
        else:
            a = scale * math.sin(th)
            b = scale * math.cos(th)
            c = th2 + sigma * sigma
            A = (a * sigma + (1.0 - b) * th) / (th * c)
            B = (C - ((b - 1.0) * sigma + a * th) / c) / th2
    c1 = np.cross(phi, tau)
    c2 = np.cross(phi, c1)
    t = C * tau + A * c1 + B * c2
    return np.concatenate([t, q, [scale]])


def sim3_retr(T, xi):
    """lietorch retr: Exp(xi) * T."""
    return sim3_mul(sim3_exp(xi), T)


# ----------------------------------------------------------------------------- residuals


def huber(r, k=1.345):
    a = np.abs(r)
    return np.where(a < k, 1.0, k / np.where(a == 0, 1.0, a))


def skew(X):
    x, y, z = X[..., 0], X[..., 1], X[..., 2]
    o = np.zeros_like(x)
    return np.stack([o, -z, y, z, o, -x, -y, x, o], axis=-1).reshape(*X.shape[:-1], 3, 3)


def act_jac(pW):
    """d(Exp(xi) T p)/dxi at 0 = [I | -skew(pW) | pW]  (act_Sim3, geometry.py:45-52)."""
    n = pW.shape[0]
    return np.concatenate([np.broadcast_to(np.eye(3), (n, 3, 3)), -skew(pW), pW[..., None]], axis=-1)


def point_to_ray_dist(X, jacobian=False):
    d = np.linalg.norm(X, axis=-1, keepdims=True)
    dinv = 1.0 / d
    r = dinv * X
    rd = np.concatenate([r, d], axis=-1)
    if not jacobian:
        return rd
    I = np.eye(3)
    dr = dinv[..., None] * (I - (dinv ** 2)[..., None] * (X[..., :, None] * X[..., None, :]))
    return rd, np.concatenate([dr, r[..., None, :]], axis=-2)


def project_calib(P, K, img_size, border, z_eps):
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        u = (fx * x + cx * z) / z
        v = (fy * y + cy * z) / z
        valid = (u > border) & (u < img_size[1] - 1 - border) & (v > border) & \
            (v < img_size[0] - 1 - border) & (z > z_eps)
        logz = np.where(z > z_eps, np.log(np.where(z > z_eps, z, 1.0)), 0.0)
        zinv = 1.0 / z
    D = np.zeros((P.shape[0], 3, 3))
    D[:, 0, 0] = fx * zinv
    D[:, 1, 1] = fy * zinv
    D[:, 0, 2] = -fx * x * zinv * zinv
    D[:, 1, 2] = -fy * y * zinv * zinv
    D[:, 2, 2] = zinv
    return np.stack([u, v, logz], axis=-1), D, valid


def _solve(sqrt_info, r, J, k):
    """tracker.py:156-171 (float64): returns tau [7], cost; raises on a non-PD system."""
    wr = sqrt_info * r
    ris = sqrt_info * np.sqrt(huber(wr, k))
    A = (ris[..., None] * J).reshape(-1, 7)
    b = (ris * r).reshape(-1, 1)
    H = A.T @ A
    g = -A.T @ b
    cost = 0.5 * float((b.T @ b)[0, 0])
    L = np.linalg.cholesky(H)  # LinAlgError when not positive definite
    tau = np.linalg.solve(L.T, np.linalg.solve(L, g))
    return tau.reshape(-1), cost


def _converged(rel_error, delta_norm, old_cost, new_cost, tau):
    with np.errstate(invalid="ignore"):
        rel = abs((old_cost - new_cost) / old_cost) if math.isfinite(old_cost) else float("nan")
    return rel < rel_error or float(np.linalg.norm(tau)) < delta_norm


def opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg, max_iters=None):
    """tracker.py:173-214 -> (T_WCf, T_CkCf, iterations, last cost)."""
    Xf, Xk, Qk = (np.asarray(a, np.float64) for a in (Xf, Xk, Qk))
    v = np.asarray(valid, np.float64)
    T_WCf = np.asarray(T_WCf, np.float64).reshape(8)
    T_WCk = np.asarray(T_WCk, np.float64).reshape(8)
    sq = np.sqrt(Qk)
    si = np.concatenate([np.repeat((1.0 / cfg["sigma_ray"]) * v * sq, 3, axis=1),
                         (1.0 / cfg["sigma_dist"]) * v * sq], axis=1)
    T = sim3_mul(sim3_inv(T_WCk), T_WCf)
    rd_k = point_to_ray_dist(Xk)
    old = float("inf")
    it = 0
    cost = 0.0
    for step in range(cfg["max_iters"] if max_iters is None else max_iters):
        X = sim3_act(T, Xf)
        rd_f, drd = point_to_ray_dist(X, jacobian=True)
        r = rd_k - rd_f
        J = -drd @ act_jac(X)
        tau, cost = _solve(si, r, J, cfg["huber"])
        T = sim3_retr(T, tau)
        it = step + 1
        if _converged(cfg["rel_error"], cfg["delta_norm"], old, cost, tau):
            break
        old = cost
    return sim3_mul(T_WCk, T), T, it, cost


def opt_pose_calib_sim3(Xf, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size, cfg,
                        max_iters=None):
    """tracker.py:216-266 -> (T_WCf, T_CkCf, iterations, last cost)."""
    Xf, Qk, meas_k = (np.asarray(a, np.float64) for a in (Xf, Qk, meas_k))
    K = np.asarray(K, np.float64)
    v = np.asarray(valid, np.float64)
    vm = np.asarray(valid_meas_k, bool)
    T_WCf = np.asarray(T_WCf, np.float64).reshape(8)
    T_WCk = np.asarray(T_WCk, np.float64).reshape(8)
    sq = np.sqrt(Qk)
    si = np.concatenate([np.repeat((1.0 / cfg["sigma_pixel"]) * v * sq, 2, axis=1),
                         (1.0 / cfg["sigma_depth"]) * v * sq], axis=1)
    T = sim3_mul(sim3_inv(T_WCk), T_WCf)
    old = float("inf")
    it = 0
    cost = 0.0
    for step in range(cfg["max_iters"] if max_iters is None else max_iters):
        X = sim3_act(T, Xf)
        pz, D, vp = project_calib(X, K, img_size, cfg["pixel_border"], cfg["depth_eps"])
        si2 = (vp[:, None] & vm).astype(np.float64) * si
        r = meas_k - pz
        J = -D @ act_jac(X)
        tau, cost = _solve(si2, r, J, cfg["huber"])
        T = sim3_retr(T, tau)
        it = step + 1
        if _converged(cfg["rel_error"], cfg["delta_norm"], old, cost, tau):
            break
        old = cost
    return sim3_mul(T_WCk, T), T, it, cost


def calib_measurements(Xk, img_size, depth_eps):
    """get_points_poses' keyframe measurement (tracker.py:146-152): (u, v, log z), 0 where
    z <= depth_eps, and the validity mask.  Xk must already be constrained to its rays."""
    h, w = img_size
    Xk = np.asarray(Xk, np.float64)
    n = np.arange(h * w)
    uv = np.stack([n % w, n // w], axis=-1).astype(np.float64)
    z = Xk[:, 2:3]
    valid = z > depth_eps
    with np.errstate(divide="ignore", invalid="ignore"):
        meas = np.concatenate([uv, np.log(np.where(valid, z, 1.0))], axis=-1)
    meas[~np.repeat(valid, 3, axis=1)] = 0.0
    return meas, valid


# ----------------------------------------------------------------------------- torch Sim3


def _torch_sim3():
    import torch

    def qmul(a, b):
        ax, ay, az, aw = a.unbind(-1)
        bx, by, bz, bw = b.unbind(-1)
        return torch.stack([aw * bx + ax * bw + ay * bz - az * by,
                            aw * by - ax * bz + ay * bw + az * bx,
                            aw * bz + ax * by - ay * bx + az * bw,
                            aw * bw - ax * bx - ay * by - az * bz], -1)

    def qrot(q, p):
        u, w = q[..., :3], q[..., 3:4]
        uv = 2.0 * torch.cross(u.expand_as(p), p, dim=-1)
        return p + w * uv + torch.cross(u.expand_as(p), uv, dim=-1)

    class Sim3T:
        """lietorch.Sim3 stand-in (same algorithm as the numpy group above, any dtype)."""

        def __init__(self, data):
            self.data = data

        def __getitem__(self, k):
            return Sim3T(self.data[k])

        @classmethod
        def Identity(cls, n, device="cpu", dtype=torch.float32):
            d = torch.zeros((n, 8), device=device, dtype=dtype)
            d[:, 6] = 1.0
            d[:, 7] = 1.0
            return cls(d)

        def act(self, p):
            d = self.data
            shp = [1] * (p.dim() - 1) + [8]
            d = d.reshape(shp) if d.numel() == 8 else d
            return d[..., 7:8] * qrot(d[..., 3:7], p) + d[..., 0:3]

        def inv(self):
            d = self.data
            s = 1.0 / d[..., 7:8]
            qi = d[..., 3:7] * torch.tensor([-1.0, -1.0, -1.0, 1.0], dtype=d.dtype)
            t = -s * qrot(qi, d[..., 0:3])
            return Sim3T(torch.cat([t, qi, s], -1))

        def __mul__(self, o):
            a, b = self.data, o.data
            t = a[..., 0:3] + a[..., 7:8] * qrot(a[..., 3:7], b[..., 0:3])
            return Sim3T(torch.cat([t, qmul(a[..., 3:7], b[..., 3:7]), a[..., 7:8] * b[..., 7:8]], -1))

        def retr(self, a):
            e = sim3_exp(a.detach().double().reshape(-1).numpy())
            E = torch.tensor(e, dtype=self.data.dtype).reshape(self.data.shape)
            return Sim3T(E) * self

    return Sim3T


def make_tracking_pair(HW_shape=(24, 32), seed=0, mode="rays", noise=0.0):
    """Synthetic frame/keyframe pair with a known relative Sim3 (test/bench input).
    Returns a dict of float32 numpy arrays shaped like the tracker's inputs."""
    rng = np.random.default_rng(seed)
    h, w = HW_shape
    n = h * w
    K = np.array([[0.8 * w, 0, w / 2], [0, 0.8 * w, h / 2], [0, 0, 1]], np.float64)
    uu, vv = np.meshgrid(np.arange(w), np.arange(h))
    z = 2.0 + 0.3 * np.sin(uu / w * 6.0) * np.cos(vv / h * 4.0) + 0.05 * rng.standard_normal((h, w))
    rays = np.stack([(uu - K[0, 2]) / K[0, 0], (vv - K[1, 2]) / K[1, 1], np.ones_like(uu, float)], -1)
    Xk = (rays * z[..., None]).reshape(n, 3)
    ang = rng.normal(0, 0.02, 3)
    th = np.linalg.norm(ang)
    q = np.concatenate([np.sin(th / 2) * ang / th, [np.cos(th / 2)]])
    T_kf = np.concatenate([rng.normal(0, 0.03, 3), q, [math.exp(rng.normal(0, 0.02))]])
    # frame points: keyframe points seen from the frame, T_CkCf * Xf = Xk
    Xf = sim3_act(sim3_inv(T_kf), Xk) + noise * rng.standard_normal((n, 3))
    ang0 = rng.normal(0, 0.1, 3)
    th0 = np.linalg.norm(ang0)
    q0 = np.concatenate([np.sin(th0 / 2) * ang0 / th0, [np.cos(th0 / 2)]])
    T_WCk = np.concatenate([rng.normal(0, 0.5, 3), q0, [math.exp(rng.normal(0, 0.1))]])
    T_WCf_true = sim3_mul(T_WCk, T_kf)
    # initial frame pose: the truth perturbed
    T_WCf0 = sim3_retr(T_WCf_true, rng.normal(0, 0.01, 7) * np.array([1, 1, 1, 1, 1, 1, 0.5]))
    Q = np.exp(rng.normal(1.0, 0.5, (n, 1)))
    valid = rng.random((n, 1)) > 0.1
    out = dict(Xf=Xf, Xk=Xk, T_WCf=T_WCf0, T_WCk=T_WCk, T_WCf_true=T_WCf_true, Qk=Q, valid=valid, K=K)
    if mode == "calib":
        meas, vm = calib_measurements(Xk, (h, w), 1e-6)
        out.update(meas_k=meas, valid_meas_k=vm)
    return {k: (v.astype(np.float32) if v.dtype.kind == "f" else v) for k, v in out.items()}


TRACKING_CFG = {  # config/base.yaml:16-33
    "min_match_frac": 0.05, "max_iters": 50, "C_conf": 0.0, "Q_conf": 1.5, "rel_error": 1e-3,
    "delta_norm": 1e-3, "huber": 1.345, "match_frac_thresh": 0.333, "sigma_ray": 0.003,
    "sigma_dist": 1e1, "sigma_pixel": 1.0, "sigma_depth": 1e1, "sigma_point": 0.05,
    "pixel_border": -10, "depth_eps": 1e-6,
}
