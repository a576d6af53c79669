"""Deterministic synthetic workloads for the backend hot path.

Keyframes observe ONE shared world height field (z_w = 3 + 0.15 sin cos, ray-cast per
pixel, + N(0, 0.003^2) point noise) through ``K = [[400,0,256],[0,400,192],[0,0,1]]``
(scaled for smaller images), so correspondences are geometrically consistent up to pixel
quantisation.  Poses are a mean-reverting Sim3 random walk (2 deg / 5 cm /
0.01 log-scale steps) so loop-closure pairs overlap; the GN start is GT composed with a
(0.5 deg, 1 cm, 0.01) perturbation, pose 0 exact.  Correspondences come from projecting
each point through the GT relative pose; ``Q = exp(N(1, 0.5))``, ``C = 1 + exp(N(0.5,0.5))``.

Configs (BASELINE.json):
  cfg1: N=2,   E=1    (rays, 5 iters)      cfg2: N=33,  E=64   (rays)
  cfg3: N=128, E=256  (calib)              cfg4: N=256, E=1024 (rays)

Everything is generated with torch on the requested device from fixed seeds.
Pose math runs in float64 on the host.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

CONFIGS = {
    "cfg1": dict(N=2, E=1, mode="rays", iters=5),
    "cfg2": dict(N=33, E=64, mode="rays", iters=10),
    "cfg3": dict(N=128, E=256, mode="calib", iters=10),
    "cfg4": dict(N=256, E=1024, mode="rays", iters=10),
}

# ----------------------------------------------------------------------------------
# float64 Sim3 helpers: T = (t[3], q[4] xyzw, s)
# ----------------------------------------------------------------------------------


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([
        aw * bx + ax * bw + ay * bz - az * by,
        aw * by - ax * bz + ay * bw + az * bx,
        aw * bz + ax * by - ay * bx + az * bw,
        aw * bw - ax * bx - ay * by - az * bz,
    ])


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)],
    ])


def axis_angle_quat(v):
    th = np.linalg.norm(v)
    if th < 1e-12:
        return np.array([0.0, 0.0, 0.0, 1.0])
    ax = v / th
    return np.concatenate([ax * math.sin(th / 2), [math.cos(th / 2)]])


def sim3_compose(A, B):
    """A * B."""
    ta, qa, sa = A
    tb, qb, sb = B
    return (sa * quat_to_rot(qa) @ tb + ta, quat_mul(qa, qb), sa * sb)


def sim3_inv(A):
    t, q, s = A
    qi = np.array([-q[0], -q[1], -q[2], q[3]])
    return (-(1.0 / s) * (quat_to_rot(qi) @ t), qi, 1.0 / s)


def sim3_to_vec(A):
    t, q, s = A
    return np.concatenate([t, q, [s]])


def vec_to_sim3(v):
    v = np.asarray(v, dtype=np.float64)
    return (v[:3].copy(), v[3:7].copy(), float(v[7]))


def intrinsics(H, W):
    f = 400.0 * W / 512.0
    return np.array([[f, 0.0, W / 2.0], [0.0, f, H / 2.0], [0.0, 0.0, 1.0]])


@dataclass
class Graph:
    """A factor graph in exactly the layout solve_GN_* hands to the op (two-way edges)."""

    Twc: torch.Tensor        # [N,8] initial estimate (op updates it in place)
    Twc_gt: torch.Tensor     # [N,8]
    Xs: torch.Tensor         # [N,HW,3]
    Cs: torch.Tensor         # [N,HW,1]
    K: torch.Tensor          # [3,3]
    ii: torch.Tensor         # [2E] global ids (two-way)
    jj: torch.Tensor         # [2E]
    idx: torch.Tensor        # [2E,HW] i64
    valid: torch.Tensor      # [2E,HW,1] bool
    Q: torch.Tensor          # [2E,HW,1]
    H: int
    W: int
    mode: str
    iters: int

    @property
    def N(self):
        return self.Xs.shape[0]

    @property
    def HW(self):
        return self.Xs.shape[1]

    @property
    def E_directed(self):
        return self.ii.shape[0]


def make_poses(N, seed, step_rot_deg=2.0, step_t=0.05, step_ls=0.01, revert=0.9):
    rng = np.random.default_rng(seed)
    poses = [(np.zeros(3), np.array([0.0, 0.0, 0.0, 1.0]), 1.0)]
    pos = np.zeros(3)
    rotv = np.zeros(3)
    ls = 0.0
    for _ in range(1, N):
        pos = revert * pos + rng.normal(0, step_t / math.sqrt(3), 3)
        rotv = revert * rotv + rng.normal(0, math.radians(step_rot_deg) / math.sqrt(3), 3)
        ls = revert * ls + rng.normal(0, step_ls)
        poses.append((pos.copy(), axis_angle_quat(rotv), math.exp(ls)))
    return poses


def perturb(poses, seed, rot_deg=0.5, t=0.01, ls=0.01):
    rng = np.random.default_rng(seed + 1000)
    out = [poses[0]]
    for P in poses[1:]:
        d = (rng.normal(0, t / math.sqrt(3), 3),
             axis_angle_quat(rng.normal(0, math.radians(rot_deg) / math.sqrt(3), 3)),
             math.exp(rng.normal(0, ls)))
        out.append(sim3_compose(P, d))
    return out


def make_edges(N, E, seed):
    """Chain edges (k-1, k) plus loop closures (j, k) with j <= k-2, deduplicated."""
    rng = np.random.default_rng(seed + 2000)
    edges = [(k - 1, k) for k in range(1, N)][:E]
    seen = set(edges)
    tries = 0
    while len(edges) < E and tries < 100 * E + 1000:
        tries += 1
        k = int(rng.integers(2, N)) if N > 2 else 1
        if k < 2:
            break
        j = int(rng.integers(0, k - 1))
        if (j, k) not in seen:
            seen.add((j, k))
            edges.append((j, k))
    return edges


def depth_maps(N, H, W, gen, device):
    v = torch.arange(H, device=device, dtype=torch.float32)[:, None]
    u = torch.arange(W, device=device, dtype=torch.float32)[None, :]
    ph = torch.rand((N, 2), generator=gen, device=device) * 2 * math.pi
    z = 2.0 + 0.4 * torch.sin(2 * math.pi * 3 * u / W + ph[:, 0, None, None]) * torch.cos(
        2 * math.pi * 2 * v / H + ph[:, 1, None, None]
    )
    lo = torch.randn((N, 1, 12, 16), generator=gen, device=device)
    z = z + 0.1 * torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=True)[:, 0]
    return z.clamp(0.5, 5.0)


def world_surface_z(xw, yw, phase):
    """Shared world height field z_w = 3 + 0.15 sin(2pi x/2 + p0) cos(2pi y/2 + p1)."""
    return 3.0 + 0.15 * torch.sin(math.pi * xw + phase[0]) * torch.cos(math.pi * yw + phase[1])


def raycast_keyframe(pose, Kn, H, W, phase, device, iters=12):
    """Camera-frame points of the shared world surface seen through every pixel of a
    keyframe with camera-to-world Sim3 ``pose`` (fixed-point ray / height-field
    intersection; the surface slope keeps the iteration contractive)."""
    t, q, s = pose
    R = torch.tensor(quat_to_rot(q), dtype=torch.float64, device=device)
    o = torch.tensor(t, dtype=torch.float64, device=device)
    v, u = torch.meshgrid(torch.arange(H, device=device, dtype=torch.float64),
                          torch.arange(W, device=device, dtype=torch.float64), indexing="ij")
    dc = torch.stack(((u - Kn[0, 2]) / Kn[0, 0], (v - Kn[1, 2]) / Kn[1, 1], torch.ones_like(u)), -1)
    dw = s * dc @ R.T  # world direction of the camera-frame ray point at depth 1
    lam = (3.0 - o[2]) / dw[..., 2]
    for _ in range(iters):
        P = o + lam[..., None] * dw
        lam = (world_surface_z(P[..., 0], P[..., 1], phase) - o[2]) / dw[..., 2]
    return (lam[..., None] * dc).reshape(H * W, 3).float()


def make_graph(cfg="cfg1", H=384, W=512, device="cpu", seed=None, mode=None, edges_only=None,
               edge_range=None, init_perturb=None, outlier_frac=0.0) -> Graph:
    """Build a synthetic graph.  ``edge_range=(lo, hi)`` materialises idx/valid/Q only for the
    directed edges lo..hi-1 (a rank's shard); ii/jj always cover all 2E directed edges.

    Stress options (a graph the GN is NOT converged on after 10 iterations): ``init_perturb =
    (rot_deg, t, log_scale)`` replaces the (0.5 deg, 1 cm, 0.01) start perturbation;
    ``outlier_frac`` of the valid matches of every directed edge point at a uniformly random
    pixel instead (gross outliers: the Huber weights and, for calib, the image-border validity
    become active).  Both draw from their own generators, so the rest of the graph is unchanged."""
    spec = dict(CONFIGS[cfg]) if isinstance(cfg, str) else dict(cfg)
    if seed is None:
        seed = {"cfg1": 1, "cfg2": 2, "cfg3": 3, "cfg4": 4}.get(cfg, 0) if isinstance(cfg, str) else 0
    N, E = spec["N"], spec["E"]
    mode = mode or spec.get("mode", "rays")
    iters = spec.get("iters", 10)
    HW = H * W
    gen = torch.Generator(device=device).manual_seed(seed)
    Kn = intrinsics(H, W)
    K = torch.tensor(Kn, dtype=torch.float32, device=device)

    gt = make_poses(N, seed)
    init = perturb(gt, seed) if init_perturb is None else perturb(gt, seed, *init_perturb)
    gen_out = torch.Generator(device=device).manual_seed(seed + 5000)
    phase = np.random.default_rng(seed + 3000).uniform(0, 2 * math.pi, 2)
    Xs = torch.stack([raycast_keyframe(gt[k], Kn, H, W, phase, device) for k in range(N)])
    Xs = Xs + 0.003 * torch.randn(Xs.shape, generator=gen, device=device)
    Cs = 1.0 + torch.exp(0.5 + 0.5 * torch.randn((N, HW, 1), generator=gen, device=device))

    und = make_edges(N, E, seed) if edges_only is None else edges_only
    ii = [a for a, b in und] + [b for a, b in und]
    jj = [b for a, b in und] + [a for a, b in und]
    E2 = len(ii)
    lo, hi = (0, E2) if edge_range is None else edge_range
    idx = torch.empty((hi - lo, HW), dtype=torch.int64, device=device)
    valid = torch.empty((hi - lo, HW, 1), dtype=torch.bool, device=device)
    Q = torch.empty((hi - lo, HW, 1), dtype=torch.float32, device=device)
    Kt = torch.tensor(Kn, dtype=torch.float32, device=device)
    for e in range(lo, hi):
        i, j = ii[e], jj[e]
        Tij = sim3_compose(sim3_inv(gt[i]), gt[j])
        R = torch.tensor(Tij[2] * quat_to_rot(Tij[1]), dtype=torch.float32, device=device)
        t = torch.tensor(Tij[0], dtype=torch.float32, device=device)
        P = Xs[j] @ R.T + t
        zc = P[:, 2]
        uu = torch.round(Kt[0, 0] * P[:, 0] / zc + Kt[0, 2])
        vv = torch.round(Kt[1, 1] * P[:, 1] / zc + Kt[1, 2])
        ok = (zc > 0) & (uu >= 0) & (uu <= W - 1) & (vv >= 0) & (vv <= H - 1)
        lin = (vv.clamp(0, H - 1) * W + uu.clamp(0, W - 1)).long()
        idx[e - lo] = torch.where(ok, lin, torch.zeros_like(lin))
        valid[e - lo, :, 0] = ok
        Q[e - lo, :, 0] = torch.exp(1.0 + 0.5 * torch.randn((HW,), generator=gen, device=device))
        if outlier_frac > 0:
            bad = ok & (torch.rand((HW,), generator=gen_out, device=device) < outlier_frac)
            wrong = torch.randint(0, HW, (HW,), generator=gen_out, device=device)
            idx[e - lo] = torch.where(bad, wrong, idx[e - lo])

    to_t = lambda ps: torch.tensor(np.stack([sim3_to_vec(p) for p in ps]), dtype=torch.float32, device=device)
    return Graph(
        Twc=to_t(init), Twc_gt=to_t(gt), Xs=Xs.contiguous(), Cs=Cs.contiguous(), K=K,
        ii=torch.tensor(ii, dtype=torch.int64, device=device),
        jj=torch.tensor(jj, dtype=torch.int64, device=device),
        idx=idx, valid=valid, Q=Q, H=H, W=W, mode=mode, iters=iters,
    )


def make_consistent_graph(N=4, E=None, H=24, W=32, seed=0, device="cpu"):
    """Known-answer graph: every keyframe sees the SAME world points (a per-frame pixel
    permutation), so the two-way residuals vanish exactly at the GT poses."""
    rng = np.random.default_rng(seed)
    HW = H * W
    gt = make_poses(N, seed, step_rot_deg=3.0, step_t=0.05, step_ls=0.02, revert=0.8)
    init = perturb(gt, seed, rot_deg=1.0, t=0.02, ls=0.02)
    P = np.stack([rng.uniform(-1, 1, HW), rng.uniform(-0.8, 0.8, HW), rng.uniform(2.0, 4.0, HW)], -1)
    perms = [rng.permutation(HW) for _ in range(N)]  # perm[f][k] = pixel of world point k in frame f
    Xs = np.zeros((N, HW, 3))
    for f in range(N):
        Tinv = sim3_inv(gt[f])
        Pf = (Tinv[2] * (quat_to_rot(Tinv[1]) @ P.T)).T + Tinv[0]
        Xs[f, perms[f]] = Pf
    und = [(k - 1, k) for k in range(1, N)]
    extra = [(a, b) for a in range(N) for b in range(a + 2, N)]
    n_extra = 2 if E is None else max(0, E - len(und))
    und += extra[:n_extra]
    ii = [a for a, b in und] + [b for a, b in und]
    jj = [b for a, b in und] + [a for a, b in und]
    inv = [np.argsort(p) for p in perms]  # inv[f][pixel] = world point
    idx = np.stack([perms[i][inv[j]] for i, j in zip(ii, jj)])  # pixel in i for pixel k of j
    E2 = len(ii)
    to_t = lambda ps: torch.tensor(np.stack([sim3_to_vec(p) for p in ps]), dtype=torch.float32, device=device)
    return Graph(
        Twc=to_t(init), Twc_gt=to_t(gt),
        Xs=torch.tensor(Xs, dtype=torch.float32, device=device),
        Cs=torch.full((N, HW, 1), 2.0, dtype=torch.float32, device=device),
        K=torch.tensor(intrinsics(H, W), dtype=torch.float32, device=device),
        ii=torch.tensor(ii, dtype=torch.int64, device=device),
        jj=torch.tensor(jj, dtype=torch.int64, device=device),
        idx=torch.tensor(idx, dtype=torch.int64, device=device),
        valid=torch.ones((E2, HW, 1), dtype=torch.bool, device=device),
        Q=torch.full((E2, HW, 1), 3.0, dtype=torch.float32, device=device),
        H=H, W=W, mode="rays", iters=10,
    )


# ----------------------------------------------------------------------------------
# matching pairs
# ----------------------------------------------------------------------------------


@dataclass
class MatchPair:
    X11: torch.Tensor  # [B,H,W,3]
    X21: torch.Tensor  # [B,H,W,3] image-2 points in frame 1
    D11: torch.Tensor  # [B,H,W,24] f32 (unit norm)
    D21: torch.Tensor  # [B,H,W,24]
    idx_gt: torch.Tensor  # [B,HW] GT linear pixel in image 1 of each image-2 pixel
    idx_init: torch.Tensor  # [B,HW] warm start: GT +- 2 px


def make_match_pair(B=1, H=384, W=512, F=24, seed=7, device="cpu") -> MatchPair:
    """X21[n] is the image-1 surface point at a smooth flow-displaced pixel (+ noise); D21[n] is
    D11 at the GT match + noise (SURVEY.md §8(d) 'Matching pair')."""
    gen = torch.Generator(device=device).manual_seed(seed)
    Kn = intrinsics(H, W)
    z = depth_maps(B, H, W, gen, device)
    v, u = torch.meshgrid(torch.arange(H, device=device), torch.arange(W, device=device), indexing="ij")
    x = (u.float() - Kn[0, 2]) / Kn[0, 0]
    y = (v.float() - Kn[1, 2]) / Kn[1, 1]
    X11 = torch.stack((x[None] * z, y[None] * z, z), dim=-1)
    # smooth flow field (a few pixels) from low-res noise
    lo = torch.randn((B, 2, 6, 8), generator=gen, device=device) * 4.0
    flow = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=True)
    ug = (u[None].float() + flow[:, 0]).round().clamp(0, W - 1).long()
    vg = (v[None].float() + flow[:, 1]).round().clamp(0, H - 1).long()
    idx_gt = (vg * W + ug).reshape(B, H * W)
    bi = torch.arange(B, device=device)[:, None]
    X21 = X11.reshape(B, H * W, 3)[bi, idx_gt].reshape(B, H, W, 3)
    X21 = X21 + 0.002 * torch.randn(X21.shape, generator=gen, device=device)
    d = torch.randn((B, F, H // 4 + 1, W // 4 + 1), generator=gen, device=device)
    d = torch.nn.functional.interpolate(d, size=(H, W), mode="bilinear", align_corners=False)
    d = d + 0.3 * torch.randn((B, F, H, W), generator=gen, device=device)
    D11 = torch.nn.functional.normalize(d.permute(0, 2, 3, 1), dim=-1).contiguous()
    D21 = D11.reshape(B, H * W, F)[bi, idx_gt] + 0.05 * torch.randn((B, H * W, F), generator=gen, device=device)
    D21 = torch.nn.functional.normalize(D21, dim=-1).reshape(B, H, W, F).contiguous()
    jit = torch.randint(-2, 3, (B, H * W, 2), generator=gen, device=device)
    ui = (idx_gt % W + jit[..., 0]).clamp(0, W - 1)
    vi = (idx_gt // W + jit[..., 1]).clamp(0, H - 1)
    return MatchPair(X11.contiguous(), X21.contiguous(), D11, D21, idx_gt, vi * W + ui)


def make_tracking_inputs(hw=(384, 512), seed=0, mode="rays", noise=0.003, device="cpu"):
    """Synthetic frame/keyframe pair in the layout FrameTracker's optimisers take
    (tracker.py:173-266): Xf [HW,3] (already gathered by the match), Xk [HW,3], T_WCf / T_WCk
    [1,8], Qk [HW,1], valid [HW,1] bool; calib adds meas_k [HW,3], valid_meas_k [HW,1], K."""
    rng = np.random.default_rng(seed)
    h, w = hw
    n = h * w
    Kn = intrinsics(h, w)
    uu, vv = np.meshgrid(np.arange(w), np.arange(h))
    z = 2.0 + 0.3 * np.sin(uu / w * 6.0) * np.cos(vv / h * 4.0) + 0.05 * rng.standard_normal((h, w))
    rays = np.stack([(uu - Kn[0, 2]) / Kn[0, 0], (vv - Kn[1, 2]) / Kn[1, 1], np.ones((h, w))], -1)
    Xk = (rays * z[..., None]).reshape(n, 3)
    T_kf = (rng.normal(0, 0.03, 3), axis_angle_quat(rng.normal(0, 0.02, 3)), math.exp(rng.normal(0, 0.02)))
    t, q, s = sim3_inv(T_kf)
    Xf = s * Xk @ quat_to_rot(q).T + t + noise * rng.standard_normal((n, 3))
    T_WCk = (rng.normal(0, 0.5, 3), axis_angle_quat(rng.normal(0, 0.1, 3)), math.exp(rng.normal(0, 0.1)))
    T_true = sim3_compose(T_WCk, T_kf)
    dT = (rng.normal(0, 0.01, 3), axis_angle_quat(rng.normal(0, 0.01, 3)), math.exp(rng.normal(0, 0.005)))
    T_WCf = sim3_compose(dT, T_true)
    f32 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device=device)
    out = dict(Xf=f32(Xf), Xk=f32(Xk), T_WCf=f32(sim3_to_vec(T_WCf)).reshape(1, 8),
               T_WCk=f32(sim3_to_vec(T_WCk)).reshape(1, 8),
               Qk=f32(np.exp(rng.normal(1.0, 0.5, (n, 1)))),
               valid=torch.tensor(rng.random((n, 1)) > 0.1, device=device), K=f32(Kn))
    if mode == "calib":
        zk = out["Xk"][:, 2:3]
        valid_meas = zk > 1e-6
        uv = torch.stack([torch.arange(n, device=device) % w, torch.arange(n, device=device) // w], -1)
        meas = torch.cat([uv.float(), torch.log(zk)], -1)
        meas[~valid_meas.repeat(1, 3)] = 0.0
        out.update(meas_k=meas.contiguous(), valid_meas_k=valid_meas.contiguous())
    return out
