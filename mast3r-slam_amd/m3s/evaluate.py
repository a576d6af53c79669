"""Trajectory output and ATE-RMSE (BASELINE.json metric "ATE-RMSE vs ref").

* ``save_traj`` mirrors mast3r_slam/evaluate.py:23-44: one TUM line per keyframe,
  ``timestamp x y z qx qy qz qw`` of the keyframe pose with the Sim3 scale dropped
  (lietorch_utils.as_SE3, :6-13).
* ``ate_rmse`` is what the reference's evaluation runs (scripts/eval_tum.sh:44-51:
  ``evo_ape tum groundtruth.txt estimate.txt -as``): timestamp association
  (evo ``sync.associate_trajectories``, max_diff 0.01 s), Umeyama Sim(3) alignment with scale
  (evo ``geometry.umeyama_alignment(..., with_scale=True)``), then the RMSE of the translation
  errors.  evo is a pip dependency absent here (no pinned version); this restates its published
  algorithm and is checked by known-answer tests (tests/test_evaluate.py) -- parity with evo
  itself is unpinned.
"""
from __future__ import annotations

import numpy as np


def read_tum(path):
    """TUM trajectory file -> (timestamps [n], xyz [n,3], quat xyzw [n,4]); '#' lines skipped."""
    rows = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s or s.startswith("#"):
                continue
            rows.append([float(v) for v in s.replace(",", " ").split()[:8]])
    a = np.asarray(rows, np.float64).reshape(-1, 8)
    return a[:, 0], a[:, 1:4], a[:, 4:8]


def write_tum(path, timestamps, xyz, quat):
    with open(path, "w") as f:
        for t, p, q in zip(timestamps, xyz, quat):
            f.write(f"{t} {p[0]} {p[1]} {p[2]} {q[0]} {q[1]} {q[2]} {q[3]}\n")


def save_traj(path, timestamps, frames):
    """evaluate.py:23-44 (uncalibrated branch): keyframe i -> timestamps[frame_id] and its
    T_WC as SE3 (t, q of the Sim3 data; scale dropped)."""
    with open(path, "w") as f:
        for i in range(len(frames)):
            kf = frames[i]
            d = kf.T_WC.data.detach().reshape(-1).cpu().numpy()
            x, y, z, qx, qy, qz, qw = d[:7]
            f.write(f"{timestamps[kf.frame_id]} {x} {y} {z} {qx} {qy} {qz} {qw}\n")


def associate(stamps_ref, stamps_est, max_diff=0.01, offset=0.0):
    """evo sync.associate_trajectories: for every stamp of the SHORTER trajectory, the nearest
    stamp of the longer one (plus offset) if within max_diff.  Returns index arrays
    (into ref, into est)."""
    stamps_ref = np.asarray(stamps_ref, np.float64)
    stamps_est = np.asarray(stamps_est, np.float64)
    est_longer = len(stamps_est) > len(stamps_ref)
    short, long_ = (stamps_ref, stamps_est + offset) if est_longer else (stamps_est, stamps_ref - offset)
    i_s, i_l = [], []
    for k, s in enumerate(short):
        d = np.abs(long_ - s)
        j = int(np.argmin(d))
        if d[j] <= max_diff:
            i_s.append(k)
            i_l.append(j)
    i_s, i_l = np.asarray(i_s, int), np.asarray(i_l, int)
    return (i_s, i_l) if est_longer else (i_l, i_s)


def umeyama(x, y, with_scale=True):
    """evo geometry.umeyama_alignment: (R, t, c) minimising sum ||y - (c R x + t)||^2,
    x, y [3,n]."""
    m, n = x.shape
    mx, my = x.mean(axis=1), y.mean(axis=1)
    sigma_x = 1.0 / n * np.sum(np.linalg.norm(x - mx[:, None], axis=0) ** 2)
    cov = 1.0 / n * (y - my[:, None]) @ (x - mx[:, None]).T
    u, d, v = np.linalg.svd(cov)
    s = np.eye(m)
    if np.linalg.det(u) * np.linalg.det(v) < 0.0:
        s[m - 1, m - 1] = -1.0
    r = u @ s @ v
    c = 1.0 / sigma_x * np.trace(np.diag(d) @ s) if with_scale else 1.0
    t = my - c * (r @ mx)
    return r, t, c


def ate_rmse(ref, est, max_diff=0.01, offset=0.0, with_scale=True):
    """APE (translation part) RMSE after association and Sim(3) alignment, as
    ``evo_ape tum ref est -as``.  ref / est: (timestamps, xyz[, quat]) tuples or TUM paths.
    Returns (rmse, details dict)."""
    if isinstance(ref, str):
        ref = read_tum(ref)
    if isinstance(est, str):
        est = read_tum(est)
    i_r, i_e = associate(ref[0], est[0], max_diff, offset)
    if len(i_r) < 3:
        raise ValueError(f"only {len(i_r)} associated poses; need >= 3 for a Sim(3) alignment")
    P = np.asarray(ref[1], np.float64)[i_r].T
    Q = np.asarray(est[1], np.float64)[i_e].T
    r, t, c = umeyama(Q, P, with_scale)
    err = np.linalg.norm(P - (c * (r @ Q) + t[:, None]), axis=0)
    rmse = float(np.sqrt(np.mean(err ** 2)))
    return rmse, dict(n=len(i_r), R=r, t=t, scale=c, errors=err, mean=float(err.mean()),
                      max=float(err.max()))
