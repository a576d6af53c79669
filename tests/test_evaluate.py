"""ATE-RMSE (m3s/evaluate.py, the reference's evo_ape -as evaluation) by known answers:
exact Sim(3)-transformed trajectories align to zero error, Umeyama is optimal against
perturbations, association follows evo's nearest-stamp rule, TUM IO round-trips."""
import numpy as np
import pytest

from m3s import evaluate as ev


def _rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _traj(n=200, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) * 0.033 + 1305031102.0
    xyz = np.cumsum(rng.normal(0, 0.02, (n, 3)), axis=0)
    q = np.tile([0.0, 0.0, 0.0, 1.0], (n, 1))
    return t, xyz, q


def test_exact_sim3_copy_has_zero_ate():
    t, xyz, q = _traj()
    rng = np.random.default_rng(1)
    R, s, tr = _rot(rng), 0.37, rng.normal(size=3)
    est_xyz = (s * (R @ xyz.T)).T + tr
    rmse, d = ev.ate_rmse((t, xyz, q), (t, est_xyz, q))
    assert rmse < 1e-10 and d["n"] == len(t)
    assert abs(d["scale"] - 1 / s) < 1e-10


def test_noise_rmse_and_alignment_optimality():
    t, xyz, q = _traj(seed=2)
    rng = np.random.default_rng(3)
    noisy = xyz + rng.normal(0, 0.01, xyz.shape)
    rmse, d = ev.ate_rmse((t, xyz, q), (t, noisy, q))
    assert 0.005 < rmse < 0.02
    # any perturbation of the optimal (R, t, c) increases the error
    P, Q = xyz.T, noisy.T

    def cost(R, tt, c):
        return np.sqrt(np.mean(np.linalg.norm(P - (c * (R @ Q) + tt[:, None]), axis=0) ** 2))

    assert abs(cost(d["R"], d["t"], d["scale"]) - rmse) < 1e-12
    for k in range(20):
        e = rng.normal(0, 1e-3, 7)
        K = np.array([[0, -e[2], e[1]], [e[2], 0, -e[0]], [-e[1], e[0], 0]])
        R2 = d["R"] @ (np.eye(3) + K)
        assert cost(R2, d["t"] + e[3:6], d["scale"] * (1 + e[6])) >= rmse - 1e-12


def test_reflection_is_excluded():
    t, xyz, q = _traj(seed=4)
    mirrored = xyz * np.array([1.0, 1.0, -1.0])
    _, d = ev.ate_rmse((t, xyz, q), (t, mirrored, q))
    assert np.linalg.det(d["R"]) > 0.999


def test_association_nearest_stamp_within_max_diff():
    ref = np.array([0.0, 1.0, 2.0, 3.0, 4.0])
    est = np.array([0.004, 1.02, 2.009, 3.0, 3.995, 10.0])  # longer: iterate over ref
    i_r, i_e = ev.associate(ref, est, max_diff=0.01)
    assert i_r.tolist() == [0, 2, 3, 4] and i_e.tolist() == [0, 2, 3, 4]
    # shorter estimate: iterate over est
    i_r, i_e = ev.associate(ref, est[:3], max_diff=0.01)
    assert i_r.tolist() == [0, 2] and i_e.tolist() == [0, 2]


def test_too_few_poses_raises():
    t, xyz, q = _traj(n=2)
    with pytest.raises(ValueError):
        ev.ate_rmse((t, xyz, q), (t, xyz, q))


def test_tum_round_trip_and_save_traj(tmp_path):
    import torch

    from m3s.global_opt import PoseBatch

    t, xyz, q = _traj(n=5)
    p = tmp_path / "a.txt"
    ev.write_tum(str(p), t, xyz, q)
    t2, xyz2, q2 = ev.read_tum(str(p))
    assert np.allclose(t2, t) and np.allclose(xyz2, xyz) and np.allclose(q2, q)

    class KF:
        def __init__(self, i):
            self.frame_id = i
            self.T_WC = PoseBatch(torch.tensor([[xyz[i][0], xyz[i][1], xyz[i][2], 0, 0, 0, 1, 2.0]]))

    frames = [KF(i) for i in range(5)]
    out = tmp_path / "traj.txt"
    ev.save_traj(str(out), t, frames)
    t3, xyz3, q3 = ev.read_tum(str(out))
    assert np.allclose(xyz3, xyz, atol=1e-6) and np.allclose(q3, q)
