"""Tracker oracle (oracle/track_oracle.py) pinned on CPU: against fixtures produced by the
REFERENCE tracker code (tests/golden/make_track_golden.py -> track_golden.npz), against the
C oracle's Sim3 exponential (the backend's expSim3 restatement), by finite differences of its
Jacobians, and by known-answer convergence to the generating relative pose."""
import os

import numpy as np
import pytest

from oracle import track_oracle as TO

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "track_golden.npz"))
CFG = TO.TRACKING_CFG


def _case(c):
    return {k[len(f"c{c}_"):]: GOLD[k] for k in GOLD.files if k.startswith(f"c{c}_")}


def _run_oracle(g):
    if str(g["mode"]) == "rays":
        return TO.opt_pose_ray_dist_sim3(g["Xf"], g["Xk"], g["T_WCf"], g["T_WCk"], g["Qk"],
                                         g["valid"], CFG)
    return TO.opt_pose_calib_sim3(g["Xf"], g["T_WCf"], g["T_WCk"], g["Qk"], g["valid"],
                                  g["meas_k"], g["valid_meas_k"], g["K"], (24, 32), CFG)


@pytest.mark.parametrize("c", range(4))
def test_oracle_matches_reference_tracker(c):
    """tracker.py:173-266 run as written (f32 torch, stub lietorch group) vs the f64 oracle."""
    g = _case(c)
    Tf, Tr, it, _ = _run_oracle(g)
    np.testing.assert_allclose(Tf, g["out_T_WCf"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(Tr, g["out_T_CkCf"], rtol=0, atol=1e-5)


def test_sim3_exp_matches_c_oracle(oracle):
    rng = np.random.default_rng(0)
    for scale in (1e-8, 1e-4, 0.1, 1.0):
        for _ in range(20):
            xi = rng.normal(0, scale, 7)
            t, q, s = oracle.exp_sim3(xi.astype(np.float32))
            e = TO.sim3_exp(xi.astype(np.float32).astype(np.float64))
            np.testing.assert_allclose(e, np.concatenate([t, q, [s]]), rtol=0, atol=2e-5 * max(1.0, scale))  # f32 C oracle: trig + cancellation in B


def test_sim3_group_laws():
    rng = np.random.default_rng(1)
    T = TO.sim3_exp(rng.normal(0, 0.3, 7))
    U = TO.sim3_exp(rng.normal(0, 0.3, 7))
    p = rng.normal(0, 1, (5, 3))
    np.testing.assert_allclose(TO.sim3_act(TO.sim3_mul(T, U), p), TO.sim3_act(T, TO.sim3_act(U, p)), atol=1e-12)
    np.testing.assert_allclose(TO.sim3_act(TO.sim3_inv(T), TO.sim3_act(T, p)), p, atol=1e-12)
    np.testing.assert_allclose(TO.sim3_retr(T, np.zeros(7)), T, atol=1e-15)


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_jacobian_matches_finite_differences(mode):
    """J = -(dh/dX)[I | -skew(X) | X] is the derivative of the residual under T <- Exp(d) T."""
    p = TO.make_tracking_pair((6, 8), seed=5, mode=mode, noise=0.01)
    T = TO.sim3_mul(TO.sim3_inv(p["T_WCk"].astype(np.float64)), p["T_WCf"].astype(np.float64))
    Xf, K = p["Xf"].astype(np.float64), p["K"].astype(np.float64)

    def res(Tx):
        X = TO.sim3_act(Tx, Xf)
        if mode == "rays":
            return TO.point_to_ray_dist(p["Xk"].astype(np.float64)) - TO.point_to_ray_dist(X)
        pz, _, _ = TO.project_calib(X, K, (6, 8), -10, 1e-6)
        return p["meas_k"].astype(np.float64) - pz

    X = TO.sim3_act(T, Xf)
    if mode == "rays":
        _, D = TO.point_to_ray_dist(X, jacobian=True)
    else:
        _, D, _ = TO.project_calib(X, K, (6, 8), -10, 1e-6)
    J = -D @ TO.act_jac(X)
    h = 1e-6
    for k in range(7):
        e = np.zeros(7)
        e[k] = h
        fd = (res(TO.sim3_retr(T, e)) - res(TO.sim3_retr(T, -e))) / (2 * h)
        np.testing.assert_allclose(J[..., k], fd, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_noise_free_pair_converges_to_truth(mode):
    p = TO.make_tracking_pair((24, 32), seed=7, mode=mode)
    cfg = dict(CFG, rel_error=0.0, delta_norm=1e-12)
    if mode == "rays":
        Tf, _, it, _ = TO.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"], cfg, max_iters=8)
    else:
        Tf, _, it, _ = TO.opt_pose_calib_sim3(p["Xf"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"], p["meas_k"],
                                              p["valid_meas_k"], p["K"], (24, 32), cfg, max_iters=8)
    np.testing.assert_allclose(Tf, p["T_WCf_true"], rtol=0, atol=2e-6)


def test_singular_system_raises():
    p = TO.make_tracking_pair((6, 8), seed=2)
    with pytest.raises(np.linalg.LinAlgError):
        TO.opt_pose_ray_dist_sim3(p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"],
                                  np.zeros_like(p["valid"]), CFG)
