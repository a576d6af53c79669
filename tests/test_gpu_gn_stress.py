"""GN parity OFF the fixed point (VERDICT r02 "what's weak" 2 / "next" 2).

The bench graphs start 0.5 deg / 1 cm from the truth with outlier-free projective matches, so
after 10 iterations both the op and the oracle sit on the same fixed point and a 1e-5 agreement
says little about the per-iteration arithmetic.  Here the headline topology (cfg3: 128 keyframes,
256 pair edges incl. 129 loop closures, gauss_newton_calib, full 512x384) starts 10 deg / 25 cm /
0.1 log-scale away and 10 % of every edge's valid matches are gross outliers (a random pixel), so
the Huber weights, the image-border and depth validity and Q < Q_thresh are all active, and the
graph is not converged after 10 iterations (checked: the 10th iteration still moves the poses by
more than the 1e-5 tolerance).

Asserted after 1, 3 and 10 iterations, against the CPU oracle (the reference backend restated,
its fp32 chains in the reference kernels' order, the reference build's FMA contraction):
  * the default (fast) path within its MEASURED distance from the oracle plus a 1.5x margin
    (MEASURED_D_ORACLE; measured on MI355X, re-measured in round 6 -- the op
    is deterministic, so the distance only moves when its summation order or formulas change),
    and within 1e-5 of the exactly summed system.  sigma = the oracle's own distance from the
    same float terms summed in double (the reference order's rounding noise) is printed beside
    it: the fast path sums in another order, so it cannot land closer than ~sigma to the oracle
    (measured: 1 iteration 2.1e-5 from the oracle with sigma 2.05e-5, but 6.2e-6 from the exact
    sums -- closer to the exactly summed system than the reference order is);
  * the reference-order mode (gn_refacc.hip) within max(1e-6, sigma / 10) of the oracle: the
    same formulas in the same order, so what remains -- the f64 solve's summation order and an
    ulp of sin / cos / exp / log -- is orders of magnitude below the fp32 summation noise sigma
    measures; mid-convergence (3 iterations) the system amplifies any perturbation ~1e3-fold
    (sigma ~2e-4 there), hence the relative bound.
"""
import numpy as np
import pytest
import torch

from m3s import synth

pytestmark = pytest.mark.gpu

LOCAL = dict(sigma_pixel=1.0, sigma_depth=10.0, C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)
STRESS = dict(init_perturb=(10.0, 0.25, 0.1), outlier_frac=0.10)
# measured fast-path distance from the oracle (max relative pose error), MI355X, re-measured in
# round 6 (profiles/r06_pcg/w_pytest_stress.log): 1 iteration takes the unpacked accumulate (a
# call of fewer than 3 iterations does not pay for the pack -- see the timed-kernel test below),
# 3 and 10 the packed ray-constrained stream the bench times, 10 also the lagged-factor PCG from
# iteration 4
MEASURED_D_ORACLE = {1: 2.09e-5, 3: 2.37e-5, 10: 1.70e-6}
# the same for the kernel the bench times forced at every iteration count (M3S_GN_PACK=2),
# measured in round 6 (same log)
MEASURED_D_ORACLE_TIMED = {1: 2.04e-5, 3: 2.37e-5}


def _rel(a, b):
    return float(np.abs(a.astype(np.float64) - b).max() / np.abs(b).max())


@pytest.fixture(scope="module")
def stress_graph():
    from m3s.geometry import constrain_points_to_ray

    g = synth.make_graph("cfg3", **STRESS)
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    return g


def _gpu(backend, g, iters):
    L = LOCAL
    Twc = g.Twc.clone().cuda()
    c = lambda t: t.cuda()
    backend.gauss_newton_calib(Twc, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                               g.H, g.W, L["pixel_border"], L["depth_eps"], L["sigma_pixel"], L["sigma_depth"],
                               L["C_conf"], L["Q_conf"], iters, 0.0)
    torch.cuda.synchronize()
    return Twc.cpu().numpy()


_ORACLE_CACHE = {}


def _oracle(oracle, g, iters, exact=False):
    key = (iters, exact)
    if key not in _ORACLE_CACHE:
        _ORACLE_CACHE[key] = _oracle_run(oracle, g, iters, exact)
    return _ORACLE_CACHE[key]


def _oracle_run(oracle, g, iters, exact):
    L = LOCAL
    P = oracle.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], K=g.K.numpy(),
                           height=g.H, width=g.W, pixel_border=L["pixel_border"], z_eps=L["depth_eps"],
                           max_iter=iters, delta_thresh=0.0)
    arrs = [t.numpy() for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]
    if exact:
        with oracle.exact_sums():
            return oracle.gauss_newton(P, *arrs)[0]
    return oracle.gauss_newton(P, *arrs)[0]


def test_stress_graph_is_active_and_unconverged(oracle, stress_graph):
    """The stress is real: many points invalid (border / depth / Q / match), Huber down-weights
    many valid ones, and the 10th iteration still moves the poses."""
    g = stress_graph
    L = LOCAL
    P = oracle.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], K=g.K.numpy(),
                           height=g.H, width=g.W, pixel_border=L["pixel_border"], z_eps=L["depth_eps"])
    ie, je, _ = oracle.remap(g.ii.numpy(), g.jj.numpy())
    # the first 24 directed edges (the residual model only; enough to show the regimes)
    sl = slice(0, 24)
    _, err, w, valid = oracle.gn_residuals(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), ie[sl], je[sl],
                                           g.idx[sl].numpy(), g.valid[sl].numpy(), g.Q[sl].numpy())
    full = (np.float32(1.0) * np.sqrt(g.Q[sl, :, 0].numpy())) ** 2
    assert 0.5 < valid.mean() < 0.95, valid.mean()
    huber_active = (w[..., 0] < 0.999 * full) & valid
    assert huber_active.mean() > 0.05, huber_active.mean()
    T9 = _oracle(oracle, g, 9)
    T10 = _oracle(oracle, g, 10)
    assert _rel(T10, T9) > 1e-5  # not converged: the 10th step still exceeds the tolerance
    assert np.abs(T10 - g.Twc_gt.numpy()).max() > 1e-2


@pytest.mark.parametrize("iters", [1, 3, 10])
def test_stress_graph_default_path_within_tolerance_of_oracle(backend, oracle, stress_graph, iters):
    g = stress_graph
    T_g = _gpu(backend, g, iters)
    T_o = _oracle(oracle, g, iters)
    T_x = _oracle(oracle, g, iters, exact=True)
    sigma = _rel(T_o, T_x)
    d_o, d_x = _rel(T_g, T_o), _rel(T_g, T_x)
    print(f"stress iters={iters}: fast vs oracle {d_o:.2e}, fast vs exact {d_x:.2e}, sigma {sigma:.2e}")
    assert np.isfinite(T_g).all()
    assert d_o <= 1.5 * MEASURED_D_ORACLE[iters], (d_o, sigma)
    assert d_x <= 1e-5, d_x


@pytest.mark.parametrize("iters", [1, 3])
def test_stress_graph_timed_kernel_within_tolerance_of_oracle(backend, oracle, stress_graph, monkeypatch, iters):
    """The bench's timed accumulate (gn_accum_packed_kernel, ray-constrained calib) priced
    mid-convergence: a 1-iteration call normally takes the unpacked accumulate (no reuse to pay
    for the pack), so M3S_GN_PACK=2 forces the timed kernel; measured 2.04e-5
    from the oracle (sigma 2.05e-5) and 5.9e-6 from the exactly summed system."""
    g = stress_graph
    monkeypatch.setenv("M3S_GN_PACK", "2")
    monkeypatch.setenv("M3S_GN_DEBUG_FLAGS", "2")
    T_g = _gpu(backend, g, iters)
    st = backend.gn_debug_flags()
    monkeypatch.delenv("M3S_GN_PACK")
    monkeypatch.delenv("M3S_GN_DEBUG_FLAGS")
    assert st["packed"] and st["ray_constrained"], st
    T_o = _oracle(oracle, g, iters)
    T_x = _oracle(oracle, g, iters, exact=True)
    sigma = _rel(T_o, T_x)
    d_o, d_x = _rel(T_g, T_o), _rel(T_g, T_x)
    print(f"stress iters={iters}: timed kernel vs oracle {d_o:.2e}, vs exact {d_x:.2e}, sigma {sigma:.2e}")
    assert np.isfinite(T_g).all()
    assert d_o <= 1.5 * MEASURED_D_ORACLE_TIMED[iters], (d_o, sigma)
    assert d_x <= 1e-5, d_x


@pytest.mark.parametrize("iters", [1, 3, 10])
def test_stress_graph_reference_order_within_1e6_of_oracle(backend, oracle, stress_graph, iters):
    g = stress_graph
    prev = backend.set_gn_order("reference")
    try:
        T_g = _gpu(backend, g, iters)
    finally:
        backend.set_gn_order(prev)
    T_o = _oracle(oracle, g, iters)
    sigma = _rel(T_o, _oracle(oracle, g, iters, exact=True))
    d = _rel(T_g, T_o)
    print(f"stress iters={iters}: reference order vs oracle {d:.2e} (sigma {sigma:.2e})")
    assert d <= max(1e-6, 0.1 * sigma), (d, sigma)
