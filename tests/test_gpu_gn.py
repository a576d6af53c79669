"""GPU parity of the Gauss-Newton ops against the CPU oracle.

Tolerances (north_star): poses within 1e-5 relative in fp32.  The normal equations of one
iteration are compared at 1e-4 relative to the matrix scale: the reference and the HIP
path sum ~10^5 fp32 terms per entry in different orders (the HIP path accumulates the
pre-adjoint Jacobian and applies the adjoint in f64), so entries agree to ~1e-6 of the
largest entry; the solved pose updates then agree far below the 1e-5 pose tolerance.
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

from m3s import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

LOCAL = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0,
             sigma_point=0.05, C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)


def _params(oracle, g, mode, iters, delta=0.0):
    L = LOCAL
    if mode == "rays":
        return oracle.make_params("rays", L["sigma_ray"], L["sigma_dist"], L["C_conf"], L["Q_conf"],
                                  max_iter=iters, delta_thresh=delta)
    if mode == "points":
        return oracle.make_params("points", L["sigma_point"], 0.0, L["C_conf"], L["Q_conf"],
                                  max_iter=iters, delta_thresh=delta)
    return oracle.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"],
                              K=g.K.numpy(), height=g.H, width=g.W, pixel_border=L["pixel_border"],
                              z_eps=L["depth_eps"], max_iter=iters, delta_thresh=delta)


def _run_gpu(backend, g, mode, iters, delta=0.0):
    L = LOCAL
    Twc = g.Twc.clone().cuda()
    c = lambda t: t.cuda()
    if mode == "rays":
        (dx,) = backend.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid),
                                          c(g.Q), L["sigma_ray"], L["sigma_dist"], L["C_conf"],
                                          L["Q_conf"], iters, delta)
    elif mode == "points":
        (dx,) = backend.gauss_newton_points(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx),
                                            c(g.valid), c(g.Q), L["sigma_point"], L["C_conf"],
                                            L["Q_conf"], iters, delta)
    else:
        (dx,) = backend.gauss_newton_calib(Twc, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx),
                                           c(g.valid), c(g.Q), g.H, g.W, L["pixel_border"],
                                           L["depth_eps"], L["sigma_pixel"], L["sigma_depth"],
                                           L["C_conf"], L["Q_conf"], iters, delta)
    torch.cuda.synchronize()
    return Twc.cpu().numpy(), (dx.cpu().numpy() if dx is not None else None)


def _run_oracle(oracle, g, mode, iters, delta=0.0):
    P = _params(oracle, g, mode, iters, delta)
    Twc, dx, it = oracle.gauss_newton(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                                      g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
    return Twc, dx, it


def _rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-12)


def _graph(mode, N=6, E=8, H=48, W=64, seed=5):
    if mode == "calib":
        g = synth.make_graph(dict(N=N, E=E), H=H, W=W, seed=seed)
        from m3s.geometry import constrain_points_to_ray

        g.Xs = constrain_points_to_ray((H, W), g.Xs, g.K).contiguous()
        return g
    return synth.make_graph(dict(N=N, E=E), H=H, W=W, seed=seed)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_normal_equations_match_oracle(backend, oracle, mode):
    from m3s.debug import build_system_gpu

    g = _graph(mode)
    P = _params(oracle, g, mode, 1)
    H_o, b_o = oracle.gn_build_system(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                                      g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
    H_g, b_g = build_system_gpu(g, mode, LOCAL)
    scale = np.abs(H_o).max()
    assert np.abs(H_g - H_o).max() / scale < 1e-4
    assert np.abs(b_g - b_o).max() / max(np.abs(b_o).max(), 1e-30) < 1e-4
    # the solved updates: 2e-5 of the largest component.  Both sides sum ~10^4 fp32 terms per
    # entry in different orders (the oracle reproduces the reference's 768-long serial
    # per-thread chains, the HIP path 32-long chains + f64 chunk sums), and calib's
    # ill-conditioned scale/depth rows amplify that ~1e-6 relative noise in b to ~1e-5 in x.
    # The north_star pose tolerance (1e-5) is checked after full GN iterations below.
    x_o = np.linalg.solve(H_o, b_o)
    x_g = np.linalg.solve(H_g, b_g)
    assert np.abs(x_g - x_o).max() < 2e-5 * max(np.abs(x_o).max(), 1e-3)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_gauss_newton_matches_oracle(backend, oracle, mode):
    g = _graph(mode)
    iters = 5 if mode != "calib" else 3
    T_g, dx_g = _run_gpu(backend, g, mode, iters)
    T_o, dx_o, _ = _run_oracle(oracle, g, mode, iters)
    assert np.isfinite(T_g).all()
    assert _rel(T_g, T_o) < 1e-5, _rel(T_g, T_o)
    assert np.abs(dx_g - dx_o).max() < 1e-5 * max(np.abs(T_o).max(), 1.0)


def test_known_answer_converges_to_gt(backend):
    g = synth.make_consistent_graph(N=5, H=24, W=32, seed=2)
    T_g, _ = _run_gpu(backend, g, "rays", 10)
    assert np.abs(T_g - g.Twc_gt.numpy()).max() < 2e-5
    T_p, _ = _run_gpu(backend, g, "points", 10)
    assert np.abs(T_p - g.Twc_gt.numpy()).max() < 2e-5


def test_early_exit_and_return(backend, oracle):
    g = synth.make_consistent_graph(N=4, H=24, W=32, seed=1)
    # a huge delta_thresh stops after the first iteration, like the reference's `break`
    T_g, dx_g = _run_gpu(backend, g, "rays", 10, delta=1e9)
    T_o, dx_o, it = _run_oracle(oracle, g, "rays", 10, delta=1e9)
    assert it == 1
    assert _rel(T_g, T_o) < 1e-5
    # max_iter = 0: no update, undefined return
    T0, dx0 = _run_gpu(backend, g, "rays", 0)
    assert dx0 is None and np.array_equal(T0, g.Twc.numpy())


def test_singular_system_gives_zero_update(backend, oracle):
    """A pose with no valid observation makes the system singular: SimplicialLLT fails,
    dx = 0 and the loop exits (gn_kernels.cu:142-150, 1219-1222)."""
    g = _graph("rays", N=4, E=3)
    g.valid[:] = False
    T_g, dx_g = _run_gpu(backend, g, "rays", 10, delta=1e-8)
    T_o, dx_o, it = _run_oracle(oracle, g, "rays", 10, delta=1e-8)
    assert it == 1
    assert np.array_equal(T_g, g.Twc.numpy()) and np.array_equal(T_o, g.Twc.numpy())
    assert np.all(dx_g == 0)


def test_sparse_global_ids_and_determinism(backend):
    g = _graph("rays", N=5, E=6)
    ids = torch.tensor([2, 7, 8, 20, 31])
    g2 = synth.Graph(**{**g.__dict__, "ii": ids[g.ii], "jj": ids[g.jj]})
    T1, _ = _run_gpu(backend, g, "rays", 4)
    T2, _ = _run_gpu(backend, g2, "rays", 4)
    T3, _ = _run_gpu(backend, g2, "rays", 4)
    assert np.array_equal(T1, T2) and np.array_equal(T2, T3)


def test_edge_shards_sum_to_full_system(backend):
    """Edge sharding (multi-GPU path) without RCCL: the compact systems of two edge
    ranges add up to the full system."""
    from m3s.debug import build_system_gpu

    g = _graph("rays", N=6, E=8)
    H_full, b_full = build_system_gpu(g, "rays", LOCAL)
    E2 = g.ii.shape[0]
    parts = [build_system_gpu(g, "rays", LOCAL, edge_range=r) for r in ((0, 5), (5, E2))]
    Hs = parts[0][0] + parts[1][0]
    bs = parts[0][1] + parts[1][1]
    assert np.abs(Hs - H_full).max() <= 1e-9 * np.abs(H_full).max()
    assert np.abs(bs - b_full).max() <= 1e-9 * np.abs(b_full).max()


def test_full_size_cfg2_matches_oracle(backend, oracle):
    """BASELINE size 512x384, cfg2 topology (33 keyframes, 128 directed edges): HIP vs the
    oracle after 2 iterations, plus determinism of two GPU runs."""
    g = synth.make_graph("cfg2")
    T1, dx1 = _run_gpu(backend, g, "rays", 2)
    T2, dx2 = _run_gpu(backend, g, "rays", 2)
    assert np.isfinite(T1).all() and np.array_equal(T1, T2)
    T_o, dx_o, _ = _run_oracle(oracle, g, "rays", 2)
    assert _rel(T1, T_o) < 1e-5, _rel(T1, T_o)


@pytest.mark.parametrize("solver", ["1", "2", "3"])
@pytest.mark.parametrize("topo", ["cfg3", "cfg4", "chain", "star", "clique", "clique27", "clique28",
                                  "clique4", "clique8", "clique17", "clique21", "hub"])
def test_sparse_elimination_matches_dense_solver(backend, monkeypatch, topo, solver):
    """The block-sparse solvers against the dense blocked Cholesky (M3S_SOLVER_DENSE=1) on the
    same system: one GN step, f64 solves of the same matrix in different orders -> updates
    agree to ~1e-9 relative.  M3S_SOLVER=1: the single-workgroup solve (gn_solve.hip; graphs
    whose tail does not fit it fall back to 2), 2: one launch per elimination round
    (gn_sparse.hip) + tiled dense core, 3: the same rounds + gn_solve's in-register core,
    back-substitution and retraction (falls back to 2 when the core does not fit).  Topologies
    cover the BASELINE graphs, a chain (everything eliminated in rounds), a star around the
    pinned pose (poses without fronts) and cliques (no independent low-degree set: dense tail
    only; 27 non-pinned poses = the largest in-register tail, 189 unknowns in 12 x 12 tiles of
    16x16; 28 = beyond it; 3 / 7 / 11 / 16 / 20 poses: tails of 2 / 4 / 6 / 8 / 10 tile rows, so
    every instantiated tile map -- dealt to the waves by MFMA work -- is exercised).  "hub": 20
    poses each linked to the same two hubs, eliminated in one round, so the hub pair's block
    target and both hubs' RHS targets take 20 contributions -- past a round record's 9 inline
    ones (sparse_plan.h: the rest from the overflow lists)."""
    if topo == "hub":
        N = 23
        und = [(0, 1), (1, 2)] + [(h, k) for k in range(3, N) for h in (1, 2)]
    elif topo == "chain":
        N = 24
        und = [(k - 1, k) for k in range(1, N)]
    elif topo == "star":
        N = 6
        und = [(0, k) for k in range(1, N)]
    elif topo.startswith("clique"):
        N = {"clique": 12, "clique27": 28, "clique28": 29, "clique4": 4, "clique8": 8, "clique17": 17,
             "clique21": 21}[topo]
        und = [(a, b) for a in range(N) for b in range(a + 1, N)]
    if topo in ("chain", "star", "hub") or topo.startswith("clique"):
        g = synth.make_graph(dict(N=N, E=len(und)), H=24, W=32, seed=3, edges_only=und)
    else:
        g = synth.make_graph(topo, H=24, W=32, seed=6)
    monkeypatch.setenv("M3S_SOLVER_DENSE", "1")
    T_d, dx_d = _run_gpu(backend, g, "rays", 1)
    monkeypatch.delenv("M3S_SOLVER_DENSE")
    monkeypatch.setenv("M3S_SOLVER", solver)
    T_s, dx_s = _run_gpu(backend, g, "rays", 1)
    assert np.isfinite(dx_s).all()
    assert np.abs(dx_s - dx_d).max() <= 1e-8 * max(np.abs(dx_d).max(), 1e-6)
    assert _rel(T_s, T_d) < 1e-6


@pytest.mark.parametrize("solver", ["1", "3"])
@pytest.mark.parametrize("cfg", ["cfg2", "cfg3"])
def test_single_workgroup_solve_matches_multilaunch(backend, monkeypatch, cfg, solver):
    """The single-workgroup solve (M3S_SOLVER=1: rounds, in-register tail, back-substitution and
    retraction in one launch) and the hybrid (3: one launch per round, then the in-register
    core + back-substitution + retraction in one launch) against the multi-launch solve
    (M3S_SOLVER=2) over 3 GN iterations: the same f64 elimination in different orders ->
    updates agree to ~1e-9."""
    g = synth.make_graph(cfg, H=24, W=32, seed=6)
    monkeypatch.setenv("M3S_SOLVER", "2")
    T_m, dx_m = _run_gpu(backend, g, "rays", 3)
    monkeypatch.setenv("M3S_SOLVER", solver)
    T_f, dx_f = _run_gpu(backend, g, "rays", 3)
    assert np.isfinite(dx_f).all()
    assert np.abs(dx_f - dx_m).max() <= 1e-8 * max(np.abs(dx_m).max(), 1e-6)
    assert _rel(T_f, T_m) < 1e-6


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_packed_stream_gives_identical_system(backend, monkeypatch, mode):
    """The per-call packed stream (gn_pack_kernel: {match index | invalid bit, sqrt q}, plus the
    calib depth array) feeds the same point math as the direct path, so the normal equations
    are bitwise identical (M3S_GN_PACK=2 forces the packed path, 0 disables it)."""
    from m3s.debug import build_system_gpu

    g = _graph(mode, N=5, E=6)
    g.Q[0, :50] = 1.0            # below Q_thresh: folded into the invalid bit
    g.valid[1, 10:90] = False    # unmatched: index 0, weight 0
    monkeypatch.setenv("M3S_GN_PACK", "0")
    H0, b0 = build_system_gpu(g, mode, LOCAL)
    monkeypatch.setenv("M3S_GN_PACK", "2")
    monkeypatch.setenv("M3S_GN_COMPACT", "0")  # the positional stream: same points, same order
    monkeypatch.setenv("M3S_GN_RAYCHECK", "0")  # (calib: Xj read whole, not rebuilt from its depth)
    H2, b2 = build_system_gpu(g, mode, LOCAL)
    assert np.array_equal(H0, H2) and np.array_equal(b0, b2)
    if mode == "calib":  # the ray-constrained stream: the same terms up to the transform's rounding
        monkeypatch.setenv("M3S_GN_RAYCHECK", "1")
        H4, b4 = build_system_gpu(g, mode, LOCAL)
        assert np.abs(H4 - H0).max() <= 1e-5 * np.abs(H0).max()
        assert np.abs(b4 - b0).max() <= 1e-5 * np.abs(b0).max()
    # the compacted stream (M3S_GN_COMPACT=1): dead points dropped, so only the summation
    # grouping moves
    monkeypatch.setenv("M3S_GN_COMPACT", "1")
    H3, b3 = build_system_gpu(g, mode, LOCAL)
    assert np.abs(H3 - H0).max() <= 1e-6 * np.abs(H0).max()
    assert np.abs(b3 - b0).max() <= 1e-6 * np.abs(b0).max()


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_confidence_pass_skips_only_passing_keyframes(backend, monkeypatch, mode):
    """The pack skips the Cj reads / Ci gathers of an edge whose two keyframes have every
    confidence above C_thresh (gn_cpass_kernel, one pass over N x HW): with C_thresh = 1.5,
    keyframes that pass wholly, keyframes with some confidences at or below it, and one with a
    NaN confidence (which fails c > C_thresh like the reference), the packed system is bitwise
    the direct path's, which tests every point."""
    from m3s.debug import build_system_gpu

    g = _graph(mode, N=6, E=8)
    Lc = dict(LOCAL, C_conf=1.5)
    Cs = g.Cs.clone()
    Cs[0] = Cs[0].clamp(min=1.6)          # passes wholly
    Cs[1] = Cs[1].clamp(min=1.6)
    Cs[2, 5:40] = 1.5                     # at the threshold: fails (strict >)
    Cs[3] = Cs[3].clamp(min=1.6)
    Cs[3, 17] = float("nan")              # fails
    Cs[4, ::7] = 0.5
    g.Cs = Cs.contiguous()
    monkeypatch.setenv("M3S_GN_PACK", "0")
    H0, b0 = build_system_gpu(g, mode, Lc)
    monkeypatch.setenv("M3S_GN_PACK", "2")
    monkeypatch.setenv("M3S_GN_COMPACT", "0")
    monkeypatch.setenv("M3S_GN_RAYCHECK", "0")  # positional Xj: bitwise the direct path's terms
    H2, b2 = build_system_gpu(g, mode, Lc)
    assert np.array_equal(H0, H2, equal_nan=True) and np.array_equal(b0, b2, equal_nan=True)


@pytest.mark.parametrize("mode,ray_constrained", [("calib", True), ("calib", False), ("rays", False),
                                                  ("points", False)])
def test_first_iteration_builds_the_packed_records(backend, monkeypatch, mode, ray_constrained):
    """A call's first accumulate builds the packed records from the reference's inputs
    (M3S_GN_PACK_FIRST=1, default) instead of a separate pack pass: the same records, so the
    poses and dx after 3 iterations are bitwise those of the separate pass -- with confidences
    at / below C_thresh, a NaN confidence, Q below Q_thresh and unmatched points; calib on both
    the ray-constrained (depth-only Xj) and the positional stream, rays and points (2 points per
    lane and step)."""
    g = _graph("calib", N=6, E=8)
    if not ray_constrained:
        g.Xs = (g.Xs * 1.0001).contiguous()  # off the rays: the positional stream
    Cs = g.Cs.clone()
    Cs[0] = Cs[0].clamp(min=1.6)
    Cs[2, 5:40] = 1.5
    Cs[3, 17] = float("nan")
    g.Cs = Cs.contiguous()
    g.Q[0, :50] = 1.0
    g.valid[1, 10:90] = False
    Lc = dict(LOCAL, C_conf=1.5)
    out = []
    for first in ("0", "1"):
        monkeypatch.setenv("M3S_GN_PACK_FIRST", first)
        Twc = g.Twc.clone().cuda()
        c = lambda t: t.cuda()
        if mode == "calib":
            (dx,) = backend.gauss_newton_calib(Twc, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx),
                                               c(g.valid), c(g.Q), g.H, g.W, Lc["pixel_border"],
                                               Lc["depth_eps"], Lc["sigma_pixel"], Lc["sigma_depth"],
                                               Lc["C_conf"], Lc["Q_conf"], 3, 0.0)
        elif mode == "rays":
            (dx,) = backend.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid),
                                              c(g.Q), Lc["sigma_ray"], Lc["sigma_dist"], Lc["C_conf"],
                                              Lc["Q_conf"], 3, 0.0)
        else:
            (dx,) = backend.gauss_newton_points(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx),
                                                c(g.valid), c(g.Q), Lc["sigma_point"], Lc["C_conf"],
                                                Lc["Q_conf"], 3, 0.0)
        torch.cuda.synchronize()
        out.append((Twc.cpu().numpy(), dx.cpu().numpy()))
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1], equal_nan=True)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_compacted_stream_keeps_nan_poisoning_and_empty_edges(backend, oracle, monkeypatch, mode):
    """Dead-point compaction (gn_pack_compact_kernel) drops a point only when its validity fails
    AND its own and its matched point are finite (then its contribution is exactly 0): a NaN
    in an invalid point must still poison the system as in the reference; an edge with no live
    point contributes nothing; and the iterated result equals the positional stream's to
    rounding and the oracle to 1e-5."""
    from m3s.debug import build_system_gpu

    monkeypatch.setenv("M3S_GN_PACK", "2")
    monkeypatch.setenv("M3S_GN_COMPACT", "1")
    g = _graph(mode, N=5, E=6)
    g.valid[2, :] = False        # one directed edge with no live point at all
    T_c, _ = _run_gpu(backend, g, mode, 3)
    monkeypatch.setenv("M3S_GN_COMPACT", "0")
    T_p, _ = _run_gpu(backend, g, mode, 3)
    monkeypatch.setenv("M3S_GN_COMPACT", "1")
    T_o, _, _ = _run_oracle(oracle, g, mode, 3)
    assert np.isfinite(T_c).all()
    assert _rel(T_c, T_p) < 1e-6 and _rel(T_c, T_o) < 1e-5
    # an invalid point with a NaN coordinate, read by no valid point: kept, and it poisons like
    # the reference's 0 * NaN
    j = int(g.jj[3])
    g.valid[g.jj == j, 5] = False                          # every edge that reads it as Xj
    g.valid[(g.ii == j)[:, None] & (g.idx == 5)] = False   # no valid point gathers it as Xi
    g.Xs[j, 5, 0] = float("nan")
    H, b = build_system_gpu(g, mode, LOCAL)
    monkeypatch.setenv("M3S_GN_COMPACT", "0")
    H_p, b_p = build_system_gpu(g, mode, LOCAL)
    assert np.isnan(H).any() and np.array_equal(np.isnan(H), np.isnan(H_p))


def test_full_size_cfg3_calib_step_closer_to_exactly_summed_system(backend, oracle):
    """BASELINE's graph (cfg3: 128 keyframes, 256 pairs, 512x384, calib), one iteration.
    Summation order matters at this size: the reference's float order (the oracle mirrors it,
    gn_kernels.cu:31-55) puts the first step 2.4e-3 (of max |dx|) from the step obtained when
    the same float terms are summed in double; the HIP path (f32 lane partials over short
    chunks, f64 across workgroups) must land closer to that exactly summed step than the
    reference order does (measured: 6e-5), and its poses are the oracle's retraction of its
    own step, bit for bit (poses after ONE step are not compared across different steps:
    see test_cfg4_full_size_one_and_ten_iterations)."""
    g = synth.make_graph("cfg3")
    from m3s.geometry import constrain_points_to_ray

    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    T_gpu, dx_gpu = _run_gpu(backend, g, "calib", 1)
    _, dx_ref, _ = _run_oracle(oracle, g, "calib", 1)
    with oracle.exact_sums():
        _, dx_x, _ = _run_oracle(oracle, g, "calib", 1)
    step = lambda d: float(np.abs(d.astype(np.float64) - dx_x).max() / np.abs(dx_x).max())
    print(f"cfg3 first step: op {step(dx_gpu):.2e}, reference order {step(dx_ref):.2e} (of max |dx|)")
    assert step(dx_gpu) <= step(dx_ref)
    assert step(dx_gpu) < 1e-3
    T0 = g.Twc.numpy()
    T_r = np.stack([T0[0]] + [oracle.retr_sim3(dx_gpu[i - 1], T0[i]) for i in range(1, T0.shape[0])])
    assert np.array_equal(T_gpu, T_r), _rel(T_gpu, T_r)


def _ray_path_taken(backend, g, iters, monkeypatch):
    """Run once more with the device flags read back: did the packed calib accumulate take the
    ray-constrained stream (Xj read as its depth)?"""
    import ctypes

    monkeypatch.setenv("M3S_GN_DEBUG_FLAGS", "2")
    _run_gpu(backend, g, "calib", iters)
    monkeypatch.delenv("M3S_GN_DEBUG_FLAGS")
    dbg = (ctypes.c_int * 4)()
    backend.lib.m3s_gn_debug_flags(dbg)
    return bool(dbg[3])


@pytest.mark.parametrize("iters", [3, 6])
def test_ray_constrained_calib_path(backend, oracle, monkeypatch, iters):
    """solve_GN_calib hands the op ray-constrained points (global_opt.py:172); the packed calib
    accumulate then reads Xj as its depth (gn_depth_kernel checks every point bit for bit) and
    applies T_ij to z (tu, tv, 1) factored per pixel row (M3S_RC_FACTOR), other roundings than
    the positional stream's s M x + t: both within 1e-5 of the oracle and of each other to float
    rounding.  The path must not be taken for unconstrained points (then the result is bitwise
    the positional stream's)."""
    from m3s.geometry import constrain_points_to_ray

    g = synth.make_graph("cfg2", H=96, W=128, mode="calib")
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    monkeypatch.setenv("M3S_GN_RAYCHECK", "1")
    T_rc, _ = _run_gpu(backend, g, "calib", iters)
    assert _ray_path_taken(backend, g, iters, monkeypatch)
    monkeypatch.setenv("M3S_GN_RAYCHECK", "0")
    T_gen, _ = _run_gpu(backend, g, "calib", iters)
    assert not _ray_path_taken(backend, g, iters, monkeypatch)
    monkeypatch.setenv("M3S_GN_RAYCHECK", "1")
    T_o, _, _ = _run_oracle(oracle, g, "calib", iters)
    assert _rel(T_rc, T_o) < 1e-5 and _rel(T_gen, T_o) < 1e-5, (_rel(T_rc, T_o), _rel(T_gen, T_o))
    assert _rel(T_rc, T_gen) < 2e-6, _rel(T_rc, T_gen)
    # one point off its ray: the check must fall back (result == generic path on those inputs)
    g.Xs[5, 77, 0] = torch.nextafter(g.Xs[5, 77, 0], torch.tensor(1e9))
    T_fb, _ = _run_gpu(backend, g, "calib", iters)
    assert not _ray_path_taken(backend, g, iters, monkeypatch)
    monkeypatch.setenv("M3S_GN_RAYCHECK", "0")
    T_fb_gen, _ = _run_gpu(backend, g, "calib", iters)
    assert np.array_equal(T_fb, T_fb_gen)


@pytest.mark.parametrize("W", [100, 102, 126])
def test_pixel_coded_calib_records_at_odd_widths(backend, oracle, monkeypatch, W):
    """The packed calib records carry the match as its pixel (v << 16 | u, decoded with a 24-bit
    multiply-add): at widths that are not powers of two, the packed call on positional Xj is
    bitwise the unpacked one (which decodes flat indices by division), and with W % 4 == 0 the
    ray-constrained stream (its own transform roundings) is within 1e-5 of the oracle too."""
    from m3s.geometry import constrain_points_to_ray

    g = synth.make_graph("cfg2", H=48, W=W, mode="calib")
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    monkeypatch.setenv("M3S_GN_RAYCHECK", "0")
    monkeypatch.setenv("M3S_GN_PACK", "2")
    T_p, _ = _run_gpu(backend, g, "calib", 3)
    monkeypatch.setenv("M3S_GN_RAYCHECK", "1")
    T_rc, _ = _run_gpu(backend, g, "calib", 3)
    monkeypatch.setenv("M3S_GN_PACK", "0")
    T_u, _ = _run_gpu(backend, g, "calib", 3)
    monkeypatch.setenv("M3S_GN_PACK", "1")
    assert np.array_equal(T_p, T_u)
    T_o, _, _ = _run_oracle(oracle, g, "calib", 3)
    assert np.abs(T_p - T_o).max() / np.abs(T_o).max() < 1e-5
    assert np.abs(T_rc - T_o).max() / np.abs(T_o).max() < 1e-5


def _cfg3_calib_graph():
    from m3s.geometry import constrain_points_to_ray

    g = synth.make_graph("cfg3")
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    return g


def test_cfg3_bench_graph_10_iterations_within_1e5_of_oracle(backend, oracle):
    """The headline workload exactly as bench.py times it (cfg3: 128 keyframes, 256 pairs incl.
    129 loop closures, 512x384, calib.yaml, max_iter = 10, delta_thresh = 0): the op's poses
    after all 10 iterations against the oracle's (the reference's float order,
    gn_kernels.cu:31-55, 1346-1543) at the north-star bar of 1e-5 relative.  The first
    iteration differs by the two summation orders' rounding (~8e-5, see the test above); at
    the GN fixed point only the gradient's rounding remains, ~2e-6 for both orders."""
    g = _cfg3_calib_graph()
    T_gpu, dx_gpu = _run_gpu(backend, g, "calib", 10)
    T_ref, dx_ref, it = _run_oracle(oracle, g, "calib", 10)
    assert it == 10
    assert np.isfinite(T_gpu).all()
    assert _rel(T_gpu, T_ref) < 1e-5, _rel(T_gpu, T_ref)
    # converged: the last update is tiny on both sides
    assert np.abs(dx_gpu).max() < 1e-4 and np.abs(dx_ref).max() < 1e-4


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_cfg1_keyframe_pair_matches_oracle(backend, oracle, mode):
    """BASELINE config 1: one keyframe pair (N=2, E=1, 2 directed edges) at 512x384, 5 GN
    iterations -- the smallest graph (a single 7-unknown system, pose 0 pinned)."""
    g = synth.make_graph("cfg1", mode=mode)
    if mode == "calib":
        from m3s.geometry import constrain_points_to_ray

        g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    T_g, dx_g = _run_gpu(backend, g, mode, 5)
    T_o, dx_o, it = _run_oracle(oracle, g, mode, 5)
    assert it == 5 and np.isfinite(T_g).all()
    assert _rel(T_g, T_o) < 1e-5, _rel(T_g, T_o)
    assert np.array_equal(T_g[0], g.Twc[0].numpy())  # pinned
    assert np.abs(dx_g - dx_o).max() < 1e-5 * max(np.abs(T_o).max(), 1.0)


@pytest.mark.timeout(600)
def test_cfg4_full_size_one_and_ten_iterations(backend, oracle):
    """BASELINE config 4 at full size on one GPU (256 keyframes, 1024 pairs = 2048 directed
    edges, 512x384, gauss_newton_rays).

    One iteration, split into its two stages:
      * the step dx (accumulate + solve): at this size it is only determined to the fp32
        rounding of its ~4e8 summed terms -- sigma = the distance of the oracle's step (the
        reference order) from the step of the same float terms summed in double (1.7e-4 of
        max |dx| on this graph) -- so the op's step must lie within max(1e-5, 4 sigma) of the
        exactly summed one (measured: 2e-5, eight times closer than the reference order);
      * the retraction: the op's poses are the oracle's retraction of the op's own step, bit
        for bit (sim3.h; both evaluate the Sim(3) exponential's transcendentals correctly
        rounded).  Poses after one step are NOT compared across different steps: the
        reference's float exponential turns a 1e-7 change of the log-scale into a ~1e-5 change
        of the translation ((expf(sigma) - 1) / sigma at sigma ~ 1e-5), whichever side is right.
    Ten iterations (the timed call): within the north-star 1e-5 of the oracle, finite,
    deterministic (two runs bitwise equal), converging."""
    g = synth.make_graph("cfg4")
    T1, dx1 = _run_gpu(backend, g, "rays", 1)
    _, dx_o, _ = _run_oracle(oracle, g, "rays", 1)
    with oracle.exact_sums():
        _, dx_x, _ = _run_oracle(oracle, g, "rays", 1)
    step = lambda d: float(np.abs(d.astype(np.float64) - dx_x).max() / np.abs(dx_x).max())
    bound = max(1e-5, 4 * step(dx_o))
    print(f"cfg4 first step: op {step(dx1):.2e}, reference order {step(dx_o):.2e} (of max |dx|)")
    assert step(dx1) < bound, (step(dx1), bound)
    T0 = g.Twc.numpy()
    T_r = np.stack([T0[0]] + [oracle.retr_sim3(dx1[i - 1], T0[i]) for i in range(1, T0.shape[0])])
    assert np.array_equal(T1, T_r), _rel(T1, T_r)
    Ta, dxa = _run_gpu(backend, g, "rays", 10)
    Tb, dxb = _run_gpu(backend, g, "rays", 10)
    assert np.isfinite(Ta).all() and np.array_equal(Ta, Tb) and np.array_equal(dxa, dxb)
    assert np.abs(dxa).max() < 1e-2 * np.abs(dx1).max()
    T10, _, it = _run_oracle(oracle, g, "rays", 10)
    assert it == 10
    assert _rel(Ta, T10) < 1e-5, _rel(Ta, T10)


@pytest.mark.parametrize("topo", ["cfg4", "cfg3", "clique28", "clique20", "clique12", "pair"])
@pytest.mark.parametrize("dense", [True, False])
def test_dataflow_factor_matches_multilaunch_factor(backend, monkeypatch, topo, dense):
    """The one-launch dataflow tile LL^T (chol_df.hip, default) against the per-panel
    potrf / trsm / update launches (M3S_CHOL_DF=0) on the same systems, 2 GN iterations: the
    same factorisation in a left- instead of right-looking summation order -> updates agree to
    ~1e-9.  dense=True factors the whole system (cfg4: 255 poses, 1785 unknowns in 28 tile
    columns = 434 tiles, more than one per workgroup); False the sparse solver's dense core
    (cfg4: 141 poses, 16 tile columns); the cliques 196 / 133 / 77 unknowns (4 / 3 / 2 tile
    columns); pair one
    tile column."""
    if topo.startswith("clique"):  # 28 / 19 / 11 free poses: 4 / 3 / 2 tile columns (dense)
        N = {"clique28": 29, "clique20": 20, "clique12": 12}[topo]
        und = [(a, b) for a in range(N) for b in range(a + 1, N)]
        g = synth.make_graph(dict(N=N, E=len(und)), H=24, W=32, seed=3, edges_only=und)
    elif topo == "pair":
        g = synth.make_graph(dict(N=2, E=1), H=24, W=32, seed=3, edges_only=[(0, 1)])
    else:
        g = synth.make_graph(topo, H=24, W=32, seed=6)
    if dense:
        monkeypatch.setenv("M3S_SOLVER_DENSE", "1")
    else:
        monkeypatch.setenv("M3S_SOLVER", "2")
    monkeypatch.setenv("M3S_CHOL_DF", "0")
    T_m, dx_m = _run_gpu(backend, g, "rays", 2)
    monkeypatch.setenv("M3S_CHOL_DF", "1")
    T_f, dx_f = _run_gpu(backend, g, "rays", 2)
    T_f2, _ = _run_gpu(backend, g, "rays", 2)
    assert np.isfinite(dx_f).all() and np.array_equal(T_f, T_f2)  # deterministic
    assert np.abs(dx_f - dx_m).max() <= 1e-8 * max(np.abs(dx_m).max(), 1e-6)
    assert _rel(T_f, T_m) < 1e-6


@pytest.mark.parametrize("chol_df", ["1", "0"])
@pytest.mark.parametrize("dense", [True, False])
def test_singular_core_fails_through_tile_factor(backend, monkeypatch, dense, chol_df):
    """SimplicialLLT's failure semantics (pivot <= 0 => dx = 0, loop exits;
    gn_kernels.cu:142-150, 1219-1222) through the tiled dense factorisations: a 29-keyframe
    clique (no low-degree elimination set: its 196-unknown core goes to the tile LL^T) with no
    valid observation.  dense=True factors the whole system, False the sparse solver's core;
    chol_df selects the dataflow launch or the per-panel launches."""
    N = 29
    und = [(a, b) for a in range(N) for b in range(a + 1, N)]
    g = synth.make_graph(dict(N=N, E=len(und)), H=24, W=32, seed=3, edges_only=und)
    g.valid[:] = False
    if dense:
        monkeypatch.setenv("M3S_SOLVER_DENSE", "1")
    else:
        monkeypatch.setenv("M3S_SOLVER", "2")
    monkeypatch.setenv("M3S_CHOL_DF", chol_df)
    T_g, dx_g = _run_gpu(backend, g, "rays", 10, delta=1e-8)
    assert np.array_equal(T_g, g.Twc.numpy())
    assert np.all(dx_g == 0)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_fused_edge_reduce_is_bitwise_the_separate_launch(backend, monkeypatch, mode):
    """The packed accumulate's last workgroup per edge runs the edge reduce (default) instead of
    gn_edge_reduce_kernel (M3S_GN_FUSE_REDUCE=0): the same f32 partials summed in chunk order,
    read back with agent-coherent loads from other workgroups / XCDs -> bitwise the same poses
    over 4 iterations (the per-edge counters are re-zeroed by the kernel between iterations)."""
    g = synth.make_graph("cfg3", H=48, W=64, seed=6)
    monkeypatch.setenv("M3S_GN_FUSE_REDUCE", "0")
    T_s, dx_s = _run_gpu(backend, g, mode, 4)
    monkeypatch.setenv("M3S_GN_FUSE_REDUCE", "1")
    T_f, dx_f = _run_gpu(backend, g, mode, 4)
    assert np.isfinite(T_f).all()
    assert np.array_equal(T_f, T_s) and np.array_equal(dx_f, dx_s)


def _solver_graph(monkeypatch, solver):
    """The graph and solver switches of the factorisation-robustness tests: the dense solver or
    the multi plan on a cfg4-topology graph, or the DEFAULT solver on a cfg3-topology graph (the
    hybrid plan, its core factored by chol_df)."""
    if solver == "hybrid":
        g = synth.make_graph("cfg3", H=24, W=32, seed=6)
        p = backend_plan(g)
        assert p["solver"] == "hybrid" and p["core_poses"] > 0, p
        return g
    g = synth.make_graph("cfg4", H=24, W=32, seed=6)
    if solver == "dense":
        monkeypatch.setenv("M3S_SOLVER_DENSE", "1")
    else:
        monkeypatch.setenv("M3S_SOLVER", "2")
    return g


def backend_plan(g):
    import mast3r_slam_backends as mb

    return mb.gn_plan_info(g.ii.tolist(), g.jj.tolist(), g.Twc.shape[0])


@pytest.mark.parametrize("solver", ["dense", "multi", "hybrid"])
def test_factorisation_timeout_is_an_error_not_a_singular_system(backend, monkeypatch, solver):
    """A bounded device-side wait of the dataflow factorisation that gives up (forced here with
    the test hook M3S_TEST_FORCE_TIMEOUT: every ready wait times out at once) raises
    RuntimeError (M3S_ERR_TIMEOUT) instead of passing for a singular system (dx = 0, early exit);
    the GPU drains normally and the next call without the hook is correct again.
    Also the default solver on a cfg3-sized graph (hybrid, chol_df core)."""
    g = _solver_graph(monkeypatch, solver)
    monkeypatch.setenv("M3S_CHOL_DF", "1")
    T_ok, dx_ok = _run_gpu(backend, g, "rays", 2)
    backend.gn_check()  # nothing pending
    monkeypatch.setenv("M3S_TEST_FORCE_TIMEOUT", "1")
    # the report is deferred (no host wait at the end of the call): gn_check raises it ...
    T_to, _ = _run_gpu(backend, g, "rays", 2)
    # ... and the timed-out call committed nothing: the device restored the poses it started from
    # (ADVICE r04), so a caller that writes Twc back before checking never stores a failed solve
    assert np.array_equal(T_to, g.Twc.numpy())
    with pytest.raises(RuntimeError, match="timed out"):
        backend.gn_check()
    backend.gn_check()  # ... once
    # ... and so does the next call, before it does any work
    _run_gpu(backend, g, "rays", 2)
    monkeypatch.delenv("M3S_TEST_FORCE_TIMEOUT")
    with pytest.raises(RuntimeError, match="an earlier call: .*timed out"):
        _run_gpu(backend, g, "rays", 2)
    T_again, dx_again = _run_gpu(backend, g, "rays", 2)
    backend.gn_check()
    assert np.array_equal(T_again, T_ok) and np.array_equal(dx_again, dx_ok)


def test_factorisation_timeout_sync_report(backend, monkeypatch):
    """M3S_GN_TIMEOUT_SYNC=1 (read once per process, hence a child process): the timed-out call
    itself raises."""
    import subprocess
    import sys

    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import numpy as np, torch\n"
        "import mast3r_slam_backends as mb\n"
        "from tests import test_gpu_gn as t\n"
        "from m3s import synth\n"
        "g = synth.make_graph('cfg4', H=24, W=32, seed=6)\n"
        "try:\n"
        "    t._run_gpu(mb, g, 'rays', 2)\n"
        "    print('NO ERROR')\n"
        "except RuntimeError as e:\n"
        "    print('RAISED', e)\n"
    ) % (ROOT, os.path.join(ROOT, "mast3r-slam_amd"))
    env = dict(os.environ, M3S_GN_TIMEOUT_SYNC="1", M3S_TEST_FORCE_TIMEOUT="1", M3S_CHOL_DF="1",
               M3S_SOLVER="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert "RAISED" in r.stdout and "timed out" in r.stdout, (r.stdout, r.stderr[-2000:])


@pytest.mark.parametrize("solver", ["multi", "hybrid"])
@pytest.mark.parametrize("nblocks", [128, 256])
def test_dataflow_factor_with_cus_held_by_another_stream(backend, monkeypatch, nblocks, solver):
    """the tracker and the backend launch on the same GPU concurrently.  Here
    workgroups on a second stream hold 64 KiB of LDS on about half / all of the CUs for 30 ms --
    chol_df's 131-KiB workgroups do not fit beside them, so part (or all) of its grid starts late.
    chol_df's workgroups claim their tasks dynamically (round 6), so the resident part only ever
    waits on tasks running workgroups hold: the op finishes with BITWISE the poses of an unhindered
    run -- no timeout branch.  The multi plan (cfg4 topology) and the default
    hybrid plan (cfg3 topology, chol_df core)."""
    from mast3r_slam_backends import variants

    g = _solver_graph(monkeypatch, solver)
    monkeypatch.setenv("M3S_CHOL_DF", "1")
    T_ref, dx_ref = _run_gpu(backend, g, "rays", 3)
    backend.gn_check()
    side = torch.cuda.Stream()
    variants.hold_cus(nblocks, 64 * 1024, 30000, side)
    T_h, dx_h = _run_gpu(backend, g, "rays", 3)
    backend.gn_check()  # no deferred timeout
    torch.cuda.synchronize()
    assert np.array_equal(T_h, T_ref) and np.array_equal(dx_h, dx_ref)


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_degenerate_graphs_leave_poses_and_match_oracle(backend, oracle, mode):
    """Degenerate pose graphs through the whole op (host plan, pre-passes, solve): no edges at all
    (an all-zero system: the Cholesky fails -> dx = 0, poses unchanged, as SimplicialLLT's
    failure path), and a graph whose only edges are self-edges and duplicates of one pair."""
    g = synth.make_graph(dict(N=3, E=1), H=24, W=32, seed=3, edges_only=[(0, 1)])
    empty = lambda t: t[:0].contiguous()
    g0 = dataclasses.replace(g, ii=empty(g.ii), jj=empty(g.jj), idx=empty(g.idx), valid=empty(g.valid),
                             Q=empty(g.Q))
    T, dx = _run_gpu(backend, g0, mode, 3)
    assert np.array_equal(T, g.Twc.numpy())
    assert dx is None or not np.any(dx)
    # duplicates of (0, 1) in both directions and a self-edge on pose 2
    und = [(0, 1), (0, 1), (2, 2)]
    g2 = synth.make_graph(dict(N=3, E=len(und)), H=24, W=32, seed=4, edges_only=und)
    T2, _ = _run_gpu(backend, g2, mode, 2)
    T_o, _, _ = _run_oracle(oracle, g2, mode, 2)
    assert np.isfinite(T2).all()
    assert _rel(T2, T_o) < 1e-5, _rel(T2, T_o)
