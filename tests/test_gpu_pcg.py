"""The lagged-factor PCG (gn_pcg.hip, DESIGN.md §4 "Round 6"): from iteration 2 on, the GN step is
solved by conjugate gradients preconditioned with the inverse of iteration 1's system, the direct
block-sparse factorisation (the reference's SimplicialLLT, gn_kernels.cu:132-153) staying enqueued
behind it as the fallback.

Checked here: the PCG path is what runs (its device counters), its poses equal the direct path's
to the CG tolerance and the oracle's to north_star's 1e-5 on the bench graphs, a forced fallback
(no convergence within kmax steps) is bitwise the direct path, the result is deterministic, and a
graph whose systems are singular keeps SimplicialLLT's dx = 0 semantics.
"""
import os

import numpy as np
import pytest
import torch

from m3s import synth

from tests.test_gpu_gn import _rel, _run_gpu, _run_oracle

pytestmark = pytest.mark.gpu

# gn_driver.hip pcg_from_for: the first PCG iteration -- 3 on cores of >= 8 tile columns (cfg4's
# multi plan, 14), 4 below (cfg3's hybrid core, 4); M from two iterations earlier
PCG_FROM = {"cfg3": 4, "cfg4": 3}


def _graph(cfg, H, W, seed=None):
    g = synth.make_graph(cfg, H=H, W=W, seed=seed)
    if synth.CONFIGS[cfg]["mode"] == "calib":
        from m3s.geometry import constrain_points_to_ray

        g.Xs = constrain_points_to_ray((H, W), g.Xs, g.K).contiguous()
    return g


def _run(backend, monkeypatch, g, mode, iters, **env):
    env.setdefault("M3S_GN_PCG", 2)  # (the default enables it on cores of >= 8 tile columns only)
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    monkeypatch.setenv("M3S_GN_DEBUG_FLAGS", "2")
    T, dx = _run_gpu(backend, g, mode, iters)
    backend.gn_check()
    st = backend.gn_debug_flags()
    for k in env:
        monkeypatch.delenv(k)
    monkeypatch.delenv("M3S_GN_DEBUG_FLAGS")
    return T, dx, st


@pytest.mark.parametrize("cfg,H,W", [("cfg3", 96, 128), ("cfg4", 48, 64)])
def test_pcg_runs_and_matches_the_direct_solve(backend, monkeypatch, cfg, H, W):
    """Both bench topologies (cfg3: the hybrid plan; cfg4: the multi plan), 10 iterations: six /
    seven PCG solves, none falling back; poses within 1e-6 of the direct solve's (the CG stop is
    sqrt(r'z / r0'z0) <= 1e-6) and bitwise reproducible."""
    mode = synth.CONFIGS[cfg]["mode"]
    g = _graph(cfg, H, W)
    T_d, dx_d, st_d = _run(backend, monkeypatch, g, mode, 10, M3S_GN_PCG=0)
    assert not st_d["pcg_planned"] and st_d["pcg_runs"] == 0
    T_p, dx_p, st = _run(backend, monkeypatch, g, mode, 10)
    print(cfg, st)
    k = PCG_FROM[cfg]
    assert st["pcg_planned"] and st["pcg_from"] == k and st["pcg_runs"] == 10 - k and st["pcg_fallbacks"] == 0, st
    assert 10 - k <= st["pcg_steps"] <= (10 - k) * 30, st
    assert np.isfinite(T_p).all()
    assert _rel(T_p, T_d) < 1e-6, _rel(T_p, T_d)
    T_p2, dx_p2, _ = _run(backend, monkeypatch, g, mode, 10)
    assert np.array_equal(T_p2, T_p) and np.array_equal(dx_p2, dx_p)


def test_pcg_fallback_is_bitwise_the_direct_solve(backend, monkeypatch):
    """kmax = 1 CG step: no PCG solve converges, every iteration falls back to the direct
    factorisation enqueued behind it -- bitwise the PCG-off call."""
    g = _graph("cfg3", 48, 64)
    T_d, dx_d, _ = _run(backend, monkeypatch, g, "calib", 6, M3S_GN_PCG=0)
    # (kmax is read once per process: a child process)
    import subprocess
    import sys

    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import numpy as np, torch\n"
        "import mast3r_slam_backends as mb\n"
        "from tests import test_gpu_pcg as t\n"
        "g = t._graph('cfg3', 48, 64)\n"
        "from tests.test_gpu_gn import _run_gpu\n"
        "T, dx = _run_gpu(mb, g, 'calib', 6)\n"
        "mb.gn_check()\n"
        "print('STATS', mb.gn_debug_flags())\n"
        "np.save(sys.argv[1], T)\n"
    ) % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
         os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mast3r-slam_amd"))
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "T.npy")
        env = dict(os.environ, M3S_PCG_KMAX="1", M3S_GN_DEBUG_FLAGS="2", M3S_GN_PCG="2")
        r = subprocess.run([sys.executable, "-c", code, out], env=env, capture_output=True, text=True, timeout=240,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        n = 6 - PCG_FROM["cfg3"]
        assert f"'pcg_runs': {n}" in r.stdout and f"'pcg_fallbacks': {n}" in r.stdout, r.stdout
        T_f = np.load(out)
    assert np.array_equal(T_f, T_d)


@pytest.mark.parametrize("cfg,H,W", [("cfg3", 384, 512), ("cfg4", 384, 512)])
def test_pcg_bench_graphs_full_size_within_1e5_of_oracle(backend, oracle, monkeypatch, cfg, H, W):
    """The timed workloads at full 512x384 (10 iterations, the default policy: PCG from iteration
    3 on cfg4, whose core has 14 tile columns, from 4 on cfg3's 4): within north_star's 1e-5 of
    the CPU oracle."""
    mode = synth.CONFIGS[cfg]["mode"]
    g = _graph(cfg, H, W)
    T_p, _, st = _run(backend, monkeypatch, g, mode, 10, M3S_GN_PCG=1)
    assert st["pcg_runs"] == 10 - PCG_FROM[cfg] and st["pcg_fallbacks"] == 0, st
    T_o, _, _ = _run_oracle(oracle, g, mode, 10)
    d = _rel(T_p, T_o)
    print(cfg, "pcg vs oracle", d, st)
    assert d < 1e-5, d


def test_pcg_singular_system_keeps_dx_zero(backend, monkeypatch):
    """Every confidence below C_thresh: all-zero systems, so the iteration-1 factorisation fails
    (the inverse is garbage) and every PCG breaks down -> the direct path's failure semantics
    (SimplicialLLT: dx = 0), poses unchanged."""
    g = _graph("cfg3", 24, 32)
    g.Cs = torch.zeros_like(g.Cs)
    T, dx, st = _run(backend, monkeypatch, g, "calib", 5)
    assert np.array_equal(T, g.Twc.numpy())
    assert dx is None or not np.any(dx)
    assert st["pcg_runs"] == st["pcg_fallbacks"], st


@pytest.mark.parametrize("nblocks", [128, 256])
def test_pcg_with_cus_held_by_another_stream(backend, monkeypatch, nblocks):
    """another stream's workgroups hold 64 KiB of LDS on about half / all of the
    CUs for 30 ms while a PCG iteration runs (cfg4 topology, PCG from iteration 3): the PCG's
    130-KiB workgroups start late, the resident ones wait in their first exchange (its bound is
    seconds, not the 30 ms) -- the call ends with bitwise the unhindered poses, no fallback."""
    from mast3r_slam_backends import variants

    g = _graph("cfg4", 48, 64)
    T_ref, dx_ref, st_ref = _run(backend, monkeypatch, g, "rays", 6, M3S_GN_PCG=1)
    assert st_ref["pcg_runs"] == 6 - PCG_FROM["cfg4"] and st_ref["pcg_fallbacks"] == 0, st_ref
    side = torch.cuda.Stream()
    variants.hold_cus(nblocks, 64 * 1024, 30000, side)
    T_h, dx_h, st = _run(backend, monkeypatch, g, "rays", 6, M3S_GN_PCG=1)
    torch.cuda.synchronize()
    assert st["pcg_fallbacks"] == 0, st
    assert np.array_equal(T_h, T_ref) and np.array_equal(dx_h, dx_ref)
