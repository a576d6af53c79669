"""The GN solve's elimination plan (sparse_plan.h, chosen by gn_driver.hip choose_sparse_plan),
checked on the host through the diagnostic m3s_gn_plan_info -- no GPU.  The reference leaves this
step to Eigen's SimplicialLLT symbolic analysis on every solve (gn_kernels.cu:132-153); here the
plan is a sequence of rounds of independent poses plus a dense core, and the checks are the
properties the device solve relies on: every pose once, each round independent in the graph as
filled by the rounds before it, the degree caps, and the bench graphs' known plans."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mast3r-slam_amd"))


def graph_lists(cfg):
    from m3s import synth

    spec = synth.CONFIGS[cfg]
    seed = {"cfg1": 1, "cfg2": 2, "cfg3": 3, "cfg4": 4}[cfg]
    und = synth.make_edges(spec["N"], spec["E"], seed)
    ii = [a for a, b in und] + [b for a, b in und]
    jj = [b for a, b in und] + [a for a, b in und]
    return ii, jj, spec["N"]


def simulate(ii, jj, N, info, dcap):
    """Replay the plan's rounds on the pose graph: each round's poses must be pairwise
    non-adjacent in the graph filled by the earlier rounds, within the degree cap; the core is
    what remains."""
    ids = sorted(set(ii) | set(jj))
    row = {k: r - 1 for r, k in enumerate(ids)}  # first row pinned
    npose = N - 1
    adj = [set() for _ in range(npose)]
    for a, b in zip(ii, jj):
        i, j = row[a], row[b]
        if i >= 0 and j >= 0 and i != j:
            adj[i].add(j)
            adj[j].add(i)
    order, rp = info["order"], info["round_ptr"]
    assert sorted(order) == list(range(npose))
    assert rp[0] == 0 and rp[-1] == info["eliminated"]
    alive = set(range(npose))
    for r in range(info["rounds"]):
        nodes = order[rp[r]:rp[r + 1]]
        assert nodes == sorted(nodes) and nodes
        S = set(nodes)
        for v in nodes:
            assert not (adj[v] & S), f"round {r}: {v} adjacent to another pose of its round"
            assert len(adj[v]) <= dcap
        for v in nodes:  # eliminate: the front becomes a clique
            F = adj[v]
            for x in F:
                adj[x] |= F - {x}
                adj[x].discard(v)
            adj[v] = set()
            alive.discard(v)
    assert sorted(order[info["eliminated"]:]) == sorted(alive)
    assert info["core_poses"] == len(alive)
    assert info["core_unknowns_padded"] == (-(-7 * len(alive) // 64) * 64 if alive else 0)


def test_bench_graphs_plans(backend):
    ii, jj, N = graph_lists("cfg3")
    p = backend.gn_plan_info(ii, jj, N)
    # cfg3 (127 free poses, 252 pairs): minimum-degree rounds until the rest fits 4 tile columns
    # of the dataflow core (<= 36 poses) and a round would remove fewer than 4 poses: 5 rounds, a
    # 34-pose core (late round 5)
    assert (p["solver"], p["rounds"], p["core_poses"], p["core_unknowns_padded"], p["pairs"]) == \
        ("hybrid", 5, 34, 256, 252)
    assert p["core_fits"]
    simulate(ii, jj, N, p, 64)
    ii, jj, N = graph_lists("cfg4")
    p = backend.gn_plan_info(ii, jj, N)
    # cfg4 (255 free poses, 1007 pairs): degree cap 32, 3 rounds -- a 4th of 2 poses would leave
    # the core's 14 tiles of 64 unchanged (M3S_MULTI_KMIN) --, a 127-pose core (889 unknowns) for
    # chol_df
    assert (p["solver"], p["rounds"], p["core_poses"], p["core_unknowns_padded"], p["pairs"]) == \
        ("multi", 3, 127, 896, 1007)
    assert p["core_fits"]
    simulate(ii, jj, N, p, 32)


def test_hybrid_core_cap_switches(backend, monkeypatch):
    ii, jj, N = graph_lists("cfg3")
    # the in-register core's bound (27 poses): 8 rounds down to 26 poses, the plan before late
    # round 5 -- also what the in-register core factorisation (M3S_HYB_CORE=0) gets by default
    monkeypatch.setenv("M3S_HYB_TAILCAP", "27")
    p = backend.gn_plan_info(ii, jj, N)
    assert (p["solver"], p["rounds"], p["core_poses"], p["core_unknowns_padded"]) == ("hybrid", 8, 26, 192)
    simulate(ii, jj, N, p, 64)
    monkeypatch.delenv("M3S_HYB_TAILCAP")
    monkeypatch.setenv("M3S_HYB_CORE", "0")
    p = backend.gn_plan_info(ii, jj, N)
    assert (p["solver"], p["rounds"], p["core_poses"]) == ("hybrid", 8, 26)


def test_multi_tile_stop_switch(backend, monkeypatch):
    ii, jj, N = graph_lists("cfg4")
    monkeypatch.setenv("M3S_MULTI_KMIN", "0")  # every round the degree cap admits
    p = backend.gn_plan_info(ii, jj, N)
    assert (p["solver"], p["rounds"], p["core_poses"], p["core_unknowns_padded"]) == ("multi", 4, 125, 896)
    simulate(ii, jj, N, p, 32)


def test_degree_cap_switch(backend, monkeypatch):
    ii, jj, N = graph_lists("cfg4")
    monkeypatch.setenv("M3S_MULTI_DCAP", "16")  # round 4's cap: fewer rounds, a bigger core
    p = backend.gn_plan_info(ii, jj, N)
    assert (p["solver"], p["rounds"], p["core_poses"]) == ("multi", 3, 141)
    simulate(ii, jj, N, p, 16)


@pytest.mark.parametrize("seed", range(12))
def test_random_graphs_plan_invariants(backend, seed):
    rng = np.random.default_rng(seed)
    N = int(rng.integers(3, 160))
    ids = rng.permutation(10 * N)[:N] + 100  # arbitrary global keyframe ids
    und = [(ids[k - 1], ids[k]) for k in range(1, N) if rng.random() < 0.9]
    for _ in range(int(rng.integers(0, 3 * N))):
        a, b = rng.integers(0, N, 2)
        und.append((ids[a], ids[b]))  # duplicates and self-edges included
    und.append((ids[0], ids[N - 1]))
    ii = [a for a, b in und] + [b for a, b in und]
    jj = [b for a, b in und] + [a for a, b in und]
    used = sorted(set(ii) | set(jj))
    p = backend.gn_plan_info(ii, jj, len(used))
    cap = 32 if p["solver"] == "multi" else 64
    simulate(ii, jj, len(used), p, cap)


@pytest.mark.parametrize("N,extra,seed", [(1250, 3, 0), (1400, 4, 1), (1800, 2, 2)])
def test_large_graphs_core_fits_when_the_untrimmed_plan_fits(backend, monkeypatch, N, extra, seed):
    """The multi plan's tile-aware stop (M3S_MULTI_KMIN) must never leave a core above the dense
    solve limit (8192 unknowns) where the plan without the stop fits: large random
    loop-closure graphs, both plans replayed."""
    rng = np.random.default_rng(seed)
    und = [(k - 1, k) for k in range(1, N)]
    for _ in range(extra * N):
        a, b = rng.integers(0, N, 2)
        if a != b:
            und.append((int(a), int(b)))
    ii = [a for a, b in und] + [b for a, b in und]
    jj = [b for a, b in und] + [a for a, b in und]
    p = backend.gn_plan_info(ii, jj, N)
    simulate(ii, jj, N, p, 32 if p["solver"] == "multi" else 64)
    monkeypatch.setenv("M3S_MULTI_KMIN", "0")
    p0 = backend.gn_plan_info(ii, jj, N)
    if p0["core_fits"]:
        assert p["core_fits"], (p["core_unknowns_padded"], p0["core_unknowns_padded"])


def test_edge_cases(backend):
    p = backend.gn_plan_info([], [], 1)
    assert p["solver"] is None and p["order"] == []
    # no edges: every pose independent, eliminated in the first round
    p = backend.gn_plan_info([], [], 5)
    assert p["eliminated"] + p["core_poses"] == 4 and sorted(p["order"]) == [0, 1, 2, 3]
    # self-edges are not pose pairs
    p = backend.gn_plan_info([7, 7, 9], [7, 9, 7], 2)
    assert p["pairs"] == 0
    with pytest.raises(RuntimeError, match="unique keyframe ids"):
        backend.gn_plan_info([1, 2, 3], [2, 3, 4], 2)


def test_large_and_negative_keyframe_ids_rank_like_small_ones(backend):
    """Keyframe ids far apart or negative take the sorted (not the dense-table) ranking: the same
    plan as the same graph on ids 0 .. N-1."""
    ii, jj, N = graph_lists("cfg3")
    ref = backend.gn_plan_info(ii, jj, N)
    for f in (lambda k: k * 10**9 + 7, lambda k: k - 50):
        p = backend.gn_plan_info([f(k) for k in ii], [f(k) for k in jj], N)
        assert p == ref
