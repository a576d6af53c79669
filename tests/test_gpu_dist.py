"""The product's edge-sharded GN op with two ranks, on the one GPU of the box.

Two spawned processes share cuda:0 and a gloo process group.  Each calls
``m3s.dist.gauss_newton_sharded`` -- the same op as bench.py --gpus N, with its accumulate,
the in-op per-iteration exchange of the compact block system and the replicated solve +
retraction -- on its contiguous directed-edge range; the exchange goes through the library's
host-callback communicator (``m3s_comm_init_host``: stream drained, system staged, gloo
all_reduce, copied back) instead of RCCL, which needs one GPU per rank.

Checked: Twc is bitwise identical on both ranks after 3 iterations (no broadcast in the op),
the callback ran once per iteration (plus once per call for the ranks' edge ranges), and the
result is BITWISE the unsharded op's: the default exchange all-gathers the ranks' f64 per-edge
records and every rank assembles all edges in edge order, as one GPU does (the per-edge records
themselves do not depend on the rank count: the chunking follows the total edge count).  The
former exchange -- an all-reduce of the ranks' assembled partial systems, M3S_GN_GATHER=0 -- is
checked to f64 summation-reorder level (1e-6 relative).  Also: the exactly summed system at the
north-star 1e-5 and the oracle within max(1e-5, 4 sigma) (sigma: the reference fp32 order's own
distance from the exact sums).
Reference seam: global_opt.py:104-110 (two-way edges), gn_kernels.cu:1201-1209 (the solve).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

LOCAL = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0,
             C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)
ITERS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# cfg2 topology at 96x128; cfg4's (256 keyframes, 1024 pair edges: the multi-launch solve with the
# dataflow core factorisation, BASELINE configs[3]'s sharded graph) at a reduced 48x64
SIZES = {"cfg2": (96, 128), "cfg4": (48, 64)}


def _graph(mode, cfg="cfg2"):
    from m3s import synth

    H, W = SIZES[cfg]
    g = synth.make_graph(cfg, H=H, W=W, seed=7)
    if mode == "calib":
        from m3s.geometry import constrain_points_to_ray

        g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    return g


def _params(g, mode):
    p = dict(LOCAL)
    if mode == "calib":
        p.update(K=g.K.cuda(), height=g.H, width=g.W)
    return p


def _worker(rank, world, port, mode, layout, cfg, exchange, out_q, iters=ITERS):
    import sys

    if exchange == "reduce":
        os.environ["M3S_GN_GATHER"] = "0"
    if exchange == "gather_early":  # iteration 0's all-gather enqueued before the host plans
        os.environ["M3S_EARLY_GATHER"] = "1"

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mast3r-slam_amd")]
    import torch.distributed as dist

    from m3s.dist import HostComm, gauss_newton_sharded, shard_range, two_way_range

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = _graph(mode, cfg)
        lo, hi = shard_range(g.ii.shape[0], world, rank)
        if layout == "two_way":  # uneven split: rank 0's range spans both halves of the store
            E = g.ii.shape[0] // 2
            lo, hi = [(0, E + 5), (E + 5, 2 * E)][rank]
        c = lambda t: t.cuda().contiguous()
        Twc = c(g.Twc)
        comm = HostComm()
        if layout == "contiguous":
            gauss_newton_sharded(mode, Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx[lo:hi]),
                                 c(g.valid[lo:hi]), c(g.Q[lo:hi]), lo, comm, iters, 0.0,
                                 **_params(g, mode))
        else:
            # a two-way edge store (forward, backward halves): the rank's directed range as views
            E = g.ii.shape[0] // 2
            fwd = (c(g.idx[:E]), c(g.valid[:E]), c(g.Q[:E]))
            bwd = (c(g.idx[E:]), c(g.valid[E:]), c(g.Q[E:]))
            first, second = two_way_range(fwd, bwd, lo, hi)
            gauss_newton_sharded(mode, Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), *first, lo, comm,
                                 iters, 0.0, second_half=second, **_params(g, mode))
        torch.cuda.synchronize()
        out_q.put((rank, Twc.cpu().numpy(), comm.calls, (lo, hi), None))
        comm.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        out_q.put((rank, None, 0, None, repr(e)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode,layout,cfg,exchange,iters", [
    ("rays", "contiguous", "cfg2", "gather", ITERS), ("calib", "contiguous", "cfg2", "gather", ITERS),
    ("rays", "two_way", "cfg2", "gather", ITERS), ("rays", "contiguous", "cfg4", "gather", ITERS),
    ("calib", "contiguous", "cfg2", "reduce", ITERS), ("rays", "contiguous", "cfg4", "reduce", ITERS),
    ("calib", "contiguous", "cfg2", "gather_early", ITERS), ("rays", "contiguous", "cfg4", "gather_early", ITERS),
    ("rays", "contiguous", "cfg4", "gather", 6)])
def test_two_rank_sharded_op_matches_unsharded(backend, oracle, mode, layout, cfg, exchange, iters):
    """layout "two_way": each rank passes its directed-edge range of a two-way edge store as
    the op's two halves (m3s.dist.two_way_range) -- the owner-sharded store layout.  cfg4: the
    scaling graph's topology (BASELINE configs[3]) at reduced resolution; at 6 iterations its
    solves from iteration 3 are the lagged-factor PCG's (gn_pcg.hip), run by every rank on the same
    all-gathered system: still bitwise the 1-rank poses."""
    world = 2
    ITERS = iters  # noqa: N806 -- (the checks below count per-iteration exchanges)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, layout, cfg, exchange, q, iters))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[4] is None, r[4]
    assert all(p.exitcode == 0 for p in procs)
    (_, T0, calls0, rng0, _), (_, T1, calls1, rng1, _) = res
    assert rng0[0] == 0 and rng0[1] == rng1[0] and rng0[1] > 0 and rng1[1] > rng1[0]
    # one exchange per iteration (+ the ranks' edge ranges once per call when gathering); cfg4's
    # dataflow factorisation (bounded device waits) adds one for the ranks' OR of the timeout flag
    gather = exchange.startswith("gather")
    assert calls0 == calls1 == ITERS + gather + (1 if cfg == "cfg4" else 0)
    # bitwise identical poses on every rank: same all-reduced system, same deterministic solve
    assert np.array_equal(T0, T1)

    g = _graph(mode, cfg)
    c = lambda t: t.cuda()
    Twc = c(g.Twc)
    if mode == "rays":
        backend.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                                  LOCAL["sigma_ray"], LOCAL["sigma_dist"], LOCAL["C_conf"],
                                  LOCAL["Q_conf"], ITERS, 0.0)
        P = oracle.make_params("rays", LOCAL["sigma_ray"], LOCAL["sigma_dist"], LOCAL["C_conf"],
                               LOCAL["Q_conf"], max_iter=ITERS, delta_thresh=0.0)
    else:
        backend.gauss_newton_calib(Twc, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx),
                                   c(g.valid), c(g.Q), g.H, g.W, LOCAL["pixel_border"],
                                   LOCAL["depth_eps"], LOCAL["sigma_pixel"], LOCAL["sigma_depth"],
                                   LOCAL["C_conf"], LOCAL["Q_conf"], ITERS, 0.0)
        P = oracle.make_params("calib", LOCAL["sigma_pixel"], LOCAL["sigma_depth"], LOCAL["C_conf"],
                               LOCAL["Q_conf"], K=g.K.numpy(), height=g.H, width=g.W,
                               pixel_border=LOCAL["pixel_border"], z_eps=LOCAL["depth_eps"],
                               max_iter=ITERS, delta_thresh=0.0)
    torch.cuda.synchronize()
    T_full = Twc.cpu().numpy()
    rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
    if gather:
        assert np.array_equal(T0, T_full), rel(T0, T_full)  # rank-count independent
    else:
        assert rel(T0, T_full) < 1e-6, rel(T0, T_full)
    arrs = (g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(), g.idx.numpy(),
            g.valid.numpy(), g.Q.numpy())
    T_o, _, _ = oracle.gauss_newton(P, *arrs)
    with oracle.exact_sums():
        T_x, _, _ = oracle.gauss_newton(P, *arrs)
    # the north-star 1e-5 against the exactly summed system; against the oracle (the reference's
    # fp32 order) within max(1e-5, 4 sigma), sigma = that order's own distance from the exact sums
    sigma = rel(T_o, T_x)
    assert rel(T0, T_x) < 1e-5, rel(T0, T_x)
    assert rel(T0, T_o) < max(1e-5, 4 * sigma), (rel(T0, T_o), sigma)


def _timeout_worker(rank, world, port, out_q):
    """cfg4 topology (the dataflow core factorisation, whose waits are bounded) with the forced
    timeout on rank 1 only"""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mast3r-slam_amd")]
    import torch.distributed as dist

    import mast3r_slam_backends as mb
    from m3s.dist import HostComm, gauss_newton_sharded, shard_range

    if rank == 1:
        os.environ["M3S_TEST_FORCE_TIMEOUT"] = "1"
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = _graph("rays", "cfg4")
        lo, hi = shard_range(g.ii.shape[0], world, rank)
        c = lambda t: t.cuda().contiguous()
        comm = HostComm()
        err = None
        Twc = c(g.Twc)
        try:
            gauss_newton_sharded("rays", Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx[lo:hi]),
                                 c(g.valid[lo:hi]), c(g.Q[lo:hi]), lo, comm, 2, 0.0, **_params(g, "rays"))
            mb.gn_check()  # the deferred report (include/m3s_backend.h m3s_gn_check)
        except RuntimeError as e:
            err = str(e)
        torch.cuda.synchronize()
        # every rank restored the poses the call started from (no rank keeps a pose
        # set the others do not have)
        restored = bool(torch.equal(Twc.cpu(), g.Twc))
        out_q.put((rank, err, comm.calls, None if restored else "Twc not restored"))
        comm.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        out_q.put((rank, None, 0, repr(e)))


@pytest.mark.timeout(300)
def test_a_timeout_on_one_rank_fails_every_rank(backend):
    """A bounded device-side wait that gives up on ONE rank (test hook on rank 1 only) must make
    every rank return M3S_ERR_TIMEOUT: the op ORs the rank-local timeout flag over the ranks before
    deciding its return code, so no rank goes on to a collective the others never reach (ADVICE
    r03).  Both ranks still ran every iteration's exchange."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in res:
        assert r[3] is None, r[3]
        assert r[1] is not None and "timed out" in r[1], r[1]
    assert res[0][2] == res[1][2] == 1 + 2 + 1  # the edge ranges, two iterations' exchanges, the flag


def _rccl_worker(port, mode, out_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mast3r-slam_amd")]
    import torch.distributed as dist

    import mast3r_slam_backends as mb
    from m3s.dist import RcclComm, gauss_newton_sharded

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=0, world_size=1)
        torch.cuda.set_device(0)
        g = _graph(mode)
        c = lambda t: t.cuda().contiguous()
        comm = RcclComm(0, 1, device=torch.device("cuda", 0))
        Twc = c(g.Twc)
        gauss_newton_sharded(mode, Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q), 0,
                             comm, ITERS, 0.0, **_params(g, mode))
        Twc_ref = c(g.Twc)
        if mode == "rays":
            mb.gauss_newton_rays(Twc_ref, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                                 LOCAL["sigma_ray"], LOCAL["sigma_dist"], LOCAL["C_conf"], LOCAL["Q_conf"],
                                 ITERS, 0.0)
        else:
            mb.gauss_newton_calib(Twc_ref, c(g.Xs), c(g.Cs), c(g.K), c(g.ii), c(g.jj), c(g.idx), c(g.valid),
                                  c(g.Q), g.H, g.W, LOCAL["pixel_border"], LOCAL["depth_eps"],
                                  LOCAL["sigma_pixel"], LOCAL["sigma_depth"], LOCAL["C_conf"],
                                  LOCAL["Q_conf"], ITERS, 0.0)
        torch.cuda.synchronize()
        out_q.put((Twc.cpu().numpy(), Twc_ref.cpu().numpy(), None))
        comm.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        out_q.put((None, None, repr(e)))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_rccl_communicator_in_the_op(backend, mode):
    """The production exchange: the library's RCCL communicator (m3s_comm_get_unique_id /
    m3s_comm_init, librccl resolved at run time) and the in-stream ncclAllReduce of the block
    system inside the op, with one rank on the box's one GPU (RCCL needs a GPU per rank, so more
    ranks are the driver's multi-GPU bench).  A one-rank sum leaves the system unchanged: the
    poses must equal the unsharded op's bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), mode, q))
    p.start()
    try:
        T, T_ref, err = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert err is None, err
    assert p.exitcode == 0
    assert np.array_equal(T, T_ref)
