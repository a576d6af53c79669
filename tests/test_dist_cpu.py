"""Multi-rank edge sharding on CPU (gloo, world_size 2): the per-rank partial normal
equations of contiguous directed-edge shards, summed with an all-reduce, equal the
single-process system, and every rank then solves to the same update.  This is the
exchange the GPU path performs with RCCL inside the op (m3s.dist)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from m3s.dist import shard_range


def test_shard_range_partitions():
    for E in (0, 1, 7, 512, 2048):
        for world in (1, 2, 3, 8):
            rs = [shard_range(E, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == E
            assert all(rs[k][1] == rs[k + 1][0] for k in range(world - 1))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mast3r-slam_amd")]
    from m3s import synth
    from m3s.dist import shard_range as sr
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.make_graph(dict(N=6, E=9), H=24, W=32, seed=4)
    E2 = g.ii.shape[0]
    lo, hi = sr(E2, world, rank)
    P = O.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1)
    ie, je, _ = O.remap(g.ii.numpy(), g.jj.numpy())
    Hs, gs = O.gn_align(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), ie[lo:hi], je[lo:hi],
                        g.idx.numpy()[lo:hi], g.valid.numpy()[lo:hi], g.Q.numpy()[lo:hi])
    H, b = O.gn_assemble(Hs, gs, ie[lo:hi] - 1, je[lo:hi] - 1, g.N)
    Ht = torch.from_numpy(np.concatenate([H.ravel(), b]))
    dist.all_reduce(Ht)  # the per-iteration exchange
    n = b.shape[0]
    Hsum, bsum = Ht[: n * n].numpy().reshape(n, n), Ht[n * n:].numpy()
    x, rc = O.cholesky_solve(Hsum, bsum)
    out_q.put((rank, Hsum, bsum, x))
    dist.destroy_process_group()


def test_two_rank_sharded_system_equals_full(oracle):
    from m3s import synth

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])

    g = synth.make_graph(dict(N=6, E=9), H=24, W=32, seed=4)
    P = oracle.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1)
    H, b = oracle.gn_build_system(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                                  g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
    x_full, _ = oracle.cholesky_solve(H, b)
    for _, Hs_, bs_, x in res:
        np.testing.assert_allclose(Hs_, H, rtol=1e-12, atol=1e-12 * np.abs(H).max())
        np.testing.assert_allclose(bs_, b, rtol=1e-12, atol=1e-12 * np.abs(b).max())
        np.testing.assert_allclose(x, x_full, rtol=1e-9, atol=1e-12)
    # both ranks hold bitwise-identical systems and solutions (no broadcast needed)
    assert np.array_equal(res[0][1], res[1][1]) and np.array_equal(res[0][3], res[1][3])


def _gather_worker(rank, world, port, ranges, out_q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "mast3r-slam_amd")]
    from m3s import synth
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = synth.make_graph(dict(N=6, E=9), H=24, W=32, seed=4)
    P = O.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1)
    ie, je, _ = O.remap(g.ii.numpy(), g.jj.numpy())
    lo, hi = ranges[rank]
    Hs, gs = O.gn_align(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), ie[lo:hi], je[lo:hi],
                        g.idx.numpy()[lo:hi], g.valid.numpy()[lo:hi], g.Q.numpy()[lo:hi])
    # the op's default exchange: every rank's per-edge records (Hs [4, E, 7, 7], gs [2, E, 7]),
    # gathered in blocks of the largest range (gn_driver.hip Plan::gather), then ALL edges
    # assembled in edge order on every rank
    n = hi - lo
    chunk = max(h - l for l, h in ranges)
    rec = np.zeros((chunk, 4 * 49 + 2 * 7))
    rec[:n] = np.concatenate([Hs.transpose(1, 0, 2, 3).reshape(n, -1), gs.transpose(1, 0, 2).reshape(n, -1)], 1)
    out = [torch.zeros_like(torch.from_numpy(rec)) for _ in range(world)]
    dist.all_gather(out, torch.from_numpy(rec))
    E2 = g.ii.shape[0]
    allrec = np.zeros((E2, rec.shape[1]))
    for r, (l, h) in enumerate(ranges):
        allrec[l:h] = out[r].numpy()[: h - l]
    Hall = np.ascontiguousarray(allrec[:, :196].reshape(E2, 4, 7, 7).transpose(1, 0, 2, 3)).astype(Hs.dtype)
    gall = np.ascontiguousarray(allrec[:, 196:].reshape(E2, 2, 7).transpose(1, 0, 2)).astype(gs.dtype)
    H, b = O.gn_assemble(Hall, gall, ie - 1, je - 1, g.N)
    out_q.put((rank, H, b))
    dist.destroy_process_group()


def test_gathered_edge_records_make_the_system_rank_count_independent(oracle):
    """Three ranks with ragged ranges: gathering the per-edge records and assembling every edge in
    edge order gives BITWISE the one-process system (the all-reduce of partial systems above
    agrees only to summation-reorder level)."""
    from m3s import synth

    g = synth.make_graph(dict(N=6, E=9), H=24, W=32, seed=4)
    E2 = g.ii.shape[0]
    ranges = [(0, 5), (5, 7), (7, E2)]
    world = len(ranges)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, ranges, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P = oracle.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1)
    ie, je, _ = oracle.remap(g.ii.numpy(), g.jj.numpy())
    Hs, gs = oracle.gn_align(P, g.Twc.numpy(), g.Xs.numpy(), g.Cs.numpy(), ie, je, g.idx.numpy(),
                             g.valid.numpy(), g.Q.numpy())
    H, b = oracle.gn_assemble(Hs, gs, ie - 1, je - 1, g.N)
    for _, Hr, br in res:
        assert np.array_equal(Hr, H) and np.array_equal(br, b)
