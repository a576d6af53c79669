#!/usr/bin/env python
"""bench.py -- keyframe-pair GN iterations/s of the MI355X backend (BASELINE.json metric).

One *step* = one ``gauss_newton_calib`` op call on the cfg3 factor graph (BASELINE.json
configs[2]: 256 keyframe-pair edges incl. 129 loop closures, 128 keyframes, 512x384,
calib.yaml parameters) with ``max_iter = 10`` and ``delta_thresh = 0`` so exactly 10 GN
iterations run.  Throughput = 256 pairs x 10 iterations x steps / time.
Inputs are synthetic (m3s.synth, fixed seed) and resident in HBM before timing.

N > 1 (torchrun, one process per GPU): the SAME graph is edge-sharded across ranks and the
per-iteration f64 per-edge records are exchanged with an RCCL all-gather inside the op (every
rank then assembles all edges in edge order: DESIGN.md §6) -> strong scaling; value = total
pair-iterations / max-over-ranks wall time.

Extra fields: ``roofline`` for the dominant kernel (the per-iteration accumulate kernel,
HBM-bound, timed with HIP events on its stream during the timed steps).  Its algorithmic bytes
are those of the packed formulation it runs: per directed point-edge the 8-B
iteration-invariant record {match | invalid bit, sqrt q} + Xj 12 B + the matched point (calib:
its depth, 4 B; rays: Xi, 12 B) = 24 / 32 B; the reference formulation's 45 B
is reported beside it as ``ref_formulation_*`` and ``cpu_baseline`` (the CPU oracle -- a restatement of the reference
backend, which has no CPU implementation -- on a bounded sample, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "keyframe-pair GN iters/sec @512×384, 256 edges; ATE-RMSE vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
REF_BYTES_PER_POINT_EDGE = 45  # Xj 12 + Xi 12 + Cj 4 + Ci 4 + Q 4 + idx 8 + valid 1
# packed formulation (>= 3 iterations per call): record 8 + Xj 12 + matched point (calib: z 4; else Xi 12);
# calib with ray-constrained keyframe points (solve_GN_calib's constrain_points_to_ray): Xj is read
# as its 4-B depth (x, y from the pixel's ray), record 8 + depth 4 + matched inverse depth 4 = 16
PACKED_BYTES_PER_POINT_EDGE = {"calib": 24, "rays": 32, "points": 32}
RAY_BYTES_PER_POINT_EDGE = 16
LOCAL = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, sigma_point=0.05,
             C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)  # base.yaml:35-50


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3", choices=["cfg1", "cfg2", "cfg3", "cfg4"])
    ap.add_argument("--iters", type=int, default=None, help="GN iterations per op call")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-matching", action="store_true", help="skip the matching-kernel section")
    ap.add_argument("--no-cfg4", action="store_true",
                    help="skip the configs[3] block (1024-edge graph, edge-sharded like the headline config)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "accum_traffic.json"))
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """``--gpus N > 1`` without a torch.distributed launcher (no WORLD_SIZE): start N ranks of this
    script with torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a CHILD
    process -- nothing here has touched the GPU -- and return its exit status."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def _dump_maps_at_exit(path):
    """Diagnostics (M3S_EXIT_MAPS=path): this process's /proc/self/maps at interpreter exit, to
    resolve the program counters of a fault during the C-level exit handlers that follow."""
    import atexit

    def dump():
        try:
            with open("/proc/self/maps") as f, open(path, "w") as o:
                o.write(f.read())
        except OSError:
            pass

    atexit.register(dump)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
    if os.environ.get("M3S_BENCH_SPAWN_CHECK"):  # tests/test_bench_cli.py: the launch, no GPU work
        from m3s import synth
        from m3s.dist import shard_range
        plan = {c: list(shard_range(2 * synth.CONFIGS[c]["E"], world, rank))
                for c in ([args.config] + (["cfg4"] if args.config != "cfg4" and not args.no_cfg4 else []))}
        print(json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "edge_ranges": plan}),
              flush=True)
        return
    if os.environ.get("M3S_EXIT_MAPS"):
        _dump_maps_at_exit(os.environ["M3S_EXIT_MAPS"])
    # M3S_BENCH_COMM=host: a rehearsal of the N-rank flow on fewer GPUs (ranks may share one):
    # gloo process group and the op's host-callback exchange instead of RCCL over xGMI
    rehearse = world > 1 and os.environ.get("M3S_BENCH_COMM", "rccl") == "host"
    if rehearse:
        local_rank = local_rank % max(torch.cuda.device_count(), 1)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    import mast3r_slam_backends as mb
    from m3s.dist import HostComm, RcclComm

    comm = (HostComm() if rehearse else RcclComm(rank, world, device=dev)) if world > 1 else None
    r = time_config(args.config, args.iters, args.steps, args.warmup, world, rank, rehearse, dev, comm)
    g, mode, iters, E_und, lo, hi = r["g"], r["mode"], r["iters"], r["E_und"], r["lo"], r["hi"]
    Twc0, Twc, elapsed = r["Twc0"], r["Twc"], r["elapsed"]
    prof, nprof, ph, nph, ray_path = r["prof"], r["nprof"], r["ph"], r["nph"], r["ray_path"]
    acc_events = r["acc_events"]
    n_ph = max(nph.value, 1)
    from m3s import synth

    spec = synth.CONFIGS[args.config]
    E_dir = 2 * E_und
    pair_iters = E_und * iters * args.steps
    value = pair_iters / elapsed
    n_it = max(nprof.value, 1)
    acc_ms = prof[0] / n_it if acc_events else ph[0] / n_ph
    # a calib call's first accumulate builds the packed records itself (M3S_GN_PACK_FIRST):
    # another kernel, timed apart from the iteration kernel the roofline prices
    first_ms = prof[1] / prof[2] if acc_events and prof[2] > 0 else None
    packed = iters >= 3 and os.environ.get("M3S_GN_PACK", "1") != "0"
    bpe = (RAY_BYTES_PER_POINT_EDGE if ray_path else PACKED_BYTES_PER_POINT_EDGE[mode]) if packed \
        else REF_BYTES_PER_POINT_EDGE
    stream = ("packed, ray-constrained Xj (depth only)" if ray_path else "packed") if packed \
        else "reference tensors"
    bytes_launch = bpe * g.HW * (hi - lo)
    ref_bytes_launch = REF_BYTES_PER_POINT_EDGE * g.HW * (hi - lo)
    achieved = bytes_launch / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            tf = json.load(open(args.traffic_file))
            if (tf.get("config") == args.config and tf.get("n_gpus", 1) == world
                    and tf.get("packed", False) == packed and tf.get("stream") == stream):
                traffic = tf.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "keyframe-pair GN iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (m3s.synth seed 3: shared ray-cast world surface, projective matches)",
        "config": {
            "workload": f"{args.config}: gauss_newton_{mode} op call, {E_und} keyframe-pair edges "
                        f"({E_dir} directed), {spec['N']} keyframes, {g.H}x{g.W}, {iters} GN iters/step, "
                        f"delta_thresh=0",
            "edges": E_und,
            "directed_edges": E_dir,
            "keyframes": spec["N"],
            "H": g.H,
            "W": g.W,
            "gn_iters_per_step": iters,
            "parallelism": f"edge-sharded x{world}" + ((" + host exchange (rehearsal: ranks share GPUs)"
                                                         if rehearse else " + RCCL all-gather of the per-edge records")
                                                        if world > 1 else ""),
        },
        "phase_ms_per_iter": {
            "accumulate": acc_ms,
            "reduce_compact_allreduce": ph[1] / n_ph,
            "solve": ph[2] / n_ph,
            "retract": ph[3] / n_ph,
        },
        "solve_path": _solve_path(r["solve_stats"], iters, r["solve_ms"]),
        "roofline": {
            "kernel": f"gn_accum_packed_kernel<{mode}>" if packed else f"gn_accum_kernel<{mode}>",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_launch,
            "algorithmic_bytes_per_point_edge": bpe,
            "stream": stream,
            "avg_launch_ms": acc_ms,
            "ref_formulation_bytes_per_launch": ref_bytes_launch,
            "ref_formulation_equiv_GBps": ref_bytes_launch / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None,
            "launches_per_step": n_it / args.steps,
            "launch_ms_spread": launch_spread(r["launch_ms"]),
            "first_accumulate_with_pack_ms": first_ms,
        },
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(g, mode, E_und, iters)
        out["accuracy"] = accuracy(g, mode, Twc0, Twc, cpu_baseline.last_poses,
                                   cpu_baseline.exact_poses, cpu_baseline.full_poses, iters,
                                   cpu_baseline.last_step, cpu_baseline.exact_step)
        out["accuracy"]["timed_kernel_parity"] = timed_kernel_parity(g, mode, Twc0, cpu_baseline.refs)
        if os.environ.get("M3S_BENCH_REF_ORDER", "1") != "0":
            out["accuracy"]["reference_order_mode"] = reference_order_block(g, mode, Twc0, args, iters)
        if mode == "calib" and os.environ.get("M3S_BENCH_STRESS", "1") != "0":
            out["accuracy"]["stress_1iter"] = stress_block(dev)
    # BASELINE.json configs[3] (1024 edges, the config SURVEY §8(e) sets the scaling target on):
    # with --gpus N it is edge-sharded like the headline config, so the driver's SCALE run
    # measures it at every N.  Its own block; ``value`` stays the headline config's.
    if args.config != "cfg4" and not args.no_cfg4:
        del g, Twc0, Twc, r  # the headline graph is not needed any more
        torch.cuda.empty_cache()
        out["cfg4"] = config_block("cfg4", args, world, rank, rehearse, dev, comm)
    if rank == 0 and world == 1 and not args.no_matching:
        out["matching"] = matching_bench(dev)
        out["tracking"] = tracking_bench(dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


def time_config(cfg, iters_arg, steps, warmup, world, rank, rehearse, dev, comm):
    """Build ``cfg``'s graph (this rank's directed-edge range only), run ``warmup`` untimed op
    calls, then time ``steps`` calls bracketed by a barrier + synchronize on both sides
    (max over ranks); one more untimed call gives the phase times, another the accumulate path
    the op took."""
    import mast3r_slam_backends as mb
    from m3s import synth
    from m3s.dist import gauss_newton_sharded, shard_range
    from m3s.geometry import constrain_points_to_ray

    spec = synth.CONFIGS[cfg]
    mode = spec["mode"]
    iters = iters_arg if iters_arg is not None else spec["iters"]
    E_und = spec["E"]
    lo, hi = shard_range(2 * E_und, world, rank)
    g = synth.make_graph(cfg, device=dev, edge_range=(lo, hi))
    if mode == "calib":  # solve_GN_calib does this before the op (global_opt.py:172)
        g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    Twc0 = g.Twc.clone()
    Twc = g.Twc.clone()
    L = dict(LOCAL, K=g.K, height=g.H, width=g.W)

    def step():
        Twc.copy_(Twc0)
        if world == 1:
            if mode == "calib":
                mb.gauss_newton_calib(Twc, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W,
                                      L["pixel_border"], L["depth_eps"], L["sigma_pixel"],
                                      L["sigma_depth"], L["C_conf"], L["Q_conf"], iters, 0.0)
            else:
                mb.gauss_newton_rays(Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, L["sigma_ray"],
                                     L["sigma_dist"], L["C_conf"], L["Q_conf"], iters, 0.0)
        else:
            gauss_newton_sharded(mode, Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, lo, comm,
                                 iters, 0.0, **L)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed region carries HIP events around each accumulate launch only (the roofline
    # kernel); the other phases are timed in one extra untimed step below
    acc_events = os.environ.get("M3S_BENCH_ACC_EVENTS", "1") != "0"
    if acc_events:
        mb.lib.m3s_prof_begin_accum()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = (ctypes.c_double * 4)()
    nprof = ctypes.c_int(0)
    mb.lib.m3s_prof_end(prof, ctypes.byref(nprof))
    launch_ms = []
    if acc_events:  # the iteration kernel launch by launch (its spread within this run)
        buf = (ctypes.c_double * 4096)()
        n_l = mb.lib.m3s_prof_launch_ms(buf, 4096)
        launch_ms = [buf[k] for k in range(min(n_l, 4096))]
    mb.lib.m3s_prof_begin()
    step()
    torch.cuda.synchronize()
    ph = (ctypes.c_double * 4)()
    nph = ctypes.c_int(0)
    mb.lib.m3s_prof_end(ph, ctypes.byref(nph))
    sbuf = (ctypes.c_double * 256)()
    solve_ms = [sbuf[k] for k in range(min(mb.lib.m3s_prof_solve_ms(sbuf, 256), 256))]
    # which accumulate path the op took (its device flags, read back by one more untimed call)
    os.environ["M3S_GN_DEBUG_FLAGS"] = "2"
    step()
    torch.cuda.synchronize()
    del os.environ["M3S_GN_DEBUG_FLAGS"]
    mb.gn_check()  # a timed-out factorisation is reported by the next call or here (deferred)
    dbg = (ctypes.c_int * 4)()
    mb.lib.m3s_gn_debug_flags(dbg)
    solve_stats = mb.gn_debug_flags()  # (that call's lagged-factor PCG solves)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return dict(g=g, mode=mode, iters=iters, E_und=E_und, lo=lo, hi=hi, Twc0=Twc0, Twc=Twc,
                elapsed=elapsed, prof=prof, nprof=nprof, ph=ph, nph=nph, ray_path=bool(dbg[3]),
                acc_events=acc_events, step=step, launch_ms=launch_ms, solve_stats=solve_stats,
                solve_ms=solve_ms)


def _solve_path(st, iters, solve_ms):
    """How a call solved its iterations: the direct block-sparse factorisation (the first
    iterations, M3S_PCG_FROM = 3 by default, and any fallback) and the lagged-factor PCG
    (gn_pcg.hip) after them; the solve phase per iteration (events of the untimed phase step)
    before and from the first PCG iteration."""
    runs = st["pcg_runs"]
    k = iters - runs  # the first PCG iteration (PCG runs on every iteration from it on)
    head, tail = solve_ms[:k], solve_ms[k:iters]
    return {"pcg_planned": st["pcg_planned"], "direct_iterations": iters - runs + st["pcg_fallbacks"],
            "pcg_iterations": runs - st["pcg_fallbacks"], "pcg_fallbacks": st["pcg_fallbacks"],
            "cg_steps_per_pcg_solve": (st["pcg_steps"] / runs) if runs else None,
            "solve_ms_before_pcg": (sum(head) / len(head)) if head else None,
            "solve_ms_pcg_iterations": (sum(tail) / len(tail)) if tail else None}


def launch_spread(ms):
    """min / median / max (and count) of per-launch kernel ms: a run's own spread, against which
    a same-box A/B gain must be read"""
    if not ms:
        return None
    s = sorted(ms)
    return {"min": s[0], "median": s[len(s) // 2], "max": s[-1], "launches": len(s)}


def config_block(cfg, args, world, rank, rehearse, dev, comm):
    """One more BASELINE config timed exactly like the headline one (same steps / warmup, same
    edge sharding over the ranks), as its own JSON block."""
    from m3s import synth
    from m3s.dist import comm_size

    r = time_config(cfg, None, args.steps, args.warmup, world, rank, rehearse, dev, comm)
    spec = synth.CONFIGS[cfg]
    nph = max(r["nph"].value, 1)
    n_it = max(r["nprof"].value, 1)
    acc_ms = r["prof"][0] / n_it if r["acc_events"] else r["ph"][0] / nph
    packed = r["iters"] >= 3 and os.environ.get("M3S_GN_PACK", "1") != "0"
    bpe = PACKED_BYTES_PER_POINT_EDGE[r["mode"]] if packed else REF_BYTES_PER_POINT_EDGE
    local = r["hi"] - r["lo"]
    bytes_launch = bpe * r["g"].HW * local
    return {
        "value": r["E_und"] * r["iters"] * args.steps / r["elapsed"],
        "unit": "keyframe-pair GN iters/s",
        "ms_per_step": r["elapsed"] / args.steps * 1e3,
        "steps": args.steps,
        "warmup": args.warmup,
        "scaling": "strong",
        "workload": f"{cfg}: gauss_newton_{r['mode']} op call, {r['E_und']} keyframe-pair edges "
                    f"({2 * r['E_und']} directed), {spec['N']} keyframes, {r['g'].H}x{r['g'].W}, "
                    f"{r['iters']} GN iters/step, delta_thresh=0",
        "directed_edges_this_rank": local,
        "n_ranks": world,
        "n_ranks_comm": comm_size(comm) if comm is not None else 1,
        "comm": (("host exchange (rehearsal)" if rehearse else "RCCL") if world > 1 else None),
        "phase_ms_per_iter": {
            "accumulate": acc_ms,
            "reduce_compact_allreduce": r["ph"][1] / nph,
            "solve": r["ph"][2] / nph,
            "retract": r["ph"][3] / nph,
        },
        "solve_path": _solve_path(r["solve_stats"], r["iters"], r["solve_ms"]),
        "accumulate_GBps": bytes_launch / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None,
        # the iteration kernel's per-launch events over the timed steps (interleaved with the
        # other phases of every call): quote cfg4 gains only beyond this spread
        "accumulate_launch_ms_spread": launch_spread(r["launch_ms"]),
        "accumulate_bytes_per_point_edge": bpe,
    }


def reference_order_block(g, mode, Twc0, args, iters, reps=3):
    """The price of parity: the same op call in the reference-order mode (gn_refacc.hip: the
    reference kernels' own float order and formulas) -- its throughput on
    this graph, and its poses after one iteration against the CPU oracle's."""
    import numpy as np

    import mast3r_slam_backends as mb

    L = dict(LOCAL, K=g.K, height=g.H, width=g.W)
    Twc = Twc0.clone()

    def call(n):
        Twc.copy_(Twc0)
        if mode == "calib":
            mb.gauss_newton_calib(Twc, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W,
                                  L["pixel_border"], L["depth_eps"], L["sigma_pixel"], L["sigma_depth"],
                                  L["C_conf"], L["Q_conf"], n, 0.0)
        else:
            mb.gauss_newton_rays(Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, L["sigma_ray"],
                                 L["sigma_dist"], L["C_conf"], L["Q_conf"], n, 0.0)

    prev = mb.set_gn_order("reference")
    try:
        call(iters)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            call(iters)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        call(1)
        T1 = Twc.cpu().numpy().astype(np.float64)
    finally:
        mb.set_gn_order(prev)
    To = np.asarray(cpu_baseline.last_poses, np.float64)
    E_und = g.ii.shape[0] // 2
    return {
        "value": E_und * iters / dt,
        "unit": "keyframe-pair GN iters/s",
        "ms_per_call": dt * 1e3,
        "calls_timed": reps,
        "pose_max_rel_err_vs_oracle_1iter": float(np.abs(T1 - To).max() / np.abs(To).max()),
    }


def stress_block(dev):
    """Mid-convergence parity, restated by every bench run: the headline
    topology started 10 deg / 25 cm / 0.1 log-scale from the truth with 10 % gross outlier matches
    (tests/test_gpu_gn_stress.py), ONE iteration.  The timed (fast) path's and the reference-order
    mode's poses against the CPU oracle (the reference's float order) and against the exactly summed
    system (the same float terms summed in double); sigma = the oracle's own distance from the
    exact sums, i.e. the reference order's rounding noise, below which no other order can land."""
    import numpy as np

    import mast3r_slam_backends as mb
    from m3s import synth
    from m3s.geometry import constrain_points_to_ray
    from oracle import oracle as O

    g = synth.make_graph("cfg3", device=dev, init_perturb=(10.0, 0.25, 0.1), outlier_frac=0.10)
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    L = LOCAL

    def gpu():
        Twc = g.Twc.clone()
        mb.gauss_newton_calib(Twc, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W,
                              L["pixel_border"], L["depth_eps"], L["sigma_pixel"], L["sigma_depth"],
                              L["C_conf"], L["Q_conf"], 1, 0.0)
        torch.cuda.synchronize()
        return Twc.cpu().numpy().astype(np.float64)

    T_fast = gpu()
    prev = mb.set_gn_order("reference")
    try:
        T_ref = gpu()
    finally:
        mb.set_gn_order(prev)
    c = lambda t: t.cpu().numpy()

    def params(n):
        return O.make_params("calib", L["sigma_pixel"], L["sigma_depth"], L["C_conf"], L["Q_conf"], K=c(g.K),
                             height=g.H, width=g.W, pixel_border=L["pixel_border"], z_eps=L["depth_eps"],
                             max_iter=n, delta_thresh=0.0)

    arrs = [c(t) for t in (g.Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q)]
    refs = {}
    for n in (1, 3):
        T_on = O.gauss_newton(params(n), *arrs)[0].astype(np.float64)
        with O.exact_sums():
            refs[n] = (T_on, O.gauss_newton(params(n), *arrs)[0].astype(np.float64))
    T_o, T_x = refs[1]
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    return {
        "graph": "cfg3 topology, 512x384, start 10 deg / 25 cm / 0.1 log-scale, 10 % outlier matches, 1 iteration",
        "path": "unpacked gn_accum_kernel (max_iter < 3); the timed packed kernel: timed_kernel",
        "fast_vs_oracle": rel(T_fast, T_o),
        "fast_vs_exact": rel(T_fast, T_x),
        "reference_order_vs_oracle": rel(T_ref, T_o),
        "sigma_oracle_vs_exact": rel(T_o, T_x),
        "timed_kernel": timed_kernel_parity(g, "calib", g.Twc, refs),
    }


def matching_bench(dev, reps=10):
    """Matching ops (SURVEY.md §8(d) 'matching pairs/s, B=1 and B=8'): iter_proj + refine_matches
    at 512x384 (inputs resident, base.yaml matching parameters), kernel time from events on the
    current stream; plus the whole match_iterative_proj call (the fused pipeline op, and the torch
    glue around the two ops for comparison).  Bytes per pixel as SURVEY
    §8(d): iter_proj 65 B, refine 128 B (+ the candidate gathers, served from L2/MALL)."""
    import mast3r_slam_backends as mb
    from m3s import synth
    from m3s.config import config as cfg0
    from m3s.matching import match_iterative_proj, prep_for_iter_proj

    mc = cfg0["matching"]
    res = {}
    for B in (1, 8):
        mp = synth.make_match_pair(B=B, H=384, W=512, seed=11, device=dev)
        rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
        b, h, w = mp.X21.shape[:3]
        D11 = mp.D11.half()
        D21 = mp.D21.view(b, h * w, -1).half()
        p1, _ = mb.iter_proj(rays, pts, p_init, mc["max_iter"], mc["lambda_init"], mc["convergence_thresh"])
        p1 = p1.long()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t_ip = t_rf = 0.0
        for r in range(reps + 2):
            ev[0].record()
            mb.iter_proj(rays, pts, p_init, mc["max_iter"], mc["lambda_init"], mc["convergence_thresh"])
            ev[1].record()
            mb.refine_matches(D11, D21, p1, mc["radius"], mc["dilation_max"])
            ev[2].record()
            torch.cuda.synchronize()
            if r >= 2:
                t_ip += ev[0].elapsed_time(ev[1]) / reps
                t_rf += ev[1].elapsed_time(ev[2]) / reps
        # A/Bs: the measurement-only refine variants (mast3r_slam_backends.variants: the LDS-tiled
        # kernel, the MFMA correlation with exact re-scoring, the dot2 bound-and-rescore)
        from mast3r_slam_backends import variants as mv

        def variant_ms(kind):
            t = 0.0
            for r in range(reps + 2):
                ev[1].record()
                mv.refine_matches_variant(kind, D11, D21, p1, mc["radius"], mc["dilation_max"])
                ev[2].record()
                torch.cuda.synchronize()
                if r >= 2:
                    t += ev[1].elapsed_time(ev[2]) / reps
            mv.variant_stats(True)
            mv.refine_matches_variant(kind, D11, D21, p1, mc["radius"], mc["dilation_max"])
            return t, mv.variant_stats(False)

        t_gather, _ = variant_ms(mv.LDS)
        t_mfma, (resc, cand) = variant_ms(mv.MFMA)
        t_exact, (resc_d, cand_d) = variant_ms(mv.DOT2)
        t_lat, (resc_l, cand_l) = variant_ms(mv.LATTICE)
        n_mfma_l = mv.mfma_issued()
        def wall_ms(fused):
            for _ in range(2):
                match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=fused)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=fused)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        t_glue = wall_ms(True)        # the fused pipeline op (csrc/match_glue.hip)
        t_torch_glue = wall_ms(False)  # the reference's torch glue around the two ops
        npx = B * h * w
        # the fused op's glue rounds like the reference's glue on the HOST (normalize / 3x3
        # conv); torch's GPU kernels round differently: how many matches that changes here
        i_f, v_f = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
        i_t, v_t = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=False)
        glue_diff = {"idx_differ": int((i_f != i_t).sum()), "valid_differ": int((v_f != v_t).sum()),
                     "pixels": npx}
        res[f"B{B}"] = {
            "pairs_per_s_kernels": B / ((t_ip + t_rf) * 1e-3),
            "pairs_per_s_glue": B / (t_glue * 1e-3),
            "iter_proj_ms": t_ip,
            "refine_ms": t_rf,
            "refine_dot2_rescore": {"ms": t_exact, "rescored_fraction": resc_d / max(cand_d, 1)},
            "refine_lds_tile_kernel_ms": t_gather,
            "refine_mfma": {
                "ms": t_mfma,
                "rescored_fraction": resc / max(cand, 1),
                # one 16x16x32 f16 MFMA per 16 (pixel, candidate) pairs (the diagonal), 245 pairs
                # per pixel; useful = the 245 x 24 MACs of the reference's correlation
                "mfma_issued_TFLOPs": 245 * 16384 / 16 * npx / (t_mfma * 1e-3) / 1e12,
                "useful_TFLOPs": 245 * 48 * npx / (t_mfma * 1e-3) / 1e12,
                "mfma_util_vs_2500TF": 245 * 16384 / 16 * npx / (t_mfma * 1e-3) / 2.5e15,
                "useful_util_vs_2500TF": 245 * 48 * npx / (t_mfma * 1e-3) / 2.5e15,
            },
            "refine_mfma_lattice": {
                # MFMA over per-level lattice buckets (refine_variants.hip): issued = the kernel's
                # count of 16x16x32 f16 MFMAs (16384 FLOP each); useful = the reference's MACs
                "ms": t_lat,
                "rescored_fraction": resc_l / max(cand_l, 1),
                "mfma_issued": n_mfma_l,
                "mfma_issued_TFLOPs": n_mfma_l * 16384 / (t_lat * 1e-3) / 1e12,
                "mfma_util_vs_2500TF": n_mfma_l * 16384 / (t_lat * 1e-3) / 2.5e15,
                "useful_TFLOPs": 245 * 48 * npx / (t_lat * 1e-3) / 1e12,
                "useful_util_vs_2500TF": 245 * 48 * npx / (t_lat * 1e-3) / 2.5e15,
            },
            "match_iterative_proj_ms": t_glue,
            "match_iterative_proj_torch_glue_ms": t_torch_glue,
            "fused_vs_torch_gpu_glue": glue_diff,
            "iter_proj_GBps": 65 * npx / (t_ip * 1e-3) / 1e9,
            "refine_GBps": 128 * npx / (t_rf * 1e-3) / 1e9,
            "refine_candidate_GBps": 245 * 48 * npx / (t_rf * 1e-3) / 1e9,
        }
    return res


def tracking_bench(dev, reps=20):
    """Frame tracking (tracker.py:173-266) as one track_sim3 op at 512x384, calib and rays:
    ms per frame with the reference's convergence test (base.yaml tracking), and ms per GN
    iteration with exactly 10 iterations.  Bytes per point and iteration: rays Xf 12 + Xk 12 +
    Q 4 + valid 1 = 29; calib Xf 12 + meas 12 + Q 4 + valid 1 + valid_meas 1 = 30."""
    import mast3r_slam_backends as mb
    from m3s.config import config as cfg0
    from m3s.synth import make_tracking_inputs

    c = cfg0["tracking"]
    res = {}
    for mode in ("calib", "rays"):
        p = make_tracking_inputs((384, 512), seed=21, mode=mode, device=dev)
        s0, s1 = (c["sigma_ray"], c["sigma_dist"]) if mode == "rays" else (c["sigma_pixel"], c["sigma_depth"])
        kw = {} if mode == "rays" else dict(meas_k=p["meas_k"], valid_meas_k=p["valid_meas_k"], K=p["K"],
                                            img_size=(384, 512), pixel_border=c["pixel_border"],
                                            z_eps=c["depth_eps"])

        def run(iters, rel, dn):
            return mb.track_sim3(mode, p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"],
                                 s0, s1, c["huber"], iters, rel, dn, **kw)

        out = {}
        for tag, (iters, rel, dn) in (("frame", (c["max_iters"], c["rel_error"], c["delta_norm"])),
                                      ("fixed10", (10, 0.0, 0.0))):
            for _ in range(3):
                run(iters, rel, dn)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                _, _, it, _ = run(iters, rel, dn)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            out[f"{tag}_ms"] = ms
            out[f"{tag}_iters"] = it
        bpp = 29 if mode == "rays" else 30
        out["ms_per_iter"] = out["fixed10_ms"] / 10
        out["frames_per_s"] = 1e3 / out["frame_ms"]
        out["GBps_per_iter"] = bpp * 384 * 512 / (out["ms_per_iter"] * 1e-3) / 1e9
        res[mode] = out
    return res


def _op_call(g, mode, Twc, n, env=None, order=None):
    """One op call of ``n`` iterations on ``Twc`` (in place) with temporary environment switches
    (read by the op per call) and/or summation order; returns (dx, debug flags of that call:
    [done, fail, packed stream, ray-constrained packed accumulate])."""
    import mast3r_slam_backends as mb

    env = dict(env or {}, M3S_GN_DEBUG_FLAGS="2")
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    prev = mb.set_gn_order(order) if order else None
    try:
        if mode == "calib":
            (dx,) = mb.gauss_newton_calib(Twc, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W,
                                          LOCAL["pixel_border"], LOCAL["depth_eps"], LOCAL["sigma_pixel"],
                                          LOCAL["sigma_depth"], LOCAL["C_conf"], LOCAL["Q_conf"], n, 0.0)
        else:
            (dx,) = mb.gauss_newton_rays(Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, LOCAL["sigma_ray"],
                                         LOCAL["sigma_dist"], LOCAL["C_conf"], LOCAL["Q_conf"], n, 0.0)
        torch.cuda.synchronize()
    finally:
        if order:
            mb.set_gn_order(prev)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    mb.gn_check()
    dbg = (ctypes.c_int * 4)()
    mb.lib.m3s_gn_debug_flags(dbg)
    return dx, list(dbg)


def timed_kernel_parity(g, mode, Twc0, refs):
    """Mid-convergence parity of the kernel the bench TIMES: a call of
    fewer than 3 iterations normally skips the packed stream (gn_driver.hip setup), so the
    1-iteration comparison is rerun with M3S_GN_PACK=2 -- the packed (calib: ray-constrained)
    accumulate the timed 10-iteration call runs -- and a 3-iteration call (packed by default)
    is added.  ``refs[n]`` = (oracle poses, exactly summed poses) after n iterations; sigma = the
    oracle's own distance from the exact sums (the reference order's fp32 rounding noise)."""
    import numpy as np

    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    out = {"path": f"gn_accum_packed_kernel<{mode}{', raycheck' if mode == 'calib' else ''}> "
                   "(M3S_GN_PACK=2 at 1 iteration; the default from 3)"}
    for n, (To, Tx) in sorted(refs.items()):
        To, Tx = np.asarray(To, np.float64), np.asarray(Tx, np.float64)
        T = Twc0.clone()
        _, dbg = _op_call(g, mode, T, n, env={"M3S_GN_PACK": "2"})
        Tf = T.cpu().numpy().astype(np.float64)
        T = Twc0.clone()
        _op_call(g, mode, T, n, order="reference")
        Tr = T.cpu().numpy().astype(np.float64)
        out[f"{n}iter"] = {
            "took_packed_stream": bool(dbg[2]),
            "took_ray_constrained_accumulate": bool(dbg[3]),
            "fast_vs_oracle": rel(Tf, To),
            "fast_vs_exact": rel(Tf, Tx),
            "reference_order_vs_oracle": rel(Tr, To),
            "sigma_oracle_vs_exact": rel(To, Tx),
        }
    return out


def accuracy(g, mode, Twc0, Twc_final, T_oracle_1, T_exact_1, T_oracle_full, iters, dx_oracle_1=None,
             dx_exact_1=None):
    """'ATE-RMSE vs ref' (BASELINE.json metric): the GPU op's poses after ONE iteration and the
    timed call's poses (``iters`` iterations) against the CPU oracle's (the reference backend
    restated) on the same inputs -- max relative error of the pose data and the Sim(3)-aligned
    ATE-RMSE of the keyframe positions (m3s.evaluate, evo_ape -as) -- and the ATE of the timed
    result against the synthetic ground truth."""
    import numpy as np

    import mast3r_slam_backends as mb
    from m3s.evaluate import ate_rmse

    T1 = Twc0.clone()
    if mode == "calib":
        (dx1,) = mb.gauss_newton_calib(T1, g.Xs, g.Cs, g.K, g.ii, g.jj, g.idx, g.valid, g.Q, g.H, g.W,
                              LOCAL["pixel_border"], LOCAL["depth_eps"], LOCAL["sigma_pixel"],
                              LOCAL["sigma_depth"], LOCAL["C_conf"], LOCAL["Q_conf"], 1, 0.0)
    else:
        (dx1,) = mb.gauss_newton_rays(T1, g.Xs, g.Cs, g.ii, g.jj, g.idx, g.valid, g.Q, LOCAL["sigma_ray"],
                             LOCAL["sigma_dist"], LOCAL["C_conf"], LOCAL["Q_conf"], 1, 0.0)
    T1 = T1.cpu().numpy().astype(np.float64)
    To = np.asarray(T_oracle_1, np.float64)
    Tx = np.asarray(T_exact_1, np.float64)
    rel = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())
    ts = np.arange(To.shape[0], dtype=np.float64)
    ate_o, _ = ate_rmse((ts, To[:, :3]), (ts, T1[:, :3]))
    gt = g.Twc_gt.cpu().numpy().astype(np.float64)
    fin = Twc_final.cpu().numpy().astype(np.float64)
    ate_gt, _ = ate_rmse((ts, gt[:, :3]), (ts, fin[:, :3]))
    ate_init, _ = ate_rmse((ts, gt[:, :3]), (ts, Twc0.cpu().numpy().astype(np.float64)[:, :3]))
    Tf = np.asarray(T_oracle_full, np.float64)
    ate_f, _ = ate_rmse((ts, Tf[:, :3]), (ts, fin[:, :3]))
    steps = {}
    if dx_exact_1 is not None:
        # the first step itself (accumulate + solve), relative to max |dx|: the poses after ONE
        # step also carry the reference's float Sim(3) exponential, which turns a 1e-7 change of
        # the log-scale step into ~1e-5 of a translation
        dxx = np.asarray(dx_exact_1, np.float64)
        steps = {"step_max_rel_err_vs_exact_sum_1iter": rel(dx1.cpu().numpy().astype(np.float64), dxx),
                 "reference_order_step_max_rel_err_vs_exact_sum_1iter": rel(np.asarray(dx_oracle_1, np.float64), dxx)}
    return {
        **steps,
        # (the *_1iter fields above and below run the call as the reference's callers would:
        # ONE iteration, which takes the unpacked accumulate; timed_kernel_parity prices the
        # packed kernel the timed calls run)
        "one_iteration_path": "unpacked gn_accum_kernel (max_iter < 3)",
        f"pose_max_rel_err_vs_oracle_{iters}iter_timed_call": rel(fin, Tf),
        f"ate_rmse_vs_oracle_{iters}iter_m": ate_f,
        "pose_max_rel_err_vs_oracle_1iter": rel(T1, To),
        # the same comparison against float terms summed in double: how far each summation
        # order (this op's, the reference's) is from the exactly summed system
        "pose_max_rel_err_vs_exact_sum_1iter": rel(T1, Tx),
        "reference_order_max_rel_err_vs_exact_sum_1iter": rel(To, Tx),
        "ate_rmse_vs_oracle_1iter_m": ate_o,
        "ate_rmse_vs_gt_m": {"initial": ate_init, "after_10_iters": ate_gt},
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _host_cores():
    """The host's CPUs as this process sees them: nproc (the machine), the affinity set, the cgroup
    CPU quota; ``usable`` = what the oracle's OpenMP pool is sized to (affinity, capped by the
    quota -- the GPU box gives a job a share of a larger machine)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable}


def cpu_baseline(g, mode, E_und, iters):
    """The CPU oracle (restatement of the reference backend, which has no CPU path) on a
    bounded sample: ONE GN iteration of the same graph (all directed edges, full 512x384),
    2 warm-ups then the median of 5 timed runs, OpenMP threads = every CPU
    this process may use (``_host_cores``: affinity set capped by the cgroup quota; nproc,
    affinity and quota are recorded beside it).  Also produces the accuracy references: the oracle's poses after 1 and
    after ``iters`` iterations, and after 1 iteration with the float terms summed in double."""
    import statistics

    from oracle import oracle as O

    c = lambda t: t.cpu().numpy()

    def params(n_iter):
        if mode == "calib":
            return O.make_params("calib", LOCAL["sigma_pixel"], LOCAL["sigma_depth"], LOCAL["C_conf"],
                                 LOCAL["Q_conf"], K=c(g.K), height=g.H, width=g.W,
                                 pixel_border=LOCAL["pixel_border"], z_eps=LOCAL["depth_eps"],
                                 max_iter=n_iter, delta_thresh=0.0)
        return O.make_params("rays", LOCAL["sigma_ray"], LOCAL["sigma_dist"], LOCAL["C_conf"],
                             LOCAL["Q_conf"], max_iter=n_iter, delta_thresh=0.0)

    arrs = [c(g.Twc), c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q)]
    hw = _host_cores()
    O.set_num_threads(hw["usable"])  # every core this process may run on
    P1 = params(1)
    times = []
    for r in range(7):
        t0 = time.perf_counter()
        T_o, dx_o, _ = O.gauss_newton(P1, *arrs)
        if r >= 2:
            times.append(time.perf_counter() - t0)
    dt = statistics.median(times)
    cpu_baseline.last_poses = T_o  # the accuracy check compares the GPU's first iteration
    cpu_baseline.last_step = dx_o
    with O.exact_sums():  # precision reference: the same float terms summed in double
        cpu_baseline.exact_poses, cpu_baseline.exact_step, _ = O.gauss_newton(P1, *arrs)
        T3x, _, _ = O.gauss_newton(params(3), *arrs)
    cpu_baseline.full_poses, _, _ = O.gauss_newton(params(iters), *arrs)
    T3o, _, _ = O.gauss_newton(params(3), *arrs)
    # oracle / exactly summed poses after 1 and 3 iterations (timed_kernel_parity)
    cpu_baseline.refs = {1: (T_o, cpu_baseline.exact_poses), 3: (T3o, T3x)}
    return {
        "value": E_und * 1 / dt,
        "unit": "keyframe-pair GN iters/s",
        "cores": O.num_threads(),
        "host": hw,
        "cpu_model": _cpu_model(),
        "kind": "port",
        "sample": f"1 GN iteration of the same graph ({E_und} pairs, {2 * E_und} directed edges, "
                  f"{g.H}x{g.W}) by the C oracle: 2 warm-ups, median of 5 = {dt:.3f} s wall "
                  f"(min {min(times):.3f}, max {max(times):.3f})",
    }


if __name__ == "__main__":
    main()
