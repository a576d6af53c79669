"""PCG tolerance probe: poses of the PCG path at two CG tolerances against the direct solve and
the oracle (cfg3 / cfg4 topologies, 10 iterations).  python tools/r06/tol_probe.py TOL"""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
if len(sys.argv) > 2:  # child: one configuration
    import numpy as np, torch
    import mast3r_slam_backends as mb
    from tests.test_gpu_gn import _run_gpu, _run_oracle, _rel
    from tests.test_gpu_pcg import _graph
    from oracle import oracle as O
    from m3s import synth
    cfg, H, W = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    g = _graph(cfg, H, W)
    mode = synth.CONFIGS[cfg]["mode"]
    os.environ["M3S_GN_DEBUG_FLAGS"] = "2"
    T_p, _ = _run_gpu(mb, g, mode, 10)
    st = mb.gn_debug_flags()
    os.environ["M3S_GN_PCG"] = "0"
    T_d, _ = _run_gpu(mb, g, mode, 10)
    T_o, _, _ = _run_oracle(O, g, mode, 10)
    print(f"tol {os.environ.get('M3S_PCG_TOL')} {cfg} {H}x{W}: pcg vs direct {_rel(T_p, T_d):.2e}, pcg vs oracle {_rel(T_p, T_o):.2e}, direct vs oracle {_rel(T_d, T_o):.2e}, steps {st['pcg_steps']}/{st['pcg_runs']}", flush=True)
    sys.exit(0)
for cfg, H, W in (("cfg3", 96, 128), ("cfg4", 48, 64), ("cfg3", 384, 512), ("cfg4", 384, 512)):
    env = dict(os.environ, M3S_PCG_TOL=sys.argv[1])
    r = subprocess.run([sys.executable, __file__, sys.argv[1], cfg, str(H), str(W)], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    print(r.stdout.strip() or r.stderr[-1500:], flush=True)
