"""GPU probe of the fused solve: fused vs the dense reference solver on several topologies
(one GN step), with per-phase device timings (M3S_SOLVE_DEBUG=1 prints from the kernel)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import mast3r_slam_backends as mb  # noqa: E402
from m3s import synth  # noqa: E402


def run(g, iters=1):
    Twc = g.Twc.clone().cuda()
    c = lambda t: t.cuda()
    (dx,) = mb.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q),
                                 0.003, 10.0, 0.0, 1.5, iters, 0.0)
    torch.cuda.synchronize()
    return dx.cpu().numpy()


def graph(topo):
    if topo == "chain":
        N = 24
        und = [(k - 1, k) for k in range(1, N)]
    elif topo.startswith("clique"):
        N = int(topo[6:])
        und = [(a, b) for a in range(N) for b in range(a + 1, N)]
    else:
        return synth.make_graph(topo, H=24, W=32, seed=int(os.environ.get("PROBE_SEED", "6")))
    return synth.make_graph(dict(N=N, E=len(und)), H=24, W=32, seed=3, edges_only=und)


for topo in sys.argv[1:] or ["chain", "clique3", "clique12", "cfg2", "cfg3"]:
    g = graph(topo)
    os.environ["M3S_SOLVER_DENSE"] = "1"
    d_ref = run(g)
    del os.environ["M3S_SOLVER_DENSE"]
    os.environ["M3S_SOLVE_FUSED"] = "0"
    d_ml = run(g)
    del os.environ["M3S_SOLVE_FUSED"]
    os.environ["M3S_SOLVE_DEBUG"] = os.environ.get("PROBE_DEBUG", "1")
    d_f = run(g)
    sys.stdout.flush()
    del os.environ["M3S_SOLVE_DEBUG"]
    s = max(np.abs(d_ref).max(), 1e-12)
    print(f"{topo}: |multilaunch-dense|/max {np.abs(d_ml - d_ref).max() / s:.3e}  "
          f"|fused-dense|/max {np.abs(d_f - d_ref).max() / s:.3e}", flush=True)
