import os, sys
sys.path[:0] = ['/root/repo', '/root/repo/mast3r-slam_amd']
import numpy as np, torch
sys.argv = ['x', 'clique3']
from m3s.debug import build_system_gpu
from m3s import synth
N=3; und=[(a,b) for a in range(N) for b in range(a+1,N)]
g = synth.make_graph(dict(N=N, E=len(und)), H=24, W=32, seed=3, edges_only=und)
L = dict(sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, sigma_point=0.05, C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6)
H, b = build_system_gpu(g, "rays", L)
np.set_printoptions(precision=6, linewidth=200)
print("H00 diag", np.diag(H)[:7])
S = H[7:, 7:] - H[7:, :7] @ np.linalg.solve(H[:7, :7], H[:7, 7:])
print("Schur block K=1:\n", S)
print("eig", np.linalg.eigvalsh(S))
os.environ["M3S_SOLVE_DEBUG"] = "2"
exec(open('/root/repo/tools/solve_probe.py').read().split("for topo in")[0])
run(g)
