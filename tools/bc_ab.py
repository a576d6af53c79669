"""Batch-cyclic vs column-cyclic chol_df on the GN stress graph: poses after 1..10 iterations
from each library (M3S_BACKEND_LIB), compared with each other and with the oracle."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
OUT = os.path.join(ROOT, "gpurun_out")
ITERS = [1, 2, 3, 5, 10]


def child(tag):
    import torch
    import mast3r_slam_backends as mb
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_gn_stress import STRESS, _gpu
    from m3s import synth
    from m3s.geometry import constrain_points_to_ray
    g = synth.make_graph("cfg3", **STRESS)
    g.Xs = constrain_points_to_ray((g.H, g.W), g.Xs, g.K).contiguous()
    res = {f"i{it}": _gpu(mb, g, it) for it in ITERS}
    np.savez(os.path.join(OUT, f"bc_ab_{tag}.npz"), **res)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1])
        sys.exit(0)
    os.makedirs(OUT, exist_ok=True)
    libs = {"new": None, "bc0": os.path.join(ROOT, "tools", "bin", "libm3s_backend_bc0.so")}
    for tag, lib in libs.items():
        env = dict(os.environ)
        env.pop("M3S_BACKEND_LIB", None)
        if lib:
            env["M3S_BACKEND_LIB"] = lib
        r = subprocess.run([sys.executable, __file__, tag], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)
    a, b = np.load(os.path.join(OUT, "bc_ab_new.npz")), np.load(os.path.join(OUT, "bc_ab_bc0.npz"))
    for it in ITERS:
        x, y = a[f"i{it}"].astype(np.float64), b[f"i{it}"].astype(np.float64)
        print(f"iters {it}: max |new - bc0| / max|bc0| = {np.abs(x - y).max() / np.abs(y).max():.3e}, "
              f"bitwise equal {np.array_equal(a[f'i{it}'], b[f'i{it}'])}")
