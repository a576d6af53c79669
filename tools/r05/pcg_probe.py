"""PCG on the cfg4 GN systems with a lagged exact-inverse preconditioner: steps to
1e-10 of the direct solve per GN iteration, 48x64 pixels, the C oracle builds the systems.
    python tools/r05/pcg_probe.py [cfg4] [stress]"""
import os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
from oracle import oracle as orc
from m3s import synth
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
stress = len(sys.argv) > 2 and sys.argv[2] == "stress"
H, W = 48, 64
kw = dict(init_perturb=(10.0, 0.25, 0.1), outlier_frac=0.10) if stress else {}
g = synth.make_graph(cfg, H=H, W=W, **kw)
mode = g.mode
if mode == "rays":
    P = orc.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1, delta_thresh=0.0)
else:
    P = orc.make_params("calib", 1.0, 10.0, 0.0, 1.5, K=g.K.numpy(), height=H, width=W, pixel_border=-10, z_eps=1e-6, max_iter=1, delta_thresh=0.0)
Twc = g.Twc.numpy().copy()
args = (g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
def pcg(A, b, Minv, tol=1e-10, maxit=120, xref=None):
    x = np.zeros_like(b); r = b.copy(); z = Minv @ r; p = z.copy(); rz = r @ z
    hist = []
    for k in range(maxit):
        q = A @ p; a = rz / (p @ q); x += a * p; r -= a * q
        err = np.linalg.norm(x - xref) / np.linalg.norm(xref)
        hist.append(err)
        if err < tol: return k + 1, hist
        z = Minv @ r; rzn = r @ z; p = z + (rzn / rz) * p; rz = rzn
    return maxit, hist
M0 = None; Mprev = None
for it in range(10):
    Hk, bk = orc.gn_build_system(P, Twc, *args)
    xd = np.linalg.solve(Hk, bk)
    if it == 0:
        M0 = np.linalg.inv(Hk)
    else:
        n0, h0 = pcg(Hk, bk, M0, xref=xd)
        n1, h1 = pcg(Hk, bk, Mprev, xref=xd)
        dH = np.linalg.norm(np.eye(len(bk)) - M0 @ Hk, 2)
        print(f"it {it}: |dx|={np.linalg.norm(xd):.3e} cond={np.linalg.cond(Hk):.2e} ||I-M0H||={dH:.3e} pcg(M0) steps={n0} pcg(Mprev) steps={n1}  errs1={[f'{e:.1e}' for e in h1[:12]]}")
    Mprev = np.linalg.inv(Hk)
    Twc, dx, _ = orc.gauss_newton(P, Twc, *args)
