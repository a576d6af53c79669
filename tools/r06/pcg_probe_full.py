"""PCG step counts (M1: the iteration-1 inverse, fixed) on the GN systems at full size (round-6 verdict item 2): the oracle builds the
system of every iteration; PCG with the iteration-0 inverse (M0) and the previous iteration's
inverse (Mprev); reports the steps to relative errors 1e-3..1e-8 of the direct solve and the
preconditioned residual sqrt(r'z)/sqrt(b'Mb) at those steps (a device-side stop criterion).
    python tools/r06/pcg_probe_full.py cfg3|cfg4 [stress] [H W]"""
import os, sys, json, time, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
from oracle import oracle as orc
from m3s import synth
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
stress = len(sys.argv) > 2 and sys.argv[2] == "stress"
H, W = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (384, 512)
kw = dict(init_perturb=(10.0, 0.25, 0.1), outlier_frac=0.10) if stress else {}
g = synth.make_graph(cfg, H=H, W=W, **kw)
if g.mode == "rays":
    P = orc.make_params("rays", 0.003, 10.0, 0.0, 1.5, max_iter=1, delta_thresh=0.0)
else:
    P = orc.make_params("calib", 1.0, 10.0, 0.0, 1.5, K=g.K.numpy(), height=H, width=W,
                        pixel_border=-10, z_eps=1e-6, max_iter=1, delta_thresh=0.0)
Twc = g.Twc.numpy().copy()
args = (g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(), g.idx.numpy(), g.valid.numpy(), g.Q.numpy())
TOLS = [1e-3, 1e-4, 1e-5, 1e-6, 1e-8]
def pcg(A, b, Minv, xref, maxit=200):
    x = np.zeros_like(b); r = b.copy(); z = Minv @ r; p = z.copy(); rz = r @ z; rz0 = rz
    out = {}
    for k in range(maxit):
        q = A @ p; a = rz / (p @ q); x += a * p; r -= a * q
        err = np.linalg.norm(x - xref) / np.linalg.norm(xref)
        z = Minv @ r; rzn = r @ z
        for t in TOLS:
            if t not in out and err < t: out[t] = (k + 1, float(np.sqrt(max(rzn, 0) / rz0)))
        if err < TOLS[-1]: break
        p = z + (rzn / rz) * p; rz = rzn
    return {f"{t:.0e}": out.get(t) for t in TOLS}
res = []
M0 = Mprev = M1 = None
for it in range(10):
    t0 = time.time()
    Hk, bk = orc.gn_build_system(P, Twc, *args)
    xd = np.linalg.solve(Hk, bk)
    row = dict(it=it, dx=float(np.linalg.norm(xd)), build_s=round(time.time() - t0, 1))
    if it > 0:
        row["M0"] = pcg(Hk, bk, M0, xd)
        row["Mprev"] = pcg(Hk, bk, Mprev, xd)
        row["I-MprevH"] = float(np.linalg.norm(np.eye(len(bk)) - Mprev @ Hk, 2))
        if M1 is not None:
            row["M1"] = pcg(Hk, bk, M1, xd)
    else:
        M0 = np.linalg.inv(Hk)
        row["cond"] = float(np.linalg.cond(Hk))
    Mprev = np.linalg.inv(Hk)
    if it == 1:
        M1 = Mprev
    print(json.dumps(row), flush=True)
    res.append(row)
    Twc, dx, _ = orc.gauss_newton(P, Twc, *args)
