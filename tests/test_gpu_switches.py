"""Round-5 performance switches are bitwise no-ops on the results (each read once per process, so
each setting runs in its own child process):
  * M3S_DF_XGRAN   -- chol_df's back-substitution hands x over as data-tagged granules (1, default)
                      or through ready words (0);
  * M3S_MULTI_DCAP -- the multi plan's elimination degree cap (32 default; 16 = round 4): another
                      ordering, so equal only to the f64 solve's rounding (poses to 1e-6);
  * M3S_IP_XCD     -- iter_proj's XCD-banded block order (1, default) or pixel order (0);
  * M3S_IP_SKIP    -- iter_proj skips the trial gather of a step that rounds to zero (1; default:
                      on launches of >= 2^19 pixels) or always gathers (0);
  * M3S_MATCH_PLANES -- the fused matching op's plane-major fp16 D11 + refine (1, default) or the
                      interleaved copy + refine_f16_kernel (0)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GN_CHILD = r"""
import sys, json; sys.path[:0] = [%r, %r]
import numpy as np, torch
import mast3r_slam_backends as mb
from m3s import synth
g = synth.make_graph("cfg4", H=24, W=32, seed=6)
Twc = g.Twc.clone().cuda()
c = lambda t: t.cuda()
mb.gauss_newton_rays(Twc, c(g.Xs), c(g.Cs), c(g.ii), c(g.jj), c(g.idx), c(g.valid), c(g.Q), 0.003, 10.0, 0.0, 1.5, 4, 0.0)
mb.gn_check()
print(json.dumps(Twc.cpu().numpy().astype(float).tolist()))
"""

MATCH_CHILD = r"""
import sys, json; sys.path[:0] = [%r, %r]
import torch
from m3s import synth
from m3s.matching import match_iterative_proj
import mast3r_slam_backends as mb
from m3s.matching import prep_for_iter_proj
mp = synth.make_match_pair(B=2, H=96, W=128, seed=5, device="cuda")
idx, valid = match_iterative_proj(mp.X11, mp.X21, mp.D11, mp.D21, mp.idx_init, fused=True)
rays, pts, p_init = prep_for_iter_proj(mp.X11, mp.X21, mp.idx_init)
p, conv = mb.iter_proj(rays, pts, p_init, 10, 1e-8, 1e-6)
torch.cuda.synchronize()
print(json.dumps([idx.cpu().tolist(), valid.cpu().int().tolist(), p.cpu().double().tolist(), conv.cpu().int().tolist()]))
"""


def _run(code, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code % (ROOT, os.path.join(ROOT, "mast3r-slam_amd"))], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_granule_x_handoff_is_bitwise_the_ready_words():
    base = dict(M3S_SOLVER="2", M3S_CHOL_DF="1")
    a = np.array(_run(GN_CHILD, dict(base, M3S_DF_XGRAN="1")))
    b = np.array(_run(GN_CHILD, dict(base, M3S_DF_XGRAN="0")))
    assert np.array_equal(a, b)


def test_elimination_degree_cap_changes_only_rounding():
    base = dict(M3S_SOLVER="2", M3S_CHOL_DF="1")
    a = np.array(_run(GN_CHILD, dict(base, M3S_MULTI_DCAP="32")))
    b = np.array(_run(GN_CHILD, dict(base, M3S_MULTI_DCAP="16")))
    assert np.abs(a - b).max() / np.abs(b).max() < 1e-6


def test_matching_switches_are_bitwise_noops():
    ref = _run(MATCH_CHILD, dict(M3S_IP_XCD="1", M3S_MATCH_PLANES="1"))
    for env in (dict(M3S_IP_XCD="0", M3S_MATCH_PLANES="1"), dict(M3S_IP_XCD="1", M3S_MATCH_PLANES="0"),
                dict(M3S_IP_SKIP="0"), dict(M3S_IP_SKIP="1")):
        assert _run(MATCH_CHILD, env) == ref, env
