"""Generate the add_factors golden fixtures from the REFERENCE Python (dev container only).

Run from the repo root:  python tests/golden/make_edges_golden.py
Writes tests/golden/edges_golden.npz.

Pinned (reference file:line): FactorGraph.add_factors after the network
(mast3r_slam/global_opt.py:53-99): Qj/Qi from the gathered confidences, the Q_conf gating, the
per-pair match fractions, the min_match_frac test that keeps consecutive keyframes, and the
resulting edge store (ii, jj, idx_ii2jj, idx_jj2ii, valid_match_j/i, Q_ii2jj/jj2ii), run as
written on CPU.  mast3r_match_symmetric (the network) is replaced by a stub returning
synthetic matches; lietorch / the backend are stubs (unused on this path).

The reference is read from /root/reference at generation time only; nothing under tests/
imports it at run time, and no reference source is copied.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def synthetic_matches(B, HW, seed):
    g = torch.Generator().manual_seed(seed)
    idx_i2j = torch.randint(0, HW, (B, HW), generator=g)
    idx_j2i = torch.randint(0, HW, (B, HW), generator=g)
    vj = torch.rand((B, HW, 1), generator=g) > 0.3
    vi = torch.rand((B, HW, 1), generator=g) > 0.3
    # per-pair confidence scales so some pairs fail the min_match_frac test
    scale = torch.linspace(0.3, 3.0, B)[:, None, None]
    Q = [torch.exp(torch.randn((B, HW, 1), generator=g) * 0.5) * scale for _ in range(4)]
    return idx_i2j, idx_j2i, vj, vi, Q[0], Q[1], Q[2], Q[3]


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from oracle.track_oracle import _torch_sim3

    lt = types.ModuleType("lietorch")
    lt.Sim3 = _torch_sim3()  # unused on this path; frame.py needs Sim3.Identity at import
    sys.modules["lietorch"] = lt
    mu = types.ModuleType("mast3r_slam.mast3r_utils")
    state = {}
    mu.mast3r_match_symmetric = lambda *a, **k: state["out"]
    mu.mast3r_match_asymmetric = None
    mu.resize_img = None
    sys.modules["mast3r_slam.mast3r_utils"] = mu
    sys.modules["mast3r_slam_backends"] = types.ModuleType("mast3r_slam_backends")
    sys.path.insert(0, REF)
    from mast3r_slam import config as rcfg
    from mast3r_slam import global_opt as rgo

    rcfg.load_config(os.path.join(REF, "config", "base.yaml"))

    class Frames:
        def __getitem__(self, i):
            return types.SimpleNamespace(feat=torch.zeros(1, 1), pos=torch.zeros(1, 1), img_true_shape=None)

    out = {}
    fg = rgo.FactorGraph(None, Frames(), device="cpu")
    HW = 12 * 16
    calls = [([0, 1, 2, 5], [1, 2, 3, 9], 11, False), ([0, 3, 4], [7, 4, 8], 12, False),
             ([2, 6], [7, 9], 13, True)]
    for c, (ii, jj, seed, reloc) in enumerate(calls):
        m = synthetic_matches(len(ii), HW, seed)
        state["out"] = m
        ret = fg.add_factors(ii, jj, rcfg.config["local_opt"]["min_match_frac"], is_reloc=reloc)
        names = ["idx_i2j", "idx_j2i", "valid_match_j", "valid_match_i", "Qii", "Qjj", "Qji", "Qij"]
        for n, t in zip(names, m):
            out[f"c{c}_{n}"] = t.numpy()
        out[f"c{c}_ii"], out[f"c{c}_jj"] = np.array(ii), np.array(jj)
        out[f"c{c}_reloc"] = np.array(reloc)
        out[f"c{c}_ret"] = np.array(bool(ret))
        for n in ["ii", "jj", "idx_ii2jj", "idx_jj2ii", "valid_match_j", "valid_match_i", "Q_ii2jj", "Q_jj2ii"]:
            out[f"c{c}_store_{n}"] = getattr(fg, n).numpy()
    out["ncalls"] = np.array(len(calls))
    out["min_match_frac"] = np.array(rcfg.config["local_opt"]["min_match_frac"])
    np.savez_compressed(os.path.join(HERE, "edges_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "edges_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
