"""Generate the tracker golden fixtures from the REFERENCE Python (dev container only).

Run from the repo root:  python tests/golden/make_track_golden.py
Writes tests/golden/track_golden.npz (inputs + reference outputs, small shapes).

Pinned (reference file:line): FrameTracker.opt_pose_ray_dist_sim3 (tracker.py:173-214) and
opt_pose_calib_sim3 (:216-266) with their solve (:156-171), check_convergence / huber
(nonlinear_optimizer.py:5-33) and act_Sim3 / point_to_ray_dist / project_calib
(geometry.py:17-104), run as written in float32 torch on CPU.  lietorch is absent: the
reference code is driven through oracle.track_oracle.Sim3T, a restatement of lietorch's Sim3
group, so the group operations themselves stay unpinned (see oracle/track_oracle.py).

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
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]

from oracle import track_oracle as TO  # noqa: E402


def install_stubs():
    lt = types.ModuleType("lietorch")
    lt.Sim3 = TO._torch_sim3()
    sys.modules["lietorch"] = lt
    mu = types.ModuleType("mast3r_slam.mast3r_utils")
    mu.mast3r_match_asymmetric = None
    mu.mast3r_match_symmetric = None
    mu.resize_img = None
    sys.modules["mast3r_slam.mast3r_utils"] = mu
    sys.path.insert(0, REF)
    return lt.Sim3


def main():
    Sim3 = install_stubs()
    from mast3r_slam import config as rcfg
    from mast3r_slam import tracker as rtr

    rcfg.load_config(os.path.join(REF, "config", "base.yaml"))
    trk = rtr.FrameTracker(None, None, "cpu")
    out = {}
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    for case, (mode, seed, noise) in enumerate((("rays", 1, 0.0), ("rays", 2, 0.003),
                                                ("calib", 3, 0.0), ("calib", 4, 0.003))):
        p = TO.make_tracking_pair((24, 32), seed=seed, mode=mode, noise=noise)
        Tf = Sim3(t(p["T_WCf"]).reshape(1, 8))
        Tk = Sim3(t(p["T_WCk"]).reshape(1, 8))
        if mode == "rays":
            T_WCf, T_CkCf = trk.opt_pose_ray_dist_sim3(t(p["Xf"]), t(p["Xk"]), Tf, Tk, t(p["Qk"]),
                                                       t(p["valid"]))
        else:
            T_WCf, T_CkCf = trk.opt_pose_calib_sim3(t(p["Xf"]), t(p["Xk"]), Tf, Tk, t(p["Qk"]),
                                                    t(p["valid"]), t(p["meas_k"]),
                                                    t(p["valid_meas_k"]), t(p["K"]), (24, 32))
        for k, v in p.items():
            out[f"c{case}_{k}"] = v
        out[f"c{case}_mode"] = np.array(mode)
        out[f"c{case}_out_T_WCf"] = T_WCf.data.numpy().reshape(8)
        out[f"c{case}_out_T_CkCf"] = T_CkCf.data.numpy().reshape(8)
    out["ncases"] = np.array(4)
    np.savez_compressed(os.path.join(HERE, "track_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "track_golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
