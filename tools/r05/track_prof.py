"""Tracker timing probe: track_sim3 on the bench's 512x384 frame (calib and rays), per call wall
time for the frame setting (reference convergence test) and for 10 fixed iterations, with and
without the host's intermediate convergence checks.  Run under rocprofv3 --kernel-trace --stats
for the kernels' own durations."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "mast3r-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import mast3r_slam_backends as mb  # noqa: E402
from m3s.config import config as cfg0  # noqa: E402
from m3s.synth import make_tracking_inputs  # noqa: E402

dev = torch.device("cuda", 0)
c = cfg0["tracking"]
res = {}
for mode in ("calib", "rays"):
    p = make_tracking_inputs((384, 512), seed=21, mode=mode, device=dev)
    s0, s1 = (c["sigma_ray"], c["sigma_dist"]) if mode == "rays" else (c["sigma_pixel"], c["sigma_depth"])
    kw = {} if mode == "rays" else dict(meas_k=p["meas_k"], valid_meas_k=p["valid_meas_k"], K=p["K"],
                                        img_size=(384, 512), pixel_border=c["pixel_border"], z_eps=c["depth_eps"])
    for tag, (iters, rel, dn) in (("frame", (c["max_iters"], c["rel_error"], c["delta_norm"])),
                                  ("fixed10", (10, 0.0, 0.0))):
        run = lambda: mb.track_sim3(mode, p["Xf"], p["Xk"], p["T_WCf"], p["T_WCk"], p["Qk"], p["valid"],
                                    s0, s1, c["huber"], iters, rel, dn, **kw)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            out = run()
        torch.cuda.synchronize()
        res[f"{mode}_{tag}_ms"] = (time.perf_counter() - t0) / 30 * 1e3
        res[f"{mode}_{tag}_iters"] = int(out[2])
print(json.dumps(res), flush=True)
