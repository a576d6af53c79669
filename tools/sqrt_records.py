"""Counts the cfg3 bench graph's point records whose sqrt(q) differs between v_sqrt_f32 and the
correctly rounded sqrtf (tools/sqrt_records.hip).  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam_amd")]
import torch  # noqa: E402

from m3s import synth  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libsqrt_records.so"))
out = {}
for cfg in ("cfg3",):
    g = synth.make_graph(cfg, H=384, W=512, seed={"cfg3": 3, "cfg4": 4}[cfg])
    q = g.Q.float().contiguous().cuda()
    res = (ctypes.c_ulonglong * 2)()
    rc = lib.count_sqrt_diff(ctypes.c_void_p(q.data_ptr()), ctypes.c_int64(q.numel()), res)
    assert rc == 0
    out[cfg] = {"differing": res[0], "counted": res[1], "fraction": res[0] / max(res[1], 1)}
print(json.dumps(out))
