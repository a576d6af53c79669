"""Turn the rocprofv3 PMC passes of tools/pmc_traffic.sh into per-launch HBM traffic of the
GN accumulate kernel (profiles/accum_traffic.json, read by bench.py's roofline.traffic).

Correction (MI355X_MICROARCH.md §HBM, re-measured by tools/pmc_calib.py in the same run):
FETCH_SIZE counts 64 B per 128-B request, so read bytes = FETCH_SIZE[KB] * 1024 * k_fetch with
k_fetch = known bytes / counted bytes of the calibration's coalesced-stream kernel (~2.0);
WRITE_SIZE is exact for 16-B/lane stores (calibrated on the fill kernel).
"""
import csv
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/accum_traffic.json"
cfg = sys.argv[3] if len(sys.argv) > 3 else "cfg3"


def load(which, counter):
    rows = list(csv.DictReader(open(os.path.join(root, f"{which}_{counter}", "run_counter_collection.csv"))))
    agg = defaultdict(list)
    for r in rows:
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


cal_f = load("calib", "FETCH_SIZE")
cal_w = load("calib", "WRITE_SIZE")
reduce_kb = [v for k, v in cal_f.items() if "reduce_kernel" in k][0][0]
k_fetch = (1 << 30) / (reduce_kb * 1024.0)
fill_kb = [v for k, v in cal_w.items() if "FillFunc" in k][0][0]
k_write = (1 << 30) / (fill_kb * 1024.0)
bf = load("bench", "FETCH_SIZE")
bw = load("bench", "WRITE_SIZE")
# the steady-state packed accumulate of this config's mode (calib 2, rays 1, points 0): not the
# call's first launch (FIRST = true, which also builds the records), the most-launched name
mode = {"cfg3": "2", "cfg4": "1"}.get(cfg, "2")
names = [k for k in bf if "gn_accum" in k]
steady = [k for k in names if f"gn_accum_packed_kernel<{mode}," in k and not k.split(">")[0].endswith("true")]
name = max(steady or [k for k in names if "packed" in k] or names, key=lambda k: len(bf[k]))
fetch_kb = sum(bf[name]) / len(bf[name])
write_kb = sum(bw[name]) / len(bw[name])
read_b = fetch_kb * 1024 * k_fetch
write_b = write_kb * 1024 * k_write
# the accumulate path the profiled bench run took (its JSON line's roofline.stream)
stream = None
for line in open(os.path.join(root, "bench_FETCH_SIZE.log")):
    if line.startswith("{"):
        stream = json.loads(line).get("roofline", {}).get("stream")
res = {
    "config": cfg,
    "stream": stream,
    "n_gpus": 1,
    "kernel": name,
    "packed": "packed" in name,
    "launches": len(bf[name]),
    "FETCH_SIZE_KB_per_launch": fetch_kb,
    "WRITE_SIZE_KB_per_launch": write_kb,
    "k_fetch_calibrated": k_fetch,
    "k_write_calibrated": k_write,
    "hbm_read_bytes_per_launch": read_b,
    "hbm_write_bytes_per_launch": write_b,
    "hbm_bytes_per_launch": read_b + write_b,
    "note": "Infinity-Cache hits are counted by FETCH_SIZE on gfx950; bytes are memory-side requests",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
