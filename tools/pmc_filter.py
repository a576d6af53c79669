"""Shrink rocprofv3 PMC output in place: keep only the m3s kernels' rows of every
run_counter_collection.csv under the given directory (the torch kernels of the bench's
setup dominate the file size), so gpurun_out/ stays under the copy-back limit."""
import csv
import os
import sys

root = sys.argv[1]
for dp, _, files in os.walk(root):
    for f in files:
        p = os.path.join(dp, f)
        if f.endswith("counter_collection.csv"):
            rows = list(csv.DictReader(open(p)))
            keep = [r for r in rows if "m3s::" in r.get("Kernel_Name", "") or "reduce_kernel" in r.get("Kernel_Name", "") or "FillFunc" in r.get("Kernel_Name", "")]
            with open(p, "w", newline="") as fh:
                if rows:
                    w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
                    w.writeheader()
                    w.writerows(keep)
        elif f.endswith(".csv") and ("kernel_trace" in f or "memory_copy" in f):
            os.remove(p)
