#!/bin/bash
# PMC passes over iter_proj_kernel at B=8 (one counter group per rocprofv3 run) + its kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_pmc_iter_proj
mkdir -p $O
export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/$tag -o run -- python tools/iter_proj_probe.py > $O/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/iter_proj_probe.py > $O/trace.log 2>&1 || exit 1
find $O/trace -type f ! -name "*kernel_stats.csv" -delete
python - <<'PY' > $O/summary.txt
import csv, glob, collections
O = "gpurun_out/r04_pmc_iter_proj"
for f in sorted(glob.glob(O + "/*/run_counter_collection.csv")):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "iter_proj" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[2], {k: "%.4g" % (v / max(n[k], 1)) for k, v in acc.items()})
for f in glob.glob(O + "/trace/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "iter_proj" in r["Name"]:
            print(r["Name"][:50], r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
cat $O/summary.txt
