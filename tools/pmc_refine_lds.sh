#!/bin/bash
# PMC passes over refine_lds_kernel (the LDS-staged candidate box, measurement-only variant) and
# the product refine_f16_kernel at B=8, one counter group per rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_pmc_refine
export TMPDIR=/tmp
for v in 1 0; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -d' ' -f1)_v$v
    VARIANT=$v REPS=5 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/r04_pmc_refine/$tag -o run -- python tools/refine_probe.py > gpurun_out/r04_pmc_refine/$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_pmc_refine/trace1 -o run -- python tools/refine_probe.py > gpurun_out/r04_pmc_refine/trace1.log 2>&1 || exit 1
VARIANT=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_pmc_refine/trace2 -o run -- python tools/refine_probe.py > gpurun_out/r04_pmc_refine/trace2.log 2>&1 || exit 1
python - <<'PY' > gpurun_out/r04_pmc_refine/summary.txt
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04_pmc_refine/*/run_counter_collection.csv")):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "refine" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[2], {k: "%.4g" % (v / max(n[k], 1)) for k, v in acc.items()})
for f in sorted(glob.glob("gpurun_out/r04_pmc_refine/trace*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "refine" in r["Name"]:
            print(f.split("/")[2], r["Name"][:60], r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
cat gpurun_out/r04_pmc_refine/summary.txt
