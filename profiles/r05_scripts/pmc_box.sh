#!/bin/bash
# PMC passes over refine_box_kernel (VARIANT=5) and the product refine_f16_kernel at B=8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
for v in 5 0; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -d' ' -f1)_v$v
    VARIANT=$v REPS=5 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/$tag -o run -- python tools/refine_probe.py > $O/$tag.log 2>&1
    rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python - <<'PY' > $O/summary.txt
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r05j/*/run_counter_collection.csv")):
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "refine" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[2], {k: "%.4g" % (v / max(n[k], 1)) for k, v in acc.items()})
PY
cat $O/summary.txt
