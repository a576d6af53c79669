#!/bin/bash
# Issue / stall counters of the single-workgroup solve kernel (gn_solve_kernel) on the cfg3
# topology (tools/solve_debug.py: 2 calls x 10 iterations), one rocprofv3 --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-r03h}"
OUT=gpurun_out/${TAG}_pmc_solve
mkdir -p $OUT
CFG="${CFG:-cfg3}"
run_pass() {  # $1 = pass name, rest = counters
    local name=$1; shift
    M3S_SOLVE_DEBUG=0 timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex gn_solve_kernel \
        --output-format csv -d $OUT/$name -o run -- python tools/solve_debug.py $CFG 10 2 > $OUT/$name.log 2>&1
    local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run_pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    SQ_INSTS_LDS SQ_WAVES &&
run_pass sq2 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
python - <<'PY'
import csv, glob, collections, os
out = os.environ.get("OUT_DIR")
PY
for f in $OUT/*/run_counter_collection.csv; do
    python -c "
import csv,collections,sys
s=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    s[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k in sorted(s): print('%-22s %14.0f  (%d records)'%(k,s[k],n[k]))
"
done
