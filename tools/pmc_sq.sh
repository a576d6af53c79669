#!/bin/bash
# Issue/stall and L2 counters of the GN kernels (rocprofv3 --pmc, kernel-trace only, one pass
# per counter group).  Output: gpurun_out/pmc_sq/<pass>/run_counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
CFG="${CFG:-cfg3}"
run_pass() {  # $1 = pass name, rest = counters
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
        python bench.py --config $CFG --steps 1 --warmup 0 --iters 3 --no-cpu-baseline --no-matching \
        > $OUT/$name.log 2>&1
    local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
run_pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run_pass tcc TCC_HIT_sum TCC_MISS_sum &&
run_pass lds SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES
python tools/pmc_filter.py $OUT
