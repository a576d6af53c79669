#!/bin/bash
# HBM traffic of the GN accumulate kernel from rocprofv3 PMC counters, in two separate
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), plus a calibration
# pass on known-byte kernels (tools/ubench_copy.hip).  Kernel-trace only: no sys/runtime
# tracing is combined with --pmc.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CFG="${CFG:-cfg3}"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_$c -o run -- \
        python bench.py --config $CFG --steps 1 --warmup 0 --iters 3 --no-cpu-baseline --no-cfg4 --no-matching \
        > $OUT/bench_$c.log 2>&1
    rc=$?; echo "pmc $c bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d $OUT/calib_$c -o run -- \
        python tools/pmc_calib.py > $OUT/calib_$c.log 2>&1
    rc=$?; echo "pmc $c calib rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_filter.py $OUT
python tools/parse_pmc.py $OUT gpurun_out/accum_traffic_$CFG.json $CFG
exit 0
