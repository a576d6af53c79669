#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; after a fault / abort / timeout nothing else
# touches the GPU (exit codes 0 = pass, 1 = test failures are the only ones we go on from).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"

ok_or_fail() {  # $1 = rc, $2 = label
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
        echo "STOP after $2 (rc=$1): no further GPU steps"
        exit "$1"
    fi
}

for s in $STEPS; do
    case "$s" in
    tests)
        timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider \
            > gpurun_out/pytest_gpu.log 2>&1
        rc=$?; echo "pytest gpu rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
        ok_or_fail $rc pytest ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
        rc=$?; echo "smoke rc=$rc"; tail -n 5 gpurun_out/smoke.log
        ok_or_fail $rc smoke ;;
    bench)
        timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
        rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -n 5 gpurun_out/bench.err
        ok_or_fail $rc bench ;;
    benchdense)
        M3S_SOLVER_DENSE=1 timeout -k 10 600 python bench.py --no-cpu-baseline \
            > gpurun_out/bench_dense.json 2> gpurun_out/bench_dense.err
        rc=$?; echo "bench (dense solver) rc=$rc"; cat gpurun_out/bench_dense.json
        ok_or_fail $rc benchdense ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
            -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
            > gpurun_out/prof.log 2>&1
        rc=$?; echo "rocprof rc=$rc"; tail -n 5 gpurun_out/prof.log
        ok_or_fail $rc rocprof ;;
    esac
done
exit 0
