#!/bin/bash
# Solve check: the GN GPU tests, the in-kernel phase clocks (entry / phases / exit), the call's
# rocprofv3 kernel durations without the debug clocks, and a short cfg3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r03e}"
CFG="${CFG:-cfg3}"
STEPS="${STEPS:-gntests dbg prof qbench}"
for s in $STEPS; do
case "$s" in
gntests)
timeout -k 10 500 python -u -m pytest tests/test_gpu_gn.py tests/test_gpu_factor_graph.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gn.log 2>&1 || { echo "gn tests failed"; tail -n 30 gpurun_out/${TAG}_pytest_gn.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_pytest_gn.log ;;
dbg2)
timeout -k 10 120 python tools/solve_debug.py cfg2 3 > gpurun_out/${TAG}_solve_cfg2.log 2>&1 || { echo "solve_debug cfg2 failed"; tail gpurun_out/${TAG}_solve_cfg2.log; exit 1; }
grep -v " K: " gpurun_out/${TAG}_solve_cfg2.log | tail -n 12 ;;
tl)
VARIANTS="" TAG=${TAG} bash tools/gpu_tdiag.sh ;;
dbg0)
M3S_SOLVE_WARM=0 timeout -k 10 120 python tools/solve_debug.py $CFG 3 > gpurun_out/${TAG}_solve_${CFG}_nowarm.log 2>&1 || { echo "solve_debug failed"; exit 1; }
grep -v " K: " gpurun_out/${TAG}_solve_${CFG}_nowarm.log | tail -n 10 ;;
dbg)
timeout -k 10 120 python tools/solve_debug.py $CFG 3 > gpurun_out/${TAG}_solve_${CFG}.log 2>&1 || { echo "solve_debug failed"; tail gpurun_out/${TAG}_solve_${CFG}.log; exit 1; }
grep -v " K: " gpurun_out/${TAG}_solve_${CFG}.log | tail -n 10 ;;
prof0)
M3S_SOLVE_WARM=0 M3S_SOLVE_DEBUG=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_solveprof0 -o run \
    -- python tools/solve_debug.py $CFG 10 10 > gpurun_out/${TAG}_solveprof0.log 2>&1 || { echo "rocprof failed"; exit 1; }
rm -f gpurun_out/${TAG}_solveprof0/*kernel_trace.csv
grep -h -E "solve" gpurun_out/${TAG}_solveprof0/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-160 ;;
prof)
M3S_SOLVE_DEBUG=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_solveprof -o run \
    -- python tools/solve_debug.py $CFG 10 10 > gpurun_out/${TAG}_solveprof.log 2>&1 || { echo "rocprof failed"; exit 1; }
rm -f gpurun_out/${TAG}_solveprof/*kernel_trace.csv
grep -h -E "solve|sp_|chol|assemble|compact" gpurun_out/${TAG}_solveprof/*kernel_stats.csv | cut -d, -f1-4 | cut -c1-160 ;;
qbench)
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching > gpurun_out/${TAG}_qbench.json 2> gpurun_out/${TAG}_qbench.err || { echo "qbench failed"; tail gpurun_out/${TAG}_qbench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_qbench.json'));print(d['value'],d['ms_per_step'],d['phase_ms_per_iter'])" ;;
esac
done
