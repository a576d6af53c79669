#!/bin/bash
# switch-equivalence tests + cfg4 kernel stats of the round-5 tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_switches.py > $O/pytest_switches.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_switches.log; exit 1; }
tail -5 $O/pytest_switches.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > $O/cfg4_rocprof.json 2> $O/cfg4_rocprof.err || { echo "rocprof rc=$?"; tail -5 $O/cfg4_rocprof.err; exit 1; }
rm -f $O/prof/*kernel_trace.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'm3s' in r['Name']: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), r['Percentage'][:5])
"
