#!/bin/bash
# round-6 closing tree: full GPU suite + smoke + default bench + rocprof stats of the default command + PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06final${1:-}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'roofline frac', d['roofline']['frac'], d.get('solve_path'), 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), c.get('phase_ms_per_iter'), c.get('solve_path'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-matching > $O/bench_rocprof.json 2> $O/bench_rocprof.err || { echo "rocprof rc=$?"; tail -5 $O/bench_rocprof.err; exit 1; }
rm -f $O/prof/*kernel_trace.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'm3s' in r['Name']: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), r['Percentage'][:5])
" | head -30
bash tools/pmc_traffic.sh > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
cp gpurun_out/accum_traffic_cfg3.json $O/pmc_traffic_cfg3.json
tail -3 $O/pmc.log
