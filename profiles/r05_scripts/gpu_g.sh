#!/bin/bash
# round-5 tree: full GPU suite + smoke + default bench + rocprof stats of the default command +
# PMC traffic of the cfg3 accumulate + the refine LDS bank simulation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'roofline frac', d['roofline']['frac'], 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), c.get('phase_ms_per_iter')); print('stress', d['accuracy'].get('stress_1iter'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-matching > $O/bench_rocprof.json 2> $O/bench_rocprof.err || { echo "rocprof rc=$?"; tail -5 $O/bench_rocprof.err; exit 1; }
rm -f $O/prof/*kernel_trace.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if float(r['Percentage']) > 0.4: print(r['Name'][:90], r['Calls'], r['AverageNs'], r['Percentage'])
"
timeout -k 10 200 python tools/refine_bank_sim.py > $O/refine_bank_sim.json 2> $O/refine_bank_sim.err || { echo "bank sim rc=$?"; tail -5 $O/refine_bank_sim.err; exit 1; }
python -c "import json; d=json.load(open('$O/refine_bank_sim.json')); [print(k, round(v['mean'],2)) for k,v in d.items()]"
