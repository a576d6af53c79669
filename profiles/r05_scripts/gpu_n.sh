#!/bin/bash
# host planner rework: GN GPU tests + per-call host phases (M3S_PROF_HOST) at N = 1 and in the
# 2-rank rehearsal + the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py tests/test_gpu_gn_stress.py tests/test_gpu_switches.py > $O/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gn.log; exit 1; }
tail -2 $O/pytest_gn.log
M3S_PROF_HOST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 3 --warmup 1 > $O/n1.json 2> $O/n1.err || { echo "n1 rc=$?"; tail -10 $O/n1.err; exit 1; }
grep "gn host: setup" $O/n1.err
M3S_BENCH_COMM=host M3S_PROF_HOST=1 timeout -k 10 400 python bench.py --gpus 2 --no-matching --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -10 $O/n2.err; exit 1; }
grep "gn host: setup" $O/n2.err | tail -8
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3))"
