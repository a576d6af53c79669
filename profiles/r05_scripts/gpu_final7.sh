#!/bin/bash
# round-5 closing tree (multi plan tile-aware stop): full GPU suite + smoke + default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05final7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); c=d['cfg4']; print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'frac', d['roofline']['frac'], 'cfg4', round(c['value']), round(c['ms_per_step'],3), c['phase_ms_per_iter'])"
