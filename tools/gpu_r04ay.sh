#!/bin/bash
# full GPU suite + smoke + default bench on the final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04ay_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04ay_pytest.log; exit 1; }
tail -1 gpurun_out/r04ay_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04ay_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r04ay_smoke.log; exit 1; }
tail -1 gpurun_out/r04ay_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04ay_bench.json 2> gpurun_out/r04ay_bench.err || { echo "bench rc=$?"; tail -10 gpurun_out/r04ay_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04ay_bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'roofline', d['roofline'], 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), c.get('phase_ms_per_iter'))"
