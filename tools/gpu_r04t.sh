#!/bin/bash
# the dense core gathered from the block system inside chol_df (no fill / scatter launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py > gpurun_out/r04t_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04t_pytest.log; exit 1; }
tail -2 gpurun_out/r04t_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04t_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04t_bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), d['ms_per_step'], d['phase_ms_per_iter'], 'cfg4', round(c.get('value',0)), c.get('ms_per_step'), c.get('phase_ms_per_iter'))"
