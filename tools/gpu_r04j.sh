#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py > gpurun_out/r04j_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04j_pytest.log; exit 1; }
tail -2 gpurun_out/r04j_pytest.log
timeout -k 10 300 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline --no-matching > gpurun_out/r04j_bench_cfg4.json 2> gpurun_out/r04j_bench_cfg4.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04j_bench_cfg4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04j_bench_cfg4.json')); print('cfg4', round(d['value']), d['ms_per_step'], d['phase_ms_per_iter'])"
