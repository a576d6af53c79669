#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_factor_graph.py > gpurun_out/r04l_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04l_pytest.log; exit 1; }
tail -2 gpurun_out/r04l_pytest.log
for v in 1 0; do
M3S_HYB_CORE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching --no-cfg4 > gpurun_out/r04l_bench_core$v.json 2> gpurun_out/r04l_bench_core$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04l_bench_core$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04l_bench_core$v.json')); print('cfg3 core_df=$v', round(d['value']), d['ms_per_step'], d['phase_ms_per_iter'])"
done
