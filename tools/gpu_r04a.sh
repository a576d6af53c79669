#!/bin/bash
# round 4, step a: the readlane panel factor / balanced syrk in chol_df -- timeline + GN tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/ubench_chol_df 1024 5 > gpurun_out/r04a_chol_df_1024.log 2>&1 || { echo "ubench rc=$?"; tail -20 gpurun_out/r04a_chol_df_1024.log; exit 1; }
tail -30 gpurun_out/r04a_chol_df_1024.log
timeout -k 10 60 tools/bin/ubench_chol_df 256 3 > gpurun_out/r04a_chol_df_256.log 2>&1 || { echo "ubench256 rc=$?"; exit 1; }
tail -4 gpurun_out/r04a_chol_df_256.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gn.py > gpurun_out/r04a_pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04a_pytest_gn.log; exit 1; }
tail -3 gpurun_out/r04a_pytest_gn.log
timeout -k 10 300 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline --no-matching > gpurun_out/r04a_bench_cfg4.json 2> gpurun_out/r04a_bench_cfg4.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04a_bench_cfg4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04a_bench_cfg4.json')); print(round(d['value']), d['ms_per_step'], d['phase_ms_per_iter'])"
