#!/bin/bash
# granule x hand-off in chol_df's back-substitution + dcap 32: GN tests, then cfg4 / cfg3 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05c
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_gn_stress.py tests/test_gpu_factor_graph.py > gpurun_out/r05c/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05c/pytest_gn.log; exit 1; }
tail -2 gpurun_out/r05c/pytest_gn.log
timeout -k 10 300 python bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r05c/cfg4.json 2> gpurun_out/r05c/cfg4.err || { echo "bench cfg4 rc=$?"; tail -5 gpurun_out/r05c/cfg4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05c/cfg4.json')); print('cfg4', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
timeout -k 10 300 python bench.py --no-cfg4 --no-matching --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r05c/cfg3.json 2> gpurun_out/r05c/cfg3.err || { echo "bench cfg3 rc=$?"; tail -5 gpurun_out/r05c/cfg3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05c/cfg3.json')); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
