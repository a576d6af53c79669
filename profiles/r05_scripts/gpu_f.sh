#!/bin/bash
# multi plan: back-substitution + retraction in one gn_solve launch (M3S_MULTI_BACK): GN tests, A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05f
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_gn_stress.py tests/test_gpu_factor_graph.py > gpurun_out/r05f/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05f/pytest_gn.log; exit 1; }
tail -2 gpurun_out/r05f/pytest_gn.log
for v in 1 0 1 0; do
  M3S_MULTI_BACK=$v timeout -k 10 300 python bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r05f/cfg4_mb$v.json 2> gpurun_out/r05f/cfg4_mb$v.err || { echo "bench cfg4 rc=$?"; tail -5 gpurun_out/r05f/cfg4_mb$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05f/cfg4_mb$v.json')); print('cfg4 multi_back $v', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
