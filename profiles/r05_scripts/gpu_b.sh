#!/bin/bash
# timeout hardening tests + cfg4 elimination-round degree-cap sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_factor_graph.py tests/test_gpu_gn.py -k "timeout or timed_out or held or factor_graph" > gpurun_out/r05b/pytest_timeout.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05b/pytest_timeout.log; exit 1; }
tail -3 gpurun_out/r05b/pytest_timeout.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_dist.py -k timeout > gpurun_out/r05b/pytest_dist_timeout.log 2>&1 || { echo "pytest dist rc=$?"; tail -30 gpurun_out/r05b/pytest_dist_timeout.log; exit 1; }
tail -2 gpurun_out/r05b/pytest_dist_timeout.log
for d in 16 24 32 64; do
  M3S_MULTI_DCAP=$d timeout -k 10 300 python bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r05b/dcap$d.json 2> gpurun_out/r05b/dcap$d.err || { echo "bench dcap $d rc=$?"; tail -5 gpurun_out/r05b/dcap$d.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r05b/dcap$d.json')); print('dcap $d', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
