#!/bin/bash
# iter_proj XCD-banded block order: matching tests, then an A/B of M3S_IP_XCD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matching.py > gpurun_out/r05e/pytest_matching.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05e/pytest_matching.log; exit 1; }
tail -2 gpurun_out/r05e/pytest_matching.log
for x in 1 0 1 0; do
  M3S_IP_XCD=$x timeout -k 10 200 python tools/r05/ip_ab.py > gpurun_out/r05e/ip_xcd$x.json 2> gpurun_out/r05e/ip_xcd$x.err || { echo "ip_ab rc=$?"; tail -5 gpurun_out/r05e/ip_xcd$x.err; exit 1; }
  cat gpurun_out/r05e/ip_xcd$x.json
done
