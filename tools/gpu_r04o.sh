#!/bin/bash
# edge-ordered gather exchange: two-rank tests (bitwise vs one rank) + the GN timeout tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_gn.py -k "dist or timeout or sharded or rccl" > gpurun_out/r04o_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r04o_pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04o_pytest.log | tail -20
