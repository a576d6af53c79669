#!/bin/bash
# round-4 GPU suite: every GPU test, then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r04w_pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/r04w_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04w_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04w_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r04w_smoke.log; exit 1; }
tail -1 gpurun_out/r04w_smoke.log
