#!/bin/bash
# refine plane-major LDS box variant: matching tests, then timings (B = 1, 8) beside the product
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05h
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matching.py > gpurun_out/r05h/pytest_matching.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05h/pytest_matching.log; exit 1; }
tail -2 gpurun_out/r05h/pytest_matching.log
timeout -k 10 200 python tools/r05/ip_ab.py > gpurun_out/r05h/ab.json 2> gpurun_out/r05h/ab.err || { echo "ab rc=$?"; tail -5 gpurun_out/r05h/ab.err; exit 1; }
cat gpurun_out/r05h/ab.json
