#!/bin/bash
# Matching-kernel session: GPU parity tests of the matching ops, then the bench's matching block.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${TAG:-match}"
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    tests/test_gpu_matching.py > gpurun_out/${TAG}_match.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_match.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python - <<'PY'
import json, sys
sys.argv = ["bench.py"]
sys.path[:0] = [".", "mast3r-slam_amd"]
import torch
import bench
print(json.dumps(bench.matching_bench(torch.device("cuda", 0))))
PY
