#!/bin/bash
# accumulate points-per-lane / ray-constrained A/B + the GN and matching GPU tests (round 3)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=acc3 TESTS="tests/test_gpu_gn.py tests/test_gpu_matching.py" VARIANTS="p2 p4" CFGS="cfg3 cfg4" bash tools/gpu_ab.sh || exit $?
TAG=acc3rc ENVS="M3S_GN_RAYCHECK=1" VARIANTS="p2 p4 p2" CFGS="cfg3" bash tools/gpu_ab.sh || exit $?
TAG=acc3b VARIANTS="p2" CFGS="cfg3" bash tools/gpu_ab.sh
