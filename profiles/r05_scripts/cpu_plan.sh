#!/bin/bash
# host planner section times on the GPU box's CPU (no GPU use)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for c in cfg3 cfg4; do echo $c; timeout -k 5 60 tools/bin/plan_time < tools/bin/$c.txt; done
