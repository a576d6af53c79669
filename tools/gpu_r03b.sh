#!/bin/bash
# Round-3 (session 3) quick GPU check: the solve's in-kernel phase clocks on cfg3 / cfg4 topology
# and a short cfg3 bench.  Each GPU step has its own limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r03d}"
timeout -k 10 120 python tools/solve_debug.py cfg3 2 > gpurun_out/${TAG}_solve_cfg3.log 2>&1 || { echo "solve_debug cfg3 failed"; exit 1; }
tail -n 30 gpurun_out/${TAG}_solve_cfg3.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching > gpurun_out/${TAG}_qbench.json 2> gpurun_out/${TAG}_qbench.err || { echo "qbench failed"; exit 1; }
cat gpurun_out/${TAG}_qbench.json
