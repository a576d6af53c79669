#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ubench_potrf64 ubench_potrf64_rl; do
timeout -k 10 60 tools/bin/$b 8 > gpurun_out/r04f_$b.log 2>&1 || exit 1
echo $b; grep -A7 "potrf_cc: mean" gpurun_out/r04f_$b.log
done
