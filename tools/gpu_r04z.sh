#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/ubench_chol_df 1024 3 > gpurun_out/r04z_chol_df.log 2>&1 || { echo "ubench rc=$?"; tail -20 gpurun_out/r04z_chol_df.log; exit 1; }
grep "rep 3\|C end\|pair\|col 15  C\|col 14  C" gpurun_out/r04z_chol_df.log
