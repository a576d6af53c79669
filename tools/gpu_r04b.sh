#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 tools/bin/ubench_potrf64 8 > gpurun_out/r04i_potrf64.log 2>&1 || exit 1
grep -A7 "potrf_cc: max\|potrf_cc: mean" gpurun_out/r04i_potrf64.log | head -9
timeout -k 10 60 tools/bin/ubench_chol_df 1024 4 > gpurun_out/r04i_chol_df.log 2>&1; rc=$?
grep -v "^col \|^potrf" gpurun_out/r04i_chol_df.log | tail -6; grep "^col  [4] " gpurun_out/r04i_chol_df.log
exit $rc
