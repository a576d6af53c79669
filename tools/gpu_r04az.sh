#!/bin/bash
# chol_df back-substitution: paired x vectors in one hand-off (xb1) vs flag-then-load per column (xb0)
mkdir -p gpurun_out
for v in xb0 xb1 xb0 xb1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_$v 1024 3 > gpurun_out/r04az_chol_df_$v.log 2>&1 || { echo "chol_df $v rc=$?"; tail -20 gpurun_out/r04az_chol_df_$v.log; exit 1; }
  echo "== $v"; grep -E "rep 3|max err|pair  [0-7]" gpurun_out/r04az_chol_df_$v.log
done
