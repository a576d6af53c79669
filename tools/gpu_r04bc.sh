#!/bin/bash
# chol_df back-substitution: syrk K-split over waves (sk1) vs 3/3/2/2 blocks (sk0)
mkdir -p gpurun_out
for v in sk0 sk1 sk0 sk1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_$v 1024 3 > gpurun_out/r04bc_chol_df_$v.log 2>&1 || { echo "chol_df $v rc=$?"; tail -20 gpurun_out/r04bc_chol_df_$v.log; exit 1; }
  echo "== $v"; grep -E "rep 3|max err|pair  [0-2]|col  [12] " gpurun_out/r04bc_chol_df_$v.log
done
