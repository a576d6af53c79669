#!/bin/bash
# potrf_bc_w: X_ww by 16 forward substitutions (fs1) vs two 8x8 inverses + products (fs0)
mkdir -p gpurun_out
for v in fs0 fs1; do
  timeout -k 10 60 tools/bin/ubench_potrf64_$v 8 > gpurun_out/r04au_potrf64_$v.log 2>&1 || { echo "potrf $v rc=$?"; tail -20 gpurun_out/r04au_potrf64_$v.log; exit 1; }
  echo "== $v"; grep -E "digest|mean" gpurun_out/r04au_potrf64_$v.log; grep -A5 "inverse (cycles" gpurun_out/r04au_potrf64_$v.log
done
for v in fs0 fs1 fs0 fs1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_$v 1024 3 > gpurun_out/r04au_chol_df_$v.log 2>&1 || { echo "chol_df $v rc=$?"; tail -20 gpurun_out/r04au_chol_df_$v.log; exit 1; }
  echo "== $v"; grep -E "rep 3|max err|col  [12] " gpurun_out/r04au_chol_df_$v.log
done
