#!/bin/bash
# potrf_bc_w: inverse products right-looking (rl1) vs left-looking (rl0)
mkdir -p gpurun_out
for v in rl0 rl1; do
  timeout -k 10 60 tools/bin/ubench_potrf64_$v 8 > gpurun_out/r04as_potrf64_$v.log 2>&1 || { echo "potrf $v rc=$?"; tail -20 gpurun_out/r04as_potrf64_$v.log; exit 1; }
  echo "== $v"; grep -E "digest|mean" gpurun_out/r04as_potrf64_$v.log; grep -A5 "inverse (cycles" gpurun_out/r04as_potrf64_$v.log
done
for v in rl0 rl1 rl0 rl1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_$v 1024 3 > gpurun_out/r04as_chol_df_$v.log 2>&1 || { echo "chol_df $v rc=$?"; tail -20 gpurun_out/r04as_chol_df_$v.log; exit 1; }
  echo "== $v"; grep -E "rep 3|max err|col  [12] " gpurun_out/r04as_chol_df_$v.log
done
