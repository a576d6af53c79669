#!/bin/bash
# batch width of the batch-cyclic tile factor: 4 vs 8 columns (potrf microbenchmark + chain), same box
mkdir -p gpurun_out
for w in 4 8; do
  timeout -k 10 60 tools/bin/ubench_potrf64_bw$w 8 > gpurun_out/r04ah_potrf64_bw$w.log 2>&1 || { echo "potrf bw$w rc=$?"; tail -20 gpurun_out/r04ah_potrf64_bw$w.log; exit 1; }
  echo "== bw$w"; sed -n 3,10p gpurun_out/r04ah_potrf64_bw$w.log
done
for w in 4 8 4 8; do
  timeout -k 10 60 tools/bin/ubench_chol_df_bw$w 1024 3 > gpurun_out/r04ah_chol_df_bw$w.log 2>&1 || { echo "chol_df bw$w rc=$?"; tail -20 gpurun_out/r04ah_chol_df_bw$w.log; exit 1; }
  echo "== bw$w"; grep -E "rep 3|max err|col  [123] " gpurun_out/r04ah_chol_df_bw$w.log
done
