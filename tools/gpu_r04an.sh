#!/bin/bash
# potrf_bc_w: sp0 = committed (two-trip hand-off, per-column readlanes); un0 = one-trip hand-off;
# un1 = one-trip hand-off + the diagonal block factored as wave-uniform values
mkdir -p gpurun_out
for v in sp0 un0 un1; do
  timeout -k 10 60 tools/bin/ubench_potrf64_$v 8 > gpurun_out/r04ao_potrf64_$v.log 2>&1 || { echo "potrf $v rc=$?"; tail -20 gpurun_out/r04ao_potrf64_$v.log; exit 1; }
  echo "== $v"; grep -E "digest|mean" gpurun_out/r04ao_potrf64_$v.log; grep -E "batch +(8|9|10|11):" gpurun_out/r04ao_potrf64_$v.log
done
for v in sp0 un0 un1 sp0 un0 un1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_$v 1024 3 > gpurun_out/r04ao_chol_df_$v.log 2>&1 || { echo "chol_df $v rc=$?"; tail -20 gpurun_out/r04ao_chol_df_$v.log; exit 1; }
  echo "== $v"; grep -E "rep 3|max err|col  [12] " gpurun_out/r04ao_chol_df_$v.log
done
