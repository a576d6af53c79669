#!/bin/bash
# batch-cyclic vs column-cyclic tile factor: potrf microbenchmark + chol_df chain, same box
mkdir -p gpurun_out
for v in 0 1; do
  timeout -k 10 60 tools/bin/ubench_potrf64_bc$v 8 > gpurun_out/r04ae_potrf64_bc$v.log 2>&1 || { echo "potrf bc$v rc=$?"; tail -20 gpurun_out/r04ae_potrf64_bc$v.log; exit 1; }
  grep -E "potrf_cc" gpurun_out/r04ae_potrf64_bc$v.log
done
for v in 0 1 0 1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_bc$v 1024 3 > gpurun_out/r04ae_chol_df_bc$v.log 2>&1 || { echo "chol_df bc$v rc=$?"; tail -20 gpurun_out/r04ae_chol_df_bc$v.log; exit 1; }
  echo "== bc$v"; grep -iE "err|us|chain" gpurun_out/r04ae_chol_df_bc$v.log | head -12
done
