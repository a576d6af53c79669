#!/bin/bash
# batch-cyclic factor with per-wave written counters: chain A/B vs column-cyclic; stress test alone
mkdir -p gpurun_out
for v in 0 1 0 1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_bc$v 1024 3 > gpurun_out/r04aj_chol_df_bc$v.log 2>&1 || { echo "chol_df bc$v rc=$?"; tail -20 gpurun_out/r04aj_chol_df_bc$v.log; exit 1; }
  echo "== bc$v"; grep -E "rep 3|max err|col  [12] " gpurun_out/r04aj_chol_df_bc$v.log
done
timeout -k 10 60 tools/bin/ubench_potrf64_bc1 8 > gpurun_out/r04aj_potrf64_bc1.log 2>&1 || { echo "potrf rc=$?"; exit 1; }
sed -n 4,10p gpurun_out/r04aj_potrf64_bc1.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn_stress.py > gpurun_out/r04aj_stress.log 2>&1; echo "stress alone rc=$?"; grep -E "stress iters|passed|failed" gpurun_out/r04aj_stress.log | tail -12
