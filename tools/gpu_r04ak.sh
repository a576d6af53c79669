#!/bin/bash
# batch-cyclic factor, single-poll written counters: chain A/B, potrf stamps, GN test files, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1; do
  timeout -k 10 60 tools/bin/ubench_chol_df_bc$v 1024 3 > gpurun_out/r04ak_chol_df_bc$v.log 2>&1 || { echo "chol_df bc$v rc=$?"; tail -20 gpurun_out/r04ak_chol_df_bc$v.log; exit 1; }
  echo "== bc$v"; grep -E "rep 3|max err|col  [12] " gpurun_out/r04ak_chol_df_bc$v.log
done
timeout -k 10 60 tools/bin/ubench_potrf64_bc1 8 > gpurun_out/r04ak_potrf64_bc1.log 2>&1 || { echo "potrf rc=$?"; exit 1; }
sed -n 4,10p gpurun_out/r04ak_potrf64_bc1.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py tests/test_gpu_gn_stress.py > gpurun_out/r04ak_pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "stress iters|Error|assert" gpurun_out/r04ak_pytest.log | head; tail -3 gpurun_out/r04ak_pytest.log; exit 1; }
tail -1 gpurun_out/r04ak_pytest.log
for v in 1 0 1 0; do
[ $v = 0 ] && export M3S_BACKEND_LIB=$PWD/tools/bin/libm3s_backend_bc0.so || unset M3S_BACKEND_LIB
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04ak_bench_bc$v.json 2> gpurun_out/r04ak_bench_bc$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04ak_bench_bc$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04ak_bench_bc$v.json')); c=d.get('cfg4',{}); print('bc=$v cfg3', round(d['value']), round(d['ms_per_step'],3), round(d['phase_ms_per_iter']['solve'],4), 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), {k: round(x,4) for k,x in c.get('phase_ms_per_iter').items()})"
done
