#!/bin/bash
# paired back-substitution tasks: ubench A/B (head vs new) at cfg4 / cfg3 core sizes, then the GN tests + bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in head new; do
  exe=tools/bin/ubench_chol_df; [ $b = head ] && exe=tools/bin/ubench_chol_df_head
  timeout -k 10 60 $exe 1024 4 > gpurun_out/r04y_$b.log 2>&1 || { echo "ubench $b rc=$?"; tail -20 gpurun_out/r04y_$b.log; exit 1; }
  timeout -k 10 60 $exe 256 4 > gpurun_out/r04y_${b}_256.log 2>&1 || { echo "ubench256 $b rc=$?"; tail -20 gpurun_out/r04y_${b}_256.log; exit 1; }
  echo "$b: $(grep 'rep 4' gpurun_out/r04y_$b.log) $(grep 'C end' gpurun_out/r04y_$b.log) | 256: $(grep 'rep 4' gpurun_out/r04y_${b}_256.log)"
  grep "max err" gpurun_out/r04y_$b.log | tail -2
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_dist.py > gpurun_out/r04y_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04y_pytest.log; exit 1; }
tail -1 gpurun_out/r04y_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04y_bench.json 2> gpurun_out/r04y_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04y_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04y_bench.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), {k: round(x,4) for k,x in d['phase_ms_per_iter'].items()}, 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), {k: round(x,4) for k,x in c.get('phase_ms_per_iter').items()})"
