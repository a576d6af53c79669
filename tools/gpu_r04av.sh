#!/bin/bash
# back-round inputs prefetched into L2 at gn_solve's start (M3S_SOLVE_PREFETCH=1) vs not: GN tests + cfg3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_gn_stress.py > gpurun_out/r04av_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/r04av_pytest.log; exit 1; }
tail -1 gpurun_out/r04av_pytest.log
for v in 1 0 1 0; do
M3S_SOLVE_PREFETCH=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching --no-cfg4 > gpurun_out/r04av_bench_pf$v.json 2> gpurun_out/r04av_bench_pf$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04av_bench_pf$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04av_bench_pf$v.json')); print('pf=$v cfg3', round(d['value']), round(d['ms_per_step'],3), {k: round(x,4) for k,x in d['phase_ms_per_iter'].items()})"
done
