#!/bin/bash
# right-looking inverse products in potrf_bc_w: GN test files + bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py tests/test_gpu_gn_stress.py > gpurun_out/r04at_pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "stress iters|Error|assert" gpurun_out/r04at_pytest.log | head; tail -3 gpurun_out/r04at_pytest.log; exit 1; }
tail -1 gpurun_out/r04at_pytest.log; grep -E "stress iters" gpurun_out/r04at_pytest.log | head
for v in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04at_bench_$v.json 2> gpurun_out/r04at_bench_$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04at_bench_$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04at_bench_$v.json')); c=d.get('cfg4',{}); print('cfg3', round(d['value']), round(d['ms_per_step'],3), round(d['phase_ms_per_iter']['solve'],4), 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), {k: round(x,4) for k,x in c.get('phase_ms_per_iter').items()})"
done
