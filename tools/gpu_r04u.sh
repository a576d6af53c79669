#!/bin/bash
# A/B in one run: M3S_DF_GATHER=1 (core gathered inside chol_df) vs 0 (fill + scatter launches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py > gpurun_out/r04u_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04u_pytest.log; exit 1; }
tail -1 gpurun_out/r04u_pytest.log
timeout -k 10 300 python tools/sqrt_records.py > gpurun_out/r04u_sqrt.json 2> gpurun_out/r04u_sqrt.err || { echo "sqrt rc=$?"; tail -5 gpurun_out/r04u_sqrt.err; exit 1; }
cat gpurun_out/r04u_sqrt.json
for v in 1 0 1; do
M3S_DF_GATHER=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04u_bench_g$v.json 2> gpurun_out/r04u_bench_g$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04u_bench_g$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04u_bench_g$v.json')); c=d.get('cfg4',{}); print('gather=$v cfg3', round(d['value']), round(d['ms_per_step'],3), {k: round(x,4) for k,x in d['phase_ms_per_iter'].items()}, 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), {k: round(x,4) for k,x in c.get('phase_ms_per_iter').items()})"
done
