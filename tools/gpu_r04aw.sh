#!/bin/bash
# rays norm table (M3S_RAYS_NTAB=1) vs inline sqrt / rcp: GN tests + cfg4 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py > gpurun_out/r04aw_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/r04aw_pytest.log; exit 1; }
tail -1 gpurun_out/r04aw_pytest.log
for v in 1 0 1 0; do
M3S_RAYS_NTAB=$v timeout -k 10 300 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline --no-matching --no-cfg4 > gpurun_out/r04aw_bench_nt$v.json 2> gpurun_out/r04aw_bench_nt$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04aw_bench_nt$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04aw_bench_nt$v.json')); print('ntab=$v cfg4', round(d['value']), round(d['ms_per_step'],3), {k: round(x,4) for k,x in d['phase_ms_per_iter'].items()}, d.get('accuracy',{}).get('max_rel_pose_err_vs_oracle'))"
done
