#!/bin/bash
# chain prefetch of the next column's P tiles (M3S_DF_PREFETCH) and the granule x hand-off of the
# back-substitution (M3S_DF_XGRAN): GN tests, then a same-box A/B on cfg4 / cfg3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05d
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_gn_stress.py tests/test_gpu_factor_graph.py > gpurun_out/r05d/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05d/pytest_gn.log; exit 1; }
tail -2 gpurun_out/r05d/pytest_gn.log
for v in 11 01 10 00 11; do
  pf=${v:0:1}; xg=${v:1:1}
  M3S_DF_PREFETCH=$pf M3S_DF_XGRAN=$xg timeout -k 10 300 python bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r05d/cfg4_$v.json 2> gpurun_out/r05d/cfg4_$v.err || { echo "bench cfg4 rc=$?"; tail -5 gpurun_out/r05d/cfg4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05d/cfg4_$v.json')); print('cfg4 pf/xg $v', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
for v in 11 00; do
  pf=${v:0:1}; xg=${v:1:1}
  M3S_DF_PREFETCH=$pf M3S_DF_XGRAN=$xg timeout -k 10 300 python bench.py --no-cfg4 --no-matching --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r05d/cfg3_$v.json 2> gpurun_out/r05d/cfg3_$v.err || { echo "bench cfg3 rc=$?"; tail -5 gpurun_out/r05d/cfg3_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05d/cfg3_$v.json')); print('cfg3 pf/xg $v', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
