#!/bin/bash
# ray-constrained calib transform factored per pixel row (M3S_RC_FACTOR): GN tests, then a
# same-box A/B of the default bench (cfg3) against the unfactored build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05am
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py > $O/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gn.log; exit 1; }
tail -1 $O/pytest_gn.log
for rep in 1 2 3; do
for v in def f0; do
if [ $v = def ]; then L=mast3r-slam_amd/lib/libm3s_backend.so; else L=mast3r-slam_amd/lib/ab_$v/libm3s_backend.so; fi
M3S_BACKEND_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --no-cfg4 --steps 10 --warmup 3 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "bench $v rc=$?"; tail -5 $O/${v}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$O/${v}_$rep.json')); a=d['accuracy']; print('$v', round(d['value']), round(d['ms_per_step'],4), 'acc', round(d['phase_ms_per_iter']['accumulate'],4), 'frac', round(d['roofline']['frac'],4), 'err10', a['pose_max_rel_err_vs_oracle_10iter_timed_call'], 'err1', a['pose_max_rel_err_vs_oracle_1iter'], 'vs exact', a['pose_max_rel_err_vs_exact_sum_1iter'])"
done
done
