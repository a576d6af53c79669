#!/bin/bash
# rays accumulate: dr/dX from r and r/|X| (168.5 VALU, 8 transcendentals per point-edge):
# GN tests, then a same-box A/B of cfg4 against the previous build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_dist.py > $O/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gn.log; exit 1; }
tail -1 $O/pytest_gn.log
for rep in 1 2 3; do
for v in def old; do
if [ $v = def ]; then L=mast3r-slam_amd/lib/libm3s_backend.so; else L=mast3r-slam_amd/lib/ab_$v/libm3s_backend.so; fi
M3S_BACKEND_LIB=$L timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "bench $v rc=$?"; tail -5 $O/${v}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$v', round(d['value']), round(d['ms_per_step'],3), 'acc', round(d['phase_ms_per_iter']['accumulate'],4))"
done
done
