#!/bin/bash
# rays iteration accumulate occupancy floor (M3S_ACC_WAVES_RAYS builds) on cfg4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ad
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for w in def w7 w8; do
if [ $w = def ]; then L=mast3r-slam_amd/lib/libm3s_backend.so; else L=mast3r-slam_amd/lib/ab_$w/libm3s_backend.so; fi
M3S_BACKEND_LIB=$L timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/${w}_$rep.json 2> $O/${w}_$rep.err || { echo "bench rc=$?"; tail -5 $O/${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$O/${w}_$rep.json')); print('$w', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], d['accuracy'].get('pose_max_rel_err_vs_oracle_1iter'))"
done
done
