#!/bin/bash
# SLP packing off for every kernel object (iter_proj, tracker, retraction, solve tail): A/B of the
# bench's matching / tracking / GN numbers, then the matching and tracking parity tests on it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ag
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for v in def noslp; do
if [ $v = def ]; then L=mast3r-slam_amd/lib/libm3s_backend.so; else L=mast3r-slam_amd/lib/ab_$v/libm3s_backend.so; fi
M3S_BACKEND_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "bench $v rc=$?"; tail -5 $O/${v}_$rep.err; exit 1; }
python -c "
import json; d=json.load(open('$O/${v}_$rep.json')); m=d['matching']; t=d['tracking']
print('$v', round(d['value']), 'solve', round(d['phase_ms_per_iter']['solve'],4), 'retract', round(d['phase_ms_per_iter']['retract'],4), 'cfg4', round(d['cfg4']['value']),
 'ip B1', round(m['B1']['iter_proj_ms'],4), 'ip B8', round(m['B8']['iter_proj_ms'],4), 'fused B1', round(m['B1']['match_iterative_proj_ms'],4), 'fused B8', round(m['B8']['match_iterative_proj_ms'],4),
 'trk calib', round(t['calib']['ms_per_iter'],4), round(t['calib']['frame_ms'],4), 'trk rays', round(t['rays']['ms_per_iter'],4))"
done
done
M3S_BACKEND_LIB=mast3r-slam_amd/lib/ab_noslp/libm3s_backend.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_track.py tests/test_gpu_switches.py > $O/pytest_noslp.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_noslp.log; exit 1; }
tail -2 $O/pytest_noslp.log
