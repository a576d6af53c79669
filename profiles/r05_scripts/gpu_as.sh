#!/bin/bash
# multi plan: stop before a round of < 4 poses that keeps the core's tile count (M3S_MULTI_KMIN):
# cfg4 A/B (3 rounds / 127-pose core vs 4 rounds / 125), then the GN tests at the candidate
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05as
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for km in 0 4; do
M3S_MULTI_KMIN=$km timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/km${km}_$rep.json 2> $O/km${km}_$rep.err || { echo "bench rc=$?"; tail -5 $O/km${km}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$O/km${km}_$rep.json')); p=d['phase_ms_per_iter']; print('kmin $km', round(d['value']), round(d['ms_per_step'],3), 'solve', round(p['solve'],4), 'acc', round(p['accumulate'],4))"
done
done
M3S_MULTI_KMIN=4 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_switches.py > $O/pytest_km4.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_km4.log; exit 1; }
tail -1 $O/pytest_km4.log
