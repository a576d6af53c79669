#!/bin/bash
# early all-gather (M3S_EARLY_GATHER) in the 2-rank tests + the rehearsal's host phases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py > $O/pytest_dist.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_dist.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_dist.log | tail -20
M3S_BENCH_COMM=host M3S_PROF_HOST=1 timeout -k 10 400 python bench.py --gpus 2 --no-matching --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -10 $O/n2.err; exit 1; }
grep "gn host" $O/n2.err | tail -8
