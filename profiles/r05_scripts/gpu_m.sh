#!/bin/bash
# per-call host phases (M3S_PROF_HOST) of cfg3 / cfg4 at N = 1 and in the 2-rank rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
M3S_PROF_HOST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 3 --warmup 1 > $O/n1.json 2> $O/n1.err || { echo "n1 rc=$?"; tail -10 $O/n1.err; exit 1; }
grep "gn host" $O/n1.err | tail -12
M3S_BENCH_COMM=host M3S_PROF_HOST=1 timeout -k 10 400 python bench.py --gpus 2 --no-matching --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -10 $O/n2.err; exit 1; }
grep "gn host" $O/n2.err | tail -12
