#!/bin/bash
# gn_solve phase clocks (M3S_SOLVE_DEBUG) on cfg3's hybrid back launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ab
mkdir -p $O
M3S_SOLVE_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --no-cfg4 --steps 2 --warmup 1 > $O/dbg.json 2> $O/dbg.err || { echo "rc=$?"; tail -20 $O/dbg.err; exit 1; }
grep -v "^$" $O/dbg.err | head -60
