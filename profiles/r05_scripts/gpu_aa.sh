#!/bin/bash
# L2 warm-up of the back rounds' inputs in gn_solve (M3S_SOLVE_WARM): solver tests + cfg3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py -k "dense_solver or multilaunch or degenerate or timeout or cus_held" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do for w in 0 1; do
M3S_SOLVE_WARM=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --no-cfg4 --steps 10 --warmup 3 > $O/w${w}_${rep}.json 2> $O/w.err || { echo "bench rc=$?"; tail -5 $O/w.err; exit 1; }
python -c "import json; d=json.load(open('$O/w${w}_${rep}.json')); print('warm=$w', round(d['value']), round(d['ms_per_step'],3), round(d['phase_ms_per_iter']['solve'],4))"
done; done
