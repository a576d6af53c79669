#!/bin/bash
# hybrid plan with a larger dense core (chol_df factors it, so the in-register 27-pose bound no
# longer applies): cfg3 A/B over M3S_HYB_TAILCAP, then the GN tests at the candidate setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ap
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for tc in 27 30 34 40k6; do
if [ $tc = 40k6 ]; then E="M3S_HYB_TAILCAP=40 M3S_HYB_KMIN=6"; else E="M3S_HYB_TAILCAP=$tc"; fi
env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --no-cfg4 --steps 10 --warmup 3 > $O/tc${tc}_$rep.json 2> $O/tc${tc}_$rep.err || { echo "bench $tc rc=$?"; tail -5 $O/tc${tc}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$O/tc${tc}_$rep.json')); print('$tc', round(d['value']), round(d['ms_per_step'],4), 'solve', round(d['phase_ms_per_iter']['solve'],4), 'acc', round(d['phase_ms_per_iter']['accumulate'],4))"
done
done
M3S_HYB_TAILCAP=34 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py > $O/pytest_tc34.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_tc34.log; exit 1; }
tail -1 $O/pytest_tc34.log
