#!/bin/bash
# iter_proj zero-step skip: matching parity tests + switch tests + A/B of the kernel time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_switches.py tests/test_glue_golden.py > $O/pytest_match.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_match.log; exit 1; }
tail -1 $O/pytest_match.log
for sk in 0 1 0 1; do
M3S_IP_SKIP=$sk timeout -k 10 300 python tools/r05/ip_ab.py > $O/ab_skip$sk.json 2> $O/ab_skip$sk.err || { echo "ab rc=$?"; tail -10 $O/ab_skip$sk.err; exit 1; }
python -c "import json; d=json.load(open('$O/ab_skip$sk.json')); print('skip=$sk', 'B1 ip', round(d['B1']['iter_proj_ms'],4), 'B8 ip', round(d['B8']['iter_proj_ms'],4), 'fused B8', round(d['B8']['refine_variants']['fused_op']['ms'],4), 'p_checksum', d['B8']['p_checksum'])"
done
for sv in 0 2 0 2; do
M3S_SOLVER=$sv timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --no-cfg4 --steps 10 --warmup 3 > $O/cfg3_solver$sv.json 2> $O/cfg3_solver$sv.err || { echo "bench rc=$?"; tail -5 $O/cfg3_solver$sv.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3_solver$sv.json')); print('solver=$sv', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
for hm in 0 1 0 1; do
M3S_HYB_MULTI=$hm timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/hybmulti$hm.json 2> $O/hybmulti$hm.err || { echo "bench rc=$?"; tail -5 $O/hybmulti$hm.err; exit 1; }
python -c "import json; d=json.load(open('$O/hybmulti$hm.json')); c=d['cfg4']; print('hyb_multi=$hm', 'cfg3', round(d['value']), round(d['ms_per_step'],3), round(d['phase_ms_per_iter']['solve'],4), 'cfg4', round(c['value']), round(c['phase_ms_per_iter']['solve'],4))"
done
