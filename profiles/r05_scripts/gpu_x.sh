#!/bin/bash
# planar ray image for the fused op's iter_proj + workgroup-uniform image base: matching tests,
# switch tests, A/B of the fused op and the standalone iter_proj, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_matching.py tests/test_gpu_switches.py tests/test_glue_golden.py > $O/pytest_match.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_match.log; exit 1; }
tail -1 $O/pytest_match.log
for rep in 1 2; do for cfg in "0 0" "1 0" "0 1" "1 1"; do set -- $cfg
M3S_MATCH_IPPLANAR=$1 M3S_IP_UB=$2 timeout -k 10 300 python tools/r05/match_ab.py > $O/ab_pl$1_ub$2_$rep.json 2> $O/ab.err || { echo "ab rc=$?"; tail -10 $O/ab.err; exit 1; }
python -c "import json; d=json.load(open('$O/ab_pl$1_ub$2_$rep.json')); print('planar=$1 ub=$2', 'B1', round(d['B1']['fused_ms'],4), 'B8', round(d['B8']['fused_ms'],4), d['B8']['idx_checksum'], d['B8']['valid'])"
done; done
for ub in 0 1 0 1; do
M3S_IP_UB=$ub timeout -k 10 300 python tools/r05/ip_ab.py > $O/ip_ub$ub.json 2> $O/ip.err || { echo "ip rc=$?"; tail -10 $O/ip.err; exit 1; }
python -c "import json; d=json.load(open('$O/ip_ub$ub.json')); print('standalone ub=$ub', 'B1 ip', round(d['B1']['iter_proj_ms'],4), 'B8 ip', round(d['B8']['iter_proj_ms'],4), d['B8']['p_checksum'])"
done
for pl in 0 1; do
M3S_MATCH_IPPLANAR=$pl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$pl -o run -- python3 tools/r05/match_ab.py > $O/rp$pl.json 2> $O/rp$pl.err || { echo "rocprof rc=$?"; tail -5 $O/rp$pl.err; exit 1; }
rm -f $O/prof$pl/*kernel_trace.csv
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof$pl/run_kernel_stats.csv')):
    if 'iter_proj' in r['Name'] or 'match_prep' in r['Name']: print('planar=$pl', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
"
done
