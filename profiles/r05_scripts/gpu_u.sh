#!/bin/bash
# pre-pass placement A/B (M3S_PREPASS 0/1/2): per-call host phases + bench, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05u
mkdir -p $O
export TMPDIR=/tmp
for m in 0 1 2 0 1 2; do
M3S_PREPASS=$m M3S_PROF_HOST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 10 --warmup 3 > $O/pp$m.json 2> $O/pp$m.err || { echo "bench rc=$?"; tail -10 $O/pp$m.err; exit 1; }
python -c "
import json,re
d=json.load(open('$O/pp$m.json')); c=d['cfg4']
L=[l for l in open('$O/pp$m.err') if 'copies + sync' in l and 'build_plan 2' not in l[:25]]
sy=[float(re.search(r'sync (\d+)',l).group(1)) for l in L]
print('prepass=$m', 'cfg3', round(d['value']), round(d['ms_per_step'],3), 'cfg4', round(c['value']), round(c['ms_per_step'],3), 'sync us (first/last 4):', sy[:4], sy[-4:])"
done
