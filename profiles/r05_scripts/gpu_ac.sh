#!/bin/bash
# compacted stream (M3S_GN_COMPACT) A/B on cfg3 and cfg4 per call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ac
mkdir -p $O
export TMPDIR=/tmp
for cm in 0 1 0 1; do
M3S_GN_COMPACT=$cm timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/compact$cm.json 2> $O/compact$cm.err || { echo "bench rc=$?"; tail -5 $O/compact$cm.err; exit 1; }
python -c "import json; d=json.load(open('$O/compact$cm.json')); c=d['cfg4']; print('compact=$cm', 'cfg3', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'], 'cfg4', round(c['value']), round(c['ms_per_step'],3), c['phase_ms_per_iter'])"
done
