#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
M3S_HYB_CORE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_prof$v -o cfg3 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-matching --no-cfg4 > gpurun_out/r04m_bench$v.json 2> gpurun_out/r04m_bench$v.err; echo "rc $?"
f=$(find gpurun_out/r04m_prof$v -name "*kernel_stats.csv" | head -1); echo "$f"
python - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n=r['Name']
    if 'm3s' in n:
        print('%-60s %6s %10.1f %10.1f' % (n.split('(')[0][-60:], r['Calls'], float(r['TotalDurationNs'])/1e3, float(r['AverageNs'])/1e3))
PY
done
