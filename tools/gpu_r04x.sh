#!/bin/bash
# round-4 measurement set: the default bench line, the rocprofv3 kernel stats of the same command,
# and the PMC traffic passes of the accumulate (tools/pmc_traffic.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r04x_bench.json 2> gpurun_out/r04x_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04x_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04x_bench.json').read().strip().splitlines()[-1]); print('cfg3', round(d['value']), d['ms_per_step'], 'roofline', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'] if d.get('cpu_baseline') else None, 'cfg4', round(d['cfg4']['value']))"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04x_prof -o bench -- python bench.py > gpurun_out/r04x_prof_bench.json 2> gpurun_out/r04x_prof.err || { echo "rocprof rc=$?"; tail -5 gpurun_out/r04x_prof.err; exit 1; }
f=$(find gpurun_out/r04x_prof -name "*kernel_stats.csv" | head -1); echo "$f"
find gpurun_out/r04x_prof -type f ! -name "*kernel_stats.csv" -delete  # (the trace: > the 64 MiB copy-back)
python - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print('%-70s %6s %10.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3))
PY
CFG=cfg3 bash tools/pmc_traffic.sh || exit 1
du -sh gpurun_out
cat gpurun_out/accum_traffic_cfg3.json | head -30
