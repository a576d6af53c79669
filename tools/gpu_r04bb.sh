#!/bin/bash
# cfg4 kernel stats of the final tree (rocprofv3 kernel trace + stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04bb_prof -o r04bb -- python3 bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04bb_bench.json 2> gpurun_out/r04bb_bench.err || { echo "rocprof rc=$?"; tail -5 gpurun_out/r04bb_bench.err; exit 1; }
rm -f gpurun_out/r04bb_prof/*kernel_trace.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r04bb_prof/r04bb_kernel_stats.csv')):
    if float(r['Percentage']) > 0.5: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
"
