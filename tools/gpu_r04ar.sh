#!/bin/bash
# cfg3 kernel-level breakdown of the GN call (rocprofv3 kernel trace + stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04ar_prof -o r04ar -- python3 bench.py --no-cfg4 --no-matching --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r04ar_bench.json 2> gpurun_out/r04ar_bench.err || { echo "rocprof rc=$?"; tail -5 gpurun_out/r04ar_bench.err; exit 1; }
find gpurun_out/r04ar_prof -name "*.csv" | head
