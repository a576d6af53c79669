#!/bin/bash
# tracker: per-call wall time, then the kernel durations under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ah
mkdir -p $O
export TMPDIR=/tmp


cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o trk -- python3 $GRAFT_REPO_ROOT/tools/r05/track_prof.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -12
