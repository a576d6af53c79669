#!/bin/bash
# tracker: every live step writes the outputs, no final launch behind the host check:
# tracker parity tests, per-call timing, kernel durations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_track.py > $O/pytest_track.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_track.log; exit 1; }
tail -1 $O/pytest_track.log
timeout -k 10 300 python tools/r05/track_prof.py > $O/track.json 2> $O/track.err || { echo "probe rc=$?"; tail -5 $O/track.err; exit 1; }
cat $O/track.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o trk -- python3 $GRAFT_REPO_ROOT/tools/r05/track_prof.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
