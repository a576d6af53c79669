#!/bin/bash
# rocprofv3 kernel stats of the default bench command, then the HBM-traffic PMC passes of the
# accumulate (tools/pmc_traffic.sh).  Every GPU step has its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-r03_prof}"
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG} -o run \
    -- python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "rocprof bench rc=$rc"; tail -n 2 gpurun_out/${TAG}_bench.err; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/${TAG}/*kernel_trace.csv
CFG=cfg3 bash tools/pmc_traffic.sh
