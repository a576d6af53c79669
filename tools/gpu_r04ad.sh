#!/bin/bash
# PMC traffic of cfg4's rays accumulate (the steady-state launch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=cfg4 bash tools/pmc_traffic.sh || exit 1
cat gpurun_out/accum_traffic_cfg4.json
