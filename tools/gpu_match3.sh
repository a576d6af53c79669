#!/bin/bash
# refine variants: GPU parity tests, then the bench's matching section
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${TAG:-m3}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_matching.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${KSEL:+-k "$KSEL"} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/${TAG}_bench.err
python -c "
import json; d = json.loads(open('gpurun_out/${TAG}_bench.json').readline())
for B in ('B1', 'B8'):
    m = d['matching'][B]
    print(B, 'iter_proj', round(m['iter_proj_ms'], 4), 'refine', round(m['refine_ms'], 4), 'fused', round(m['match_iterative_proj_ms'], 4), 'lattice', round(m['refine_mfma_lattice']['ms'], 4))
"
exit $rc
