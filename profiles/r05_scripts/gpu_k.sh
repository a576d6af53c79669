#!/bin/bash
# fused matching op with the plane-major fp16 D11 (M3S_MATCH_PLANES): matching tests + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matching.py tests/test_glue_golden.py > gpurun_out/r05k/pytest_matching.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r05k/pytest_matching.log; exit 1; }
tail -2 gpurun_out/r05k/pytest_matching.log
for pl in 1 0 1 0; do
  M3S_MATCH_PLANES=$pl timeout -k 10 200 python tools/r05/ip_ab.py > gpurun_out/r05k/ab_pl$pl.json 2> gpurun_out/r05k/ab_pl$pl.err || { echo "ab rc=$?"; tail -5 gpurun_out/r05k/ab_pl$pl.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05k/ab_pl$pl.json')); print('planes $pl', {b: (round(d[b]['refine_ms'],3), {k: round(v['ms'],3) for k,v in d[b]['refine_variants'].items()}, d[b]['refine_variants']['fused_op']['idx_checksum']) for b in ('B1','B8')})"
done
