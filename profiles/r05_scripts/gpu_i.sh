#!/bin/bash
# box variant phase split (M3S_BOX_DIAG: 1 no staging, 2 no scoring), B = 1 / 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05i
for dg in 0 1 2; do
  M3S_BOX_DIAG=$dg timeout -k 10 200 python tools/r05/ip_ab.py > gpurun_out/r05i/ab_diag$dg.json 2> gpurun_out/r05i/ab_diag$dg.err || { echo "ab rc=$?"; tail -5 gpurun_out/r05i/ab_diag$dg.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r05i/ab_diag$dg.json')); print('diag $dg', {b: (round(d[b]['refine_ms'],3), {k: round(v['ms'],3) for k,v in d[b]['refine_variants'].items()}) for b in ('B1','B8')})"
done
