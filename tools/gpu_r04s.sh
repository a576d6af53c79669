#!/bin/bash
# two-rank one-GPU rehearsal of bench.py --gpus 2 (gloo + the host exchange), then the refine PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
M3S_BENCH_COMM=host timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-matching > gpurun_out/r04s_rehearse2.json 2> gpurun_out/r04s_rehearse2.err || { echo "rehearse rc=$?"; tail -20 gpurun_out/r04s_rehearse2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04s_rehearse2.json').read().strip().splitlines()[-1]); c=d['cfg4']; print('n_gpus', d['n_gpus'], 'cfg3', round(d['value']), 'cfg4', round(c['value']), c.get('n_ranks'), c.get('n_ranks_comm'), c.get('comm'))"
bash tools/pmc_refine_lds.sh
