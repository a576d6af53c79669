#!/bin/bash
# two-rank rehearsal of bench.py --gpus 2 on one GPU (gloo + the op's host exchange), with the PCG on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06rh
mkdir -p $O
export TMPDIR=/tmp
M3S_BENCH_COMM=host timeout -k 10 600 python bench.py --gpus 2 --no-cpu-baseline --no-matching --steps 3 --warmup 1 > $O/rehearse2.json 2> $O/rehearse2.err || { echo "rehearsal rc=$?"; tail -20 $O/rehearse2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/rehearse2.json') if l.startswith('{')][-1]); c=d['cfg4']; print('n_gpus', d['n_gpus'], 'scaling', d['scaling'], 'cfg3', round(d['value']), round(d['ms_per_step'],3), d.get('solve_path'), 'cfg4', round(c['value']), round(c['ms_per_step'],3), c.get('solve_path'))"
