#!/bin/bash
# accumulate task order: edges by (j, i) (M3S_ACC_SCHED=1, default) vs by (i, j) (2): cfg3 + cfg4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 2 1 2; do
M3S_ACC_SCHED=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04ax_bench_s$v.json 2> gpurun_out/r04ax_bench_s$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04ax_bench_s$v.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04ax_bench_s$v.json')); c=d['cfg4']; print('sched=$v cfg3', round(d['value']), round(d['phase_ms_per_iter']['accumulate'],4), 'cfg4', round(c['value']), round(c['phase_ms_per_iter']['accumulate'],4))"
done
