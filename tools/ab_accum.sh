#!/bin/bash
# A/B of accumulate-kernel scheduling knobs (one process per setting, same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for cfg in "M3S_ACC_SCHED=1 M3S_ACC_CHUNK=8192" "M3S_ACC_SCHED=0 M3S_ACC_CHUNK=8192" \
           "M3S_ACC_SCHED=1 M3S_ACC_CHUNK=4096" "M3S_ACC_SCHED=1 M3S_ACC_CHUNK=16384" \
           "M3S_ACC_SCHED=0 M3S_ACC_CHUNK=12288"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err
    rc=$?
    python -c "import json,sys; b=json.load(open('gpurun_out/ab/$tag.json')); print('$cfg', round(b['value']), {k: round(v,4) for k,v in b['phase_ms_per_iter'].items()})" || echo "$cfg rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
