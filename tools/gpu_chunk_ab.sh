#!/bin/bash
# accumulate chunk size A/B (M3S_ACC_CHUNK points per workgroup task), cfg3 and cfg4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for cfg in cfg3 cfg4; do
    for ch in ${CHUNKS:-16384 24576 32768 49152 65536 16384}; do
        M3S_ACC_CHUNK=$ch timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-matching --steps 5 --warmup 2 \
            > gpurun_out/ab/chunk_${cfg}_$ch.json 2> gpurun_out/ab/chunk_${cfg}_$ch.err
        rc=$?; [ $rc -ne 0 ] && { echo "chunk $ch $cfg rc=$rc"; tail -3 gpurun_out/ab/chunk_${cfg}_$ch.err; exit $rc; }
        python -c "
import json; d = json.load(open('gpurun_out/ab/chunk_${cfg}_$ch.json'))
print('$cfg chunk $ch', round(d['value']), {k: round(v, 4) for k, v in d['phase_ms_per_iter'].items()})"
    done
done
exit 0
