#!/bin/bash
# A/B the variant libraries (tools/build_variants.sh) on the bench, one GPU box call.
# usage: VARIANTS="a b c" [ENVS="X=1 Y=2"] bash tools/ab_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
CFG="${CFG:-cfg3}"
for v in $VARIANTS; do
    env ${ENVS:-} M3S_BACKEND_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so timeout -k 10 300 \
        python bench.py --config $CFG --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/ab/$v.err; exit $rc; fi
    python -c "
import json; d = json.load(open('gpurun_out/ab/$v.json'))
print('$v', round(d['value']), {k: round(v, 4) for k, v in d['phase_ms_per_iter'].items()})"
done
