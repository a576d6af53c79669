#!/bin/bash
# One GPU call: optional GN tests on the current library, then a quick bench A/B of variant
# libraries (mast3r-slam_amd/lib/variants/<v>.so).  Every GPU step has its own limit; the script
# stops at the first failure.
# usage: TESTS="tests/test_gpu_gn.py ..." VARIANTS="base v1" CFGS="cfg3 cfg4" bash tools/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
TAG="${TAG:-ab}"
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 600 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 \
        --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/${TAG}_pytest.log
    [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CFGS:-cfg3}; do
    for v in ${VARIANTS:-}; do
        env ${ENVS:-} M3S_BACKEND_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so timeout -k 10 300 \
            python bench.py --config $cfg ${BENCH_FLAGS:---no-cpu-baseline} --no-matching --steps ${STEPS:-5} --warmup 2 \
            > gpurun_out/ab/${TAG}_${cfg}_$v.json 2> gpurun_out/ab/${TAG}_${cfg}_$v.err
        rc=$?
        if [ $rc -ne 0 ]; then echo "variant $v $cfg rc=$rc"; tail -5 gpurun_out/ab/${TAG}_${cfg}_$v.err; exit $rc; fi
        python -c "
import json; d = json.load(open('gpurun_out/ab/${TAG}_${cfg}_$v.json'))
print('$cfg $v', round(d['value']), {k: round(v, 4) for k, v in d['phase_ms_per_iter'].items()}, 'acc1', d.get('accuracy', {}).get('pose_max_rel_err_vs_oracle_1iter'), 'acc10', d.get('accuracy', {}).get('pose_max_rel_err_vs_oracle_10iter_timed_call'))"
    done
done
exit 0
