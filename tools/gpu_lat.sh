#!/bin/bash
# lattice-bucket refine variant: parity tests, then the probe on the default and diagnostic builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_matching.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "refine" > gpurun_out/lat_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/lat_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in "" rv_d1 rv_d2 rv_d3; do
    if [ -n "$v" ]; then export M3S_VARIANTS_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so; fi
    for b in 1 8; do
        B=$b timeout -k 10 200 python tools/lattice_probe.py >> gpurun_out/lat_probe.jsonl 2>> gpurun_out/lat_probe.err
        rc=$?; echo "probe $v B=$b rc=$rc"; tail -n 1 gpurun_out/lat_probe.jsonl; [ $rc -ne 0 ] && exit $rc
    done
done
exit 0
