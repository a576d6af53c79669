#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "" rv_d1 rv_d2 rv_d3; do
    if [ -n "$v" ]; then export M3S_VARIANTS_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python tools/lattice_probe.py >> gpurun_out/lat_probe.jsonl 2>> gpurun_out/lat_probe.err
    rc=$?; echo "probe $v rc=$rc"; tail -n 1 gpurun_out/lat_probe.jsonl; [ $rc -ne 0 ] && exit $rc
done
exit 0
