#!/bin/bash
# cfg4: elimination-round degree cap sweep (core size vs round count), same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r05a
for d in 16 24 32 64; do
  M3S_MULTI_DCAP=$d timeout -k 10 300 python bench.py --config cfg4 --no-cfg4 --no-matching --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r05a/dcap$d.json 2> gpurun_out/r05a/dcap$d.err || { echo "bench dcap $d rc=$?"; tail -5 gpurun_out/r05a/dcap$d.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r05a/dcap$d.json')); print('dcap $d', round(d['value']), round(d['ms_per_step'],3), d['phase_ms_per_iter'])"
done
