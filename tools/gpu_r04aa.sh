#!/bin/bash
# launch-overhead knob: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export HIP_FORCE_DEV_KERNARG=1; else unset HIP_FORCE_DEV_KERNARG; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-matching > gpurun_out/r04aa_bench_k$v.json 2> gpurun_out/r04aa_bench_k$v.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04aa_bench_k$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04aa_bench_k$v.json')); c=d.get('cfg4',{}); print('devkernarg=$v cfg3', round(d['value']), round(d['ms_per_step'],3), {k: round(x,4) for k,x in d['phase_ms_per_iter'].items()}, 'cfg4', round(c.get('value',0)), round(c.get('ms_per_step'),3), {k: round(x,4) for k,x in c.get('phase_ms_per_iter').items()})"
done
