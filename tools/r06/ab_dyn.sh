set -o pipefail
for v in 1 0; do
  M3S_GN_PCG=0 M3S_DF_DYN=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching > gpurun_out/r06_c_ab_dyn$v.json 2>>gpurun_out/r06_c_ab.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r06_c_ab_dyn$v.json'))
print('dyn=$v', round(d['value']), d['phase_ms_per_iter']['solve'], round(d['cfg4']['value']), d['cfg4']['phase_ms_per_iter']['solve'])" | tee -a gpurun_out/r06_c_ab.txt
done
