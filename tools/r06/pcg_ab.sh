# PCG A/B on one box: phase clocks, the direct solve vs PCG (cfg3 + cfg4 blocks), the PCG tests
# usage: bash tools/r06/pcg_ab.sh TAG
set -o pipefail
T=${1:-f}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r06/pcg_debug.py > gpurun_out/r06_${T}_pcg_debug.log 2>&1 || { tail -30 gpurun_out/r06_${T}_pcg_debug.log; exit 1; }
grep -E "pcg\[(2|3)\]|pcg_runs" gpurun_out/r06_${T}_pcg_debug.log | head -12
run() {
  tag=$1; shift
  env "$@" > gpurun_out/r06_${T}_$tag.json 2>> gpurun_out/r06_${T}.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r06_${T}_$tag.json'))
sp=lambda b: {k:(round(v,4) if isinstance(v,float) else v) for k,v in (b.get('solve_path') or {}).items()}
print('$tag', round(d['value']), round(d['phase_ms_per_iter']['solve'],4), sp(d), '| cfg4', round(d['cfg4']['value']), round(d['cfg4']['phase_ms_per_iter']['solve'],4), sp(d['cfg4']))" | tee -a gpurun_out/r06_${T}_ab.txt
}
run direct M3S_GN_PCG=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching
run pcg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py -s > gpurun_out/r06_${T}_pytest_pcg.log 2>&1; tail -12 gpurun_out/r06_${T}_pytest_pcg.log
