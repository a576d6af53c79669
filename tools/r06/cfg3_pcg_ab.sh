# cfg3 (headline) with the PCG forced at lags 2 / 3 against the direct solve, interleaved twice
# usage: bash tools/r06/cfg3_pcg_ab.sh TAG
set -o pipefail
T=${1:-n}
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" > gpurun_out/r06_${T}_$tag.json 2>> gpurun_out/r06_${T}.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r06_${T}_$tag.json'))
sp=lambda b: {k:(round(v,4) if isinstance(v,float) else v) for k,v in (b.get('solve_path') or {}).items()}
print('$tag', round(d['value']), round(d['ms_per_step'],4), round(d['phase_ms_per_iter']['solve'],4), sp(d))" | tee -a gpurun_out/r06_${T}_ab.txt
}
for rep in 1 2; do
run direct$rep M3S_GN_PCG=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching --no-cfg4
run lag2_$rep M3S_GN_PCG=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching --no-cfg4
run lag3_$rep M3S_GN_PCG=2 M3S_PCG_FROM=4 M3S_PCG_LAG=3 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching --no-cfg4
done
