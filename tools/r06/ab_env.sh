# same-box A/B of bench variants, interleaved REPS times: bash tools/r06/ab_env.sh TAG REPS "BENCH ARGS" tag1="ENV..." tag2="ENV..."
# prints per run: value, ms/step, solve ms/iter, solve_path (headline block, and cfg4's when present)
set -o pipefail
T=$1; REPS=$2; BARGS=$3; shift 3
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    tag=${v%%=*}; envs=${v#*=}
    env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching $BARGS > gpurun_out/r06_${T}_${tag}_$rep.json 2>> gpurun_out/r06_${T}.err || exit 1
    python -c "
import json;d=json.load(open('gpurun_out/r06_${T}_${tag}_$rep.json'))
sp=lambda b: {k:(round(v,4) if isinstance(v,float) else v) for k,v in (b.get('solve_path') or {}).items() if k in ('pcg_iterations','pcg_fallbacks','cg_steps_per_pcg_solve','solve_ms_before_pcg','solve_ms_pcg_iterations')}
s='${tag}_$rep %d %.4f %.4f %s' % (d['value'], d['ms_per_step'], d['phase_ms_per_iter']['solve'], sp(d))
if 'cfg4' in d: s += ' | cfg4 %d %.4f %s' % (d['cfg4']['value'], d['cfg4']['phase_ms_per_iter']['solve'], sp(d['cfg4']))
print(s)" | tee -a gpurun_out/r06_${T}_ab.txt
  done
done
