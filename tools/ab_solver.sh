#!/bin/bash
# A/B of the GN solve variants on the bench graph (cfg3 unless CFG is set): phase ms/iter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG="${CFG:-cfg3}"
run() {  # $1 label, rest env assignments
    local label=$1; shift
    env "$@" timeout -k 10 120 python bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-matching \
        > gpurun_out/ab_$label.json 2> gpurun_out/ab_$label.err || { echo "$label FAILED rc=$?"; tail -5 gpurun_out/ab_$label.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$label.json')); p=d['phase_ms_per_iter']; print('%-24s ms/step %.3f  acc %.3f sys %.3f solve %.3f retr %.3f' % ('$label', d['ms_per_step'], p['accumulate'], p['reduce_compact_allreduce'], p['solve'], p['retract']))"
}
for v in ${VARIANTS:-default}; do
    case $v in
    default) run default M3S_X=0 ;;
    fused) run fused M3S_SOLVER=1 M3S_FUSED_MAX_ROUNDS=64 ;;
    fused_nosplit) run fused_nosplit M3S_SOLVER=1 M3S_FUSED_MAX_ROUNDS=64 M3S_SOLVE_SPLIT=0 ;;
    fused_nommd) run fused_nommd M3S_SOLVER=1 M3S_SPARSE_MMD=0 M3S_FUSED_MAX_ROUNDS=64 ;;
    multi) run multi M3S_SOLVER=2 ;;
    multi_mmd) run multi_mmd M3S_SOLVER=2 M3S_MULTI_MMD=1 ;;
    hybrid) run hybrid M3S_SOLVER=3 ;;
    dense) run dense M3S_SOLVER_DENSE=1 ;;
    esac
done
