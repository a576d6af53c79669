# GPU check after a solve-path change: the PCG tests, then the GN tests, then a short bench.
# usage: bash tools/r06/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-x}
K=${2:-}
OUT=gpurun_out/r06_${TAG}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_pcg.py ${K:+-k "$K"} > ${OUT}_pytest_pcg.log 2>&1 || { tail -30 ${OUT}_pytest_pcg.log; exit 1; }
tail -3 ${OUT}_pytest_pcg.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_dist.py -s > ${OUT}_pytest_gn.log 2>&1 || { tail -30 ${OUT}_pytest_gn.log; exit 1; }
tail -3 ${OUT}_pytest_gn.log
M3S_PROF_HOST=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-matching > ${OUT}_bench.json 2> ${OUT}_bench.err || { tail -20 ${OUT}_bench.err; exit 1; }
python - <<PY
import json; d=json.load(open('${OUT}_bench.json'))
print('cfg3', round(d['value']), d['phase_ms_per_iter'], d.get('solve_path'))
c=d['cfg4']; print('cfg4', round(c['value']), c['phase_ms_per_iter'], c.get('solve_path'))
PY
