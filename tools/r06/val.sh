# validation after a solve-path change: PCG debug clocks + direct/PCG A/B, PCG tests, GN suites
set -o pipefail
T=${1:-j}
bash tools/r06/pcg_ab.sh $T || exit 1
grep -E "inverse" gpurun_out/r06_${T}_pcg_debug.log | grep -v " [0-9]\.[0-9] us" | head -6
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_gn_stress.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py -s > gpurun_out/r06_${T}_pytest_gn.log 2>&1; tail -4 gpurun_out/r06_${T}_pytest_gn.log; grep -E "stress iters" gpurun_out/r06_${T}_pytest_gn.log | head -12
