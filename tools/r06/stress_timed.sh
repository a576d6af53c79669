set -o pipefail
T=${1:-w}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn_stress.py -s -k "timed_kernel or default_path" > gpurun_out/r06_${T}_pytest_stress.log 2>&1; rc=$?; grep -E "stress iters|passed|failed|Error" gpurun_out/r06_${T}_pytest_stress.log | head -20; exit $rc
