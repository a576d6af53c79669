set -o pipefail
T=${1:-x}
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py -s > gpurun_out/r06_${T}_pytest_pcg.log 2>&1 || { tail -30 gpurun_out/r06_${T}_pytest_pcg.log; exit 1; }
tail -2 gpurun_out/r06_${T}_pytest_pcg.log
bash tools/r06/ab_env.sh $T 2 "" df1="M3S_SOLVE_DF=1" df0="M3S_SOLVE_DF=0" df2="M3S_SOLVE_DF=2" || exit 1
M3S_SOLVE_DF=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gn.py > gpurun_out/r06_${T}_pytest_gn_df2.log 2>&1; tail -3 gpurun_out/r06_${T}_pytest_gn_df2.log
