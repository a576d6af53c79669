set -o pipefail
T=${1:-z}
M3S_SOLVE_DF=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py > gpurun_out/r06_${T}_pytest_gn_df2.log 2>&1 || { tail -30 gpurun_out/r06_${T}_pytest_gn_df2.log; exit 1; }
tail -1 gpurun_out/r06_${T}_pytest_gn_df2.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py > gpurun_out/r06_${T}_pytest_pcg.log 2>&1 || { tail -30 gpurun_out/r06_${T}_pytest_pcg.log; exit 1; }
tail -1 gpurun_out/r06_${T}_pytest_pcg.log
bash tools/r06/ab_env.sh $T 3 "" f4="M3S_GN_PCG=1" f3="M3S_PCG_FROM=3" direct="M3S_GN_PCG=0"
