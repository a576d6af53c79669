set -o pipefail
T=${1:-p}
bash tools/r06/ab_env.sh $T 2 "--no-cfg4" direct="M3S_GN_PCG=0" pcg="M3S_GN_PCG=2" pcg_twox="M3S_GN_PCG=2 M3S_PCG_ONEX=0" pcg_roundfb="M3S_GN_PCG=2 M3S_PCG_FALLBACK_COOP=0" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py -s > gpurun_out/r06_${T}_pytest_pcg.log 2>&1; tail -3 gpurun_out/r06_${T}_pytest_pcg.log
