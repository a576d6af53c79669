set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py -k held -s > gpurun_out/r06_held_pcg.log 2>&1 || { tail -30 gpurun_out/r06_held_pcg.log; exit 1; }
tail -1 gpurun_out/r06_held_pcg.log
bash tools/r06/rehearse2.sh
