set -o pipefail
M3S_PCG_ONEX=1 timeout -k 10 300 python -u tools/r06/pcg_debug.py cfg3 > gpurun_out/r06_ox_debug.log 2>&1 || { tail -20 gpurun_out/r06_ox_debug.log; exit 1; }
grep -E "pcg\[(2|3)\]|pcg_runs" gpurun_out/r06_ox_debug.log | head -6
timeout -k 10 300 python -u tools/r06/pcg_debug.py cfg3 > gpurun_out/r06_ox_debug0.log 2>&1 || exit 1
grep -E "pcg\[(2|3)\]" gpurun_out/r06_ox_debug0.log | head -3
bash tools/r06/ab_env.sh ox 3 "--no-cfg4" onex="M3S_PCG_ONEX=1" base="M3S_PCG_ONEX=0"
