set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r06/pcg_debug.py > gpurun_out/r06_${1:-g}_pcg_debug.log 2>&1 || { tail -30 gpurun_out/r06_${1:-g}_pcg_debug.log; exit 1; }
grep -E "inverse|pcg\[(2|3)\]|pcg_runs" gpurun_out/r06_${1:-g}_pcg_debug.log | head -40
