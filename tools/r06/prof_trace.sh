# kernel trace of a short PCG bench (cfg3) for the timeline of one call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_${1:-i}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_${1:-i}_prof -o trace -- python3 bench.py --no-cpu-baseline --no-matching ${2:---no-cfg4} --steps 3 --warmup 1 > gpurun_out/r06_${1:-i}_prof_bench.json 2> gpurun_out/r06_${1:-i}_prof_bench.err
find gpurun_out/r06_${1:-i}_prof -name "*.csv" | head
