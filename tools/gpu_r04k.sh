#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_gpu_gn.py -k "timeout or two_rank or rccl or dataflow or singular" > gpurun_out/r04k_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r04k_pytest.log; exit 1; }
tail -2 gpurun_out/r04k_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_prof -o cfg4 -- python bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-matching > gpurun_out/r04k_rocprof_cfg4.log 2>&1; echo "rocprof cfg4 exit code $?"
find gpurun_out/r04k_prof -name "*kernel_stats.csv" | head -3
timeout -k 10 600 python bench.py > gpurun_out/r04k_bench.json 2> gpurun_out/r04k_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r04k_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r04k_bench.json'))
print('cfg3', round(d['value']), d['ms_per_step'], d['phase_ms_per_iter'])
print('cfg4 block', {k: d['cfg4'][k] for k in ('value','ms_per_step','phase_ms_per_iter','n_ranks','n_ranks_comm')})
print('ref order', d['accuracy'].get('reference_order_mode'))
print('roofline', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
