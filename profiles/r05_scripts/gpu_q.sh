#!/bin/bash
# edge lists to the host by the staging kernel instead of DMA copies: GN tests, per-call host
# phases (M3S_PROF_HOST) A/B against M3S_STAGE_DMA=1, the 2-rank rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gn.py tests/test_gpu_dist.py tests/test_gpu_factor_graph.py tests/test_gpu_gn_stress.py tests/test_gpu_gn_reference_order.py > $O/pytest_gn.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_gn.log; exit 1; }
tail -1 $O/pytest_gn.log
for dma in 0 1; do
M3S_STAGE_DMA=$dma M3S_PROF_HOST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching --steps 5 --warmup 2 > $O/n1_dma$dma.json 2> $O/n1_dma$dma.err || { echo "n1 rc=$?"; tail -10 $O/n1_dma$dma.err; exit 1; }
echo "dma=$dma"; grep "gn host: build_plan" $O/n1_dma$dma.err | tail -4; grep "gn host: setup" $O/n1_dma$dma.err | tail -2
python -c "import json; d=json.load(open('$O/n1_dma$dma.json')); c=d['cfg4']; print('cfg3', round(d['value']), round(d['ms_per_step'],3), 'cfg4', round(c['value']), round(c['ms_per_step'],3))"
done
M3S_BENCH_COMM=host M3S_PROF_HOST=1 timeout -k 10 400 python bench.py --gpus 2 --no-matching --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "n2 rc=$?"; tail -10 $O/n2.err; exit 1; }
grep "gn host" $O/n2.err | tail -8
