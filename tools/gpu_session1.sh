export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_gn.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gn.log
if [ $rc -gt 1 ]; then exit $rc; fi
VARIANTS="default multi hybrid fused" timeout -k 10 300 bash tools/ab_solver.sh || exit 1
M3S_SOLVER=3 M3S_SOLVE_DEBUG=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --iters 3 --no-cpu-baseline --no-matching > gpurun_out/dbg.json 2> gpurun_out/dbg.err
echo "dbg rc=$?"; grep -E "solve plan|round:|gn_solve" gpurun_out/dbg.err | head -40
