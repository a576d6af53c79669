#!/bin/bash
# Round-3 GPU session: full GPU tests, smoke, bench cfg3 (default), bench cfg4 + its rocprofv3
# kernel stats.  Every GPU step has its own limit; after a fault / abort / timeout nothing else
# touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r03}"
STEPS="${STEPS:-tests smoke bench bench4 prof4}"
ok_or_fail() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (rc=$1)"; exit "$1"; fi; }
for s in $STEPS; do
    case "$s" in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 \
            --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
        rc=$?; echo "pytest gpu rc=$rc"; tail -n 5 gpurun_out/${TAG}_pytest_gpu.log; ok_or_fail $rc pytest ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
        rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/${TAG}_smoke.log; ok_or_fail $rc smoke ;;
    bench)
        timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
        rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; tail -n 3 gpurun_out/${TAG}_bench.err; ok_or_fail $rc bench ;;
    gntests)
        timeout -k 10 600 python -u -m pytest tests/test_gpu_gn.py tests/test_gpu_gn_reference_order.py -x -q \
            -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gn.log 2>&1
        rc=$?; echo "pytest gn rc=$rc"; tail -n 5 gpurun_out/${TAG}_pytest_gn.log; ok_or_fail $rc pytest_gn ;;
    qbench)
        timeout -k 10 300 python bench.py --no-cpu-baseline --no-matching > gpurun_out/${TAG}_qbench.json 2> gpurun_out/${TAG}_qbench.err
        rc=$?; echo "qbench rc=$rc"; cat gpurun_out/${TAG}_qbench.json; tail -n 3 gpurun_out/${TAG}_qbench.err; ok_or_fail $rc qbench ;;
    qbench4)
        timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-matching > gpurun_out/${TAG}_qbench4.json 2> gpurun_out/${TAG}_qbench4.err
        rc=$?; echo "qbench4 rc=$rc"; cat gpurun_out/${TAG}_qbench4.json; tail -n 3 gpurun_out/${TAG}_qbench4.err; ok_or_fail $rc qbench4 ;;
    bench4)
        timeout -k 10 600 python bench.py --config cfg4 --no-matching \
            > gpurun_out/${TAG}_bench_cfg4.json 2> gpurun_out/${TAG}_bench_cfg4.err
        rc=$?; echo "bench cfg4 rc=$rc"; cat gpurun_out/${TAG}_bench_cfg4.json; tail -n 3 gpurun_out/${TAG}_bench_cfg4.err; ok_or_fail $rc bench4 ;;
    prof)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof \
            -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-matching \
            > gpurun_out/${TAG}_prof.log 2>&1
        rc=$?; echo "rocprof rc=$rc"; tail -n 3 gpurun_out/${TAG}_prof.log
        rm -f gpurun_out/${TAG}_prof/*kernel_trace.csv; ok_or_fail $rc rocprof ;;
    prof4)
        M3S_EXIT_MAPS=gpurun_out/${TAG}_prof4_maps.txt timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof4 \
            -o run -- python bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-matching \
            > gpurun_out/${TAG}_prof4.log 2>&1
        rc=$?; echo "rocprof cfg4 rc=$rc"; tail -n 3 gpurun_out/${TAG}_prof4.log
        rm -f gpurun_out/${TAG}_prof4/*kernel_trace.csv; ok_or_fail $rc rocprof4 ;;
    matching)
        timeout -k 10 600 python -u -m pytest tests/test_gpu_matching.py -x -q -p no:cacheprovider --timeout 400 \
            --timeout-method thread > gpurun_out/${TAG}_pytest_matching.log 2>&1
        rc=$?; echo "pytest matching rc=$rc"; tail -n 5 gpurun_out/${TAG}_pytest_matching.log; ok_or_fail $rc pytest_matching ;;
    alltests)  # every GPU test, no -x, passing tests' prints kept (-rP)
        timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rfEP -p no:cacheprovider --timeout 400 \
            --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
        rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed" gpurun_out/${TAG}_pytest_gpu.log | tail -n 3; ok_or_fail $rc pytest ;;
    probe)  # accuracy probe of the default library, with the H / b split of the first step
        timeout -k 10 600 python tools/accuracy_probe.py --tag default ${PROBE_ARGS:---system} \
            >> gpurun_out/${TAG}_accprobe.jsonl 2>> gpurun_out/${TAG}_accprobe.err
        rc=$?; echo "accprobe default rc=$rc"; tail -n 1 gpurun_out/${TAG}_accprobe.jsonl; ok_or_fail $rc accprobe ;;
    abrays)  # rays-mode norm variants (lib/variants/rcr{0,1,2}.so): accuracy probe + cfg4 timing
        for v in ${VARIANTS:-rcr0 rcr1 rcr2}; do
            M3S_BACKEND_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so timeout -k 10 400 python tools/accuracy_probe.py \
                --tag $v >> gpurun_out/${TAG}_accprobe.jsonl 2>> gpurun_out/${TAG}_accprobe.err
            rc=$?; echo "accprobe $v rc=$rc"; tail -n 1 gpurun_out/${TAG}_accprobe.jsonl; ok_or_fail $rc accprobe_$v
            M3S_BACKEND_LIB=$PWD/mast3r-slam_amd/lib/variants/$v.so timeout -k 10 300 python bench.py --config cfg4 \
                --no-cpu-baseline --no-matching > gpurun_out/${TAG}_qbench4_$v.json 2> gpurun_out/${TAG}_qbench4_$v.err
            rc=$?; echo "qbench4 $v rc=$rc"; cat gpurun_out/${TAG}_qbench4_$v.json; ok_or_fail $rc qbench4_$v
        done ;;
    rehearse2)  # the 2-rank bench flow on this one GPU (gloo + host all-reduce instead of RCCL)
        M3S_BENCH_COMM=host timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
            --no-matching > gpurun_out/${TAG}_rehearse2.json 2> gpurun_out/${TAG}_rehearse2.err
        rc=$?; echo "rehearse2 rc=$rc"; cat gpurun_out/${TAG}_rehearse2.json; tail -n 3 gpurun_out/${TAG}_rehearse2.err; ok_or_fail $rc rehearse2 ;;
    repro0)  # diagnostics of the exit-time SIGSEGV: no cooperative launch
        timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_repro0 -o run \
            -- tools/bin/repro_coop_exit 0 > gpurun_out/${TAG}_repro0.log 2>&1
        rc=$?; echo "repro coop=0 rc=$rc"; tail -n 2 gpurun_out/${TAG}_repro0.log; ok_or_fail $rc repro0 ;;
    repro1)  # ... one cooperative launch (may fault at exit: run it last)
        timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_repro1 -o run \
            -- tools/bin/repro_coop_exit 1 > gpurun_out/${TAG}_repro1.log 2>&1
        rc=$?; echo "repro coop=1 rc=$rc"; tail -n 2 gpurun_out/${TAG}_repro1.log; ok_or_fail $rc repro1 ;;
    prof4nocoop)  # cfg4 with the per-panel factorisation (no cooperative launch)
        M3S_CHOL_DF=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof4nc \
            -o run -- python bench.py --config cfg4 --steps 3 --warmup 1 --no-cpu-baseline --no-matching \
            > gpurun_out/${TAG}_prof4nc.log 2>&1
        rc=$?; echo "rocprof cfg4 (no coop) rc=$rc"; tail -n 3 gpurun_out/${TAG}_prof4nc.log
        rm -f gpurun_out/${TAG}_prof4nc/*kernel_trace.csv; ok_or_fail $rc rocprof4nc ;;
    esac
done
exit 0
