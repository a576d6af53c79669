# A/B on one box: the round-5 library (lib_r05, its bench) vs this tree's direct solve vs PCG
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env..., cmd
  tag=$1; shift
  env "$@" > gpurun_out/r06_e_$tag.json 2>> gpurun_out/r06_e.err || exit 1
  python -c "
import json;d=json.load(open('gpurun_out/r06_e_$tag.json'))
print('$tag', round(d['value']), {k:round(v,4) for k,v in d['phase_ms_per_iter'].items()}, round(d['cfg4']['value']), {k:round(v,4) for k,v in d['cfg4']['phase_ms_per_iter'].items()}, d.get('solve_path'), d['cfg4'].get('solve_path'))" | tee -a gpurun_out/r06_e_ab.txt
}
run r05 M3S_BACKEND_LIB=mast3r-slam_amd/lib_r05/libm3s_backend.so timeout -k 10 200 python -u bench_r05.py --no-cpu-baseline --no-matching
run direct M3S_GN_PCG=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching
run pcg timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-matching
run r05b M3S_BACKEND_LIB=mast3r-slam_amd/lib_r05/libm3s_backend.so timeout -k 10 200 python -u bench_r05.py --no-cpu-baseline --no-matching
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_pcg.py -s > gpurun_out/r06_e_pytest_pcg.log 2>&1; tail -12 gpurun_out/r06_e_pytest_pcg.log
timeout -k 10 300 python -u tools/r06/pcg_debug.py > gpurun_out/r06_e_pcg_debug.log 2>&1; tail -20 gpurun_out/r06_e_pcg_debug.log
