#!/bin/bash
# reference-order accumulate rebuilt (point math unrolled, branch-free, f32 IEEE 1/x, no SLP):
# bitwise A/B of Hs / gs / poses against the previous build, timing per unroll, parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05af
mkdir -p $O
export TMPDIR=/tmp
for v in old def u1 u3 u4; do
if [ $v = def ]; then L=mast3r-slam_amd/lib/libm3s_backend.so; else L=mast3r-slam_amd/lib/ab_$v/libm3s_backend.so; fi
M3S_BACKEND_LIB=$L timeout -k 10 300 python tools/r05/refacc_ab.py $O/$v.npz > $O/$v.json 2> $O/$v.err || { echo "ab $v rc=$?"; tail -5 $O/$v.err; exit 1; }
cat $O/$v.json
done
python - <<'PY'
import numpy as np
O = "gpurun_out/r05af"
a = np.load(f"{O}/old.npz")
for v in ("def", "u1", "u3", "u4"):
    b = np.load(f"{O}/{v}.npz")
    bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
    print(v, "bitwise equal to old:", not bad, bad[:6])
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_gn_reference_order.py tests/test_gpu_gn_stress.py > $O/pytest_ref.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest_ref.log; exit 1; }
tail -2 $O/pytest_ref.log
