#!/bin/bash
# Tail-factor diagnostics: the solve's phase clocks for diagnostic builds (lib/variants/tdiag*.so:
# no L stores / no MFMA / no extraction; timing only, wrong results) against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r03i}"
for v in default ${VARIANTS:-tdiag1 tdiag2 tdiag4 tdiag7}; do
    lib=$PWD/mast3r-slam_amd/lib/libm3s_backend.so
    [ $v != default ] && lib=$PWD/mast3r-slam_amd/lib/variants/$v.so
    M3S_BACKEND_LIB=$lib timeout -k 10 120 python tools/solve_debug.py cfg3 3 > gpurun_out/${TAG}_$v.log 2>&1 || { echo "$v failed"; tail -n 5 gpurun_out/${TAG}_$v.log; exit 1; }
    python - "$v" gpurun_out/${TAG}_$v.log <<'PY'
import sys, re
v, f = sys.argv[1], sys.argv[2]
txt = open(f).read().split("gn_solve entry->first tick")[-1]
vals = {}
steps = []
for line in txt.splitlines():
    m = re.match(r"gn_solve\s+(.*?)\s+([-\d.]+) us", line)
    if not m: continue
    k, t = m.group(1).strip(), float(m.group(2))
    if k.startswith("K:"): steps.append(t)
    else: vals[k] = t
fac = sum(steps) + vals.get("tail factor", 0)
print(f"{v:8s} entry->exit {vals.get('entry->exit',0):7.2f}  tail factor {fac:6.2f}  back {vals.get('tail back',0):6.2f}  rounds {vals.get('back rounds',0):6.2f}  last steps " + " ".join(f"{x:.2f}" for x in steps[-6:]))
PY
done
