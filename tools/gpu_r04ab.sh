#!/bin/bash
# iter_proj: gradients gathered with the trial point's rays (one round trip per iteration)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_matching.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for B in 8 1; do
B=$B timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace$B -o run -- python tools/iter_proj_probe.py > $O/trace$B.log 2>&1 || exit 1
find $O/trace$B -type f ! -name "*kernel_stats.csv" -delete
python - $O/trace$B/run_kernel_stats.csv $B <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "iter_proj" in r["Name"]:
        print("B=" + sys.argv[2], r["Name"][:45], r["Calls"], "avg us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
