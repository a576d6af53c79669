#!/bin/bash
# Instruction-cache counters of the GN kernels (cfg3, 3 iterations): is the solve kernel's first
# pass through its ~200 KB of code cold-miss bound?  Its own pass, kernel trace only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH --output-format csv -d $OUT -o run -- \
    python bench.py --steps 1 --warmup 0 --iters 3 --no-cpu-baseline --no-matching > $OUT.log 2>&1
rc=$?; echo "pmc icache rc=$rc"; tail -n 3 $OUT.log
python tools/pmc_filter.py $OUT
python - <<'PY'
import csv, collections, glob
rows = []
for f in glob.glob("gpurun_out/pmc_icache/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()}, "launches", len(next(iter(v.values()))))
PY
exit $rc
