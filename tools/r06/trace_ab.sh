# kernel traces of cfg4 with the direct solve and with the PCG, same box, then per-iteration accumulate times
set -o pipefail
T=${1:-u}
M3S_GN_PCG=0 bash tools/r06/prof_trace.sh ${T}d "--config cfg4 --no-cfg4" || exit 1
bash tools/r06/prof_trace.sh ${T}p "--config cfg4 --no-cfg4" || exit 1
for v in d p; do
python - gpurun_out/r06_${T}${v}_prof/trace_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels where name like '%gn_accum_packed_kernel%' order by start").fetchall()
d = [(r[2]-r[1])/1e3 for r in rows]
# calls of 10: the first of a call is the records-building one (longest)
print(sys.argv[1].split('/')[1], 'accumulate launches', len(d))
for i in range(0, min(len(d), 60), 10):
    print(' '.join('%7.1f' % x for x in d[i:i+10]))
PY
done
