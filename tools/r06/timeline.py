"""Timeline of one GN call from a rocprofv3 kernel-trace database (rocpd SQLite): every dispatch
between the K-th and (K+1)-th launch of a marker kernel, with its start offset, duration, stream
and grid, so overlap between the side stream (the PCG inverse) and the main stream is visible.
python tools/r06/timeline.py DB [marker-substring] [K]"""
import re
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "gn_accum"
K = int(sys.argv[3]) if len(sys.argv) > 3 else -3
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, stream_id, queue_id, grid_x, workgroup_x, lds_size from kernels "
                 "order by start").fetchall()
short = lambda n: re.sub(r"\(.*", "", n).replace("m3s::", "").replace("(anonymous namespace)::", "")[:48]
# a call = the launches from one marker (first accumulate of a call: gap before it) to the next
marks = [i for i, r in enumerate(rows) if marker in r[0]]
calls, prev = [], None
for i in marks:
    if prev is None or rows[i][1] - rows[prev][2] > 200_000:  # > 200 us idle -> a new call
        calls.append(i)
    prev = i
print(f"{len(rows)} dispatches, {len(calls)} calls")
a = calls[K]
b = calls[K + 1] if K + 1 < len(calls) and K != -1 else len(rows)
t0 = rows[a][1]
for r in rows[a:b]:
    print(f"{(r[1]-t0)/1e3:9.1f} {(r[2]-r[1])/1e3:8.1f} us  s{r[3]} q{r[4]}  grid {r[5]//max(r[6],1):5d}x{r[6]:4d} lds {r[7]:6d}  {short(r[0])}")
