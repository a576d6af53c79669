"""Per-kernel statistics (calls, total / average / min / max ns) from a rocprofv3 rocpd SQLite
database -- the `--kernel-trace --stats` summary as CSV, for profiles/.
python tools/r06/db_stats.py DB > out.csv"""
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                 "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage")
for r in rows:
    name = re.sub(r"\s+", " ", r[0]).replace(",", ";")
    print(f"\"{name}\",{r[1]},{r[2]},{r[3]:.1f},{r[4]},{r[5]},{100.0 * r[2] / tot:.2f}")
