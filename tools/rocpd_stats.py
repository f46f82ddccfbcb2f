#!/usr/bin/env python
"""Per-kernel stats from a rocprofv3 rocpd SQLite database (ROCm 7 default output):
python tools/rocpd_stats.py RESULTS.db [OUT.csv] -- name, calls, average / total / min / max us."""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1000.0, "
                 "min(end - start) / 1000.0, max(end - start) / 1000.0 from kernels group by name "
                 "order by 4 desc").fetchall()
hdr = ["Name", "Calls", "AverageUs", "TotalUs", "MinUs", "MaxUs"]
out = csv.writer(open(sys.argv[2], "w", newline="")) if len(sys.argv) > 2 else None
if out:
    out.writerow(hdr)
for r in rows:
    if out:
        out.writerow([r[0], r[1]] + [round(v, 3) for v in r[2:]])
    print(f"{r[0][:70]:70s} {r[1]:5d} {r[2]:10.1f} {r[3]:10.1f}")
