#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max ns, %) from a rocprofv3 SQLite results.db,
in the column layout of rocprofv3's kernel_stats.csv. usage: rocpd_stats.py results.db [out.csv]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
lines = ['"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"']
for n, c, s, a, mn, mx in rows:
    lines.append(f'"{n}",{c},{s},{a:.1f},{100.0 * s / tot:.3f},{mn},{mx}')
out = "\n".join(lines) + "\n"
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out)
print(out, end="")
