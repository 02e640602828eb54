"""Summarise a rocprofv3 rocpd database (kernel name, calls, total/avg/min/max ns)
into CSV like rocprofv3's kernel_stats.csv.  usage: rocpd_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
out = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
out.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
for r in rows:
    out.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / tot, 2)])
