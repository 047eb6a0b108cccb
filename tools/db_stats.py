"""rocprofv3 rocpd database (run_results.db) -> kernel_stats-style CSV (name, calls, total ns,
average ns, percentage), for profiles/ summaries when a run was not asked for --output-format csv.
usage: python tools/db_stats.py RUN_RESULTS_DB OUT_CSV"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], round(r[2] * 1000), round(r[3] * 1000), round(r[4], 3)])
print(f"{len(rows)} kernels -> {out}")
