"""Kernel statistics (name, calls, total ns, average ns, percent) from a rocprofv3 rocpd
database (the default output format) as CSV.  usage: prof_db_stats.py run_results.db > kernel_stats.csv"""
import csv
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for name, calls, total_us, avg_us, pct in c.execute(
        "select name, total_calls, total_duration, average, percentage from top_kernels"):
    w.writerow([name, calls, round(total_us * 1e3), round(avg_us * 1e3, 1), round(pct, 3)])
