"""Diagnostic: the durations (and gaps) of one kernel's dispatches in a rocprofv3 kernel trace,
in dispatch order.  usage: python tools/diag/trace_list.py <kernel_trace.csv> <name-substring> [last]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
prev = None
for i, r in enumerate(rows[-last:]):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{i:4d} dur {(e - s) / 1e3:7.2f} us  gap {((s - prev) / 1e3) if prev else 0:8.2f} us")
    prev = e
