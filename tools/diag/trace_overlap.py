"""Diagnostic: overlap of a kernel's consecutive dispatches in a rocprofv3 kernel trace (CSV):
per pair of dispatches of the named kernel, start gap and overlap, and their queues.
usage: python tools/diag/trace_overlap.py <kernel_trace.csv> <kernel-name-substring>"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = np.array([int(r["Start_Timestamp"]) for r in rows]) / 1e3
en = np.array([int(r["End_Timestamp"]) for r in rows]) / 1e3
q = [r["Queue_Id"] for r in rows]
dur = en - st
ov = [min(en[i], en[i + 1]) - max(st[i], st[i + 1]) for i in range(0, len(st) - 1, 2)]
print(f"{len(rows)} dispatches; duration us p50 {np.median(dur):.1f}; queues {sorted(set(q))}")
print(f"pairs: overlap us p50 {np.median(ov):.1f} min {np.min(ov):.1f} max {np.max(ov):.1f}; "
      f"second start - first start p50 {np.median(st[1::2][:len(ov)] - st[0::2][:len(ov)]):.1f}")
for i in range(0, min(len(st) - 1, 12), 2):
    print(f"  {st[i] - st[0]:10.1f} {dur[i]:6.1f} q{q[i]} | {st[i + 1] - st[0]:10.1f} {dur[i + 1]:6.1f} q{q[i + 1]}")
