"""Per-dispatch durations and gaps of the plan kernel from a rocprofv3 kernel-trace CSV.

usage: python tools/diag/trace_ramp.py <run_kernel_trace.csv> [...]
Prints the first 40 durations and gaps and the mean over windows of the timed loop: the
gaps expose per-group event records, the windows the clock ramp after an idle start.
"""
import csv
import statistics as S
import sys


def main(paths):
    for p in paths:
        rows = [r for r in csv.DictReader(open(p)) if "plan_kernel" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        st = [int(r["Start_Timestamp"]) for r in rows]
        en = [int(r["End_Timestamp"]) for r in rows]
        d = [(e - s) / 1e3 for s, e in zip(st, en)]
        g = [(st[i + 1] - en[i]) / 1e3 for i in range(len(st) - 1)]
        print(p, "dispatches", len(rows))
        print(" duration us, first 40:", " ".join(f"{x:.1f}" for x in d[:40]))
        print(" gap us, first 40:     ", " ".join(f"{x:.1f}" for x in g[:40]))
        for a, b in [(25, 100), (100, 300), (300, 600), (600, 1000), (1000, 1500), (1500, 2000)]:
            if len(d) > b:
                print(f"  dispatches {a}-{b}: duration {S.mean(d[a:b]):.2f} gap {S.mean(g[a:b]):.2f}")


if __name__ == "__main__":
    main(sys.argv[1:])
