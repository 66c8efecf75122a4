"""Per-kernel PMC means (tools/pmc_summary.py output) + the kernel trace's average duration ->
one JSON entry per kernel (the bench's `issue.pmc` reads it: bench.py pmc_issue).
usage: python tools/pmc_kernels.py out.json KERNEL=summary.txt,kernel_stats.csv[,shape] ..."""
import csv
import json
import re
import sys

ISSUE_PEAK = 256 * 4 * 16 * 2.4e9       # lanes/cycle x clock: bench.py ISSUE_PEAK_LANE_INSTR


def parse_summary(path, kernel):
    vals, on = {}, False
    for line in open(path):
        if not line.startswith(" "):
            on = kernel in line
            continue
        m = re.match(r"\s+(\w+)\s+mean/dispatch\s+([\d.]+)", line)
        if on and m:
            vals[m.group(1)] = float(m.group(2))
    return vals


def main():
    out, entries = sys.argv[1], {}
    for spec in sys.argv[2:]:
        name, rest = spec.split("=", 1)
        parts = rest.split(",")
        summ, stats = parts[0], parts[1]
        v = parse_summary(summ, name)
        avg = next(float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(stats)) if name in r["Name"])
        e = {k: v[k] for k in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
                               "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE") if k in v}
        if "FETCH_SIZE" in v:
            e["FETCH_SIZE_KB"] = v["FETCH_SIZE"]
        if "WRITE_SIZE" in v:
            e["WRITE_SIZE_KB"] = v["WRITE_SIZE"]
        e["rocprof_avg_us"] = avg
        e["issue_frac"] = e["SQ_INSTS_VALU"] * 64 / (avg * 1e-6) / ISSUE_PEAK
        e["wait_share"] = e["SQ_WAIT_ANY"] / e["SQ_WAVE_CYCLES"]
        e["source"] = f"{stats} (kernel trace) + {summ} (one counter group per run)"
        if len(parts) > 2:
            e["shape"] = parts[2]
        entries[name] = e
    json.dump(entries, open(out, "w"), indent=1)
    print(json.dumps(entries, indent=1))


if __name__ == "__main__":
    main()
