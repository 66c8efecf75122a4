"""Refresh one kernel's entry of profiles/r05/pmc_kernels.json (the bench's `issue.pmc` input)
from a tools/gpu_r05_prof.sh run: the PMC summary (mean per dispatch) and the kernel trace's
average duration.  usage: python tools/pmc_kernels_update.py <prof dir> ctl|nlp <shape note>"""
import csv
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof, which, shape = sys.argv[1], sys.argv[2], sys.argv[3]
kname = {"ctl": "ctl_kernel", "nlp": "nlp_kernel"}[which]
vals = {}
for line in open(os.path.join(prof, f"pmc_{which}", "summary.txt")):
    m = re.match(r"\s+(\S+)\s+mean/dispatch\s+([0-9.]+)", line)
    if m:
        vals[m.group(1)] = float(m.group(2))
stats = os.path.join(prof, f"trace_{which}", "run_kernel_stats.csv")
avg = None
for r in csv.DictReader(open(stats)):
    if kname in r["Name"]:
        avg = float(r["AverageNs"]) / 1e3
ISSUE_PEAK = 256 * 4 * 16 * 2.4e9          # lane-instructions/s (bench.py ISSUE_PEAK_LANE_INSTR)
e = {k: vals[k] for k in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY",
                          "SQ_ACTIVE_INST_VALU")}
e["FETCH_SIZE_KB"] = vals["FETCH_SIZE"]
e["WRITE_SIZE_KB"] = vals["WRITE_SIZE"]
e["rocprof_avg_us"] = avg
e["issue_frac"] = vals["SQ_INSTS_VALU"] * 64 / (avg * 1e-6) / ISSUE_PEAK
e["wait_share"] = vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]
e["source"] = f"{prof}: trace_{which}/run_kernel_stats.csv (kernel trace) + pmc_{which}/summary.txt (one counter group per run)"
e["shape"] = shape
path = os.path.join(REPO, "profiles", "r05", "pmc_kernels.json")
d = json.load(open(path))
d[kname] = e
json.dump(d, open(path, "w"), indent=1)
print(kname, json.dumps(e, indent=1))
