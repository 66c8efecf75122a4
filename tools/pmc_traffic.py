"""HBM bytes per plan-kernel launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(tools/pmc.sh), corrected by the calibration dispatch of tools/pmc_calib.py (8-B/lane
streaming: factor = counter bytes / true bytes), written into profiles/pmc_lookahead.json
under the bench key.  usage: pmc_traffic.py PMC_DIR KEY"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, key = sys.argv[1], sys.argv[2]
n_cal = 1 << 26


def per_dispatch(counter, kname):
    vals = defaultdict(float)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and kname in r.get("Kernel_Name", ""):
                vals[(f, r.get("Dispatch_Id"))] += float(r["Counter_Value"])
    return list(vals.values())


def mean(xs):
    return sum(xs) / len(xs) if xs else float("nan")


f_plan, w_plan = per_dispatch("FETCH_SIZE", "plan_kernel"), per_dispatch("WRITE_SIZE", "plan_kernel")
f_cal = [v for v in per_dispatch("FETCH_SIZE", "math_kernel") if v * 1024 > 1e8]
w_cal = [v for v in per_dispatch("WRITE_SIZE", "math_kernel") if v * 1024 > 1e8]
kf = mean(f_cal) * 1024 / (8 * n_cal)          # counter bytes per true byte (KB units)
kw = mean(w_cal) * 1024 / (8 * n_cal)
fetch, write = mean(f_plan) * 1024, mean(w_plan) * 1024
out = {"kernel": "plan_kernel", "fetch_kb": mean(f_plan), "write_kb": mean(w_plan),
       "calibration": {"fetch_per_true_byte": kf, "write_per_true_byte": kw,
                       "kernel": "math_kernel fn 9, 2^26 doubles in/out, 8 B/lane coalesced"},
       "hbm_bytes_per_launch": fetch / kf + write / kw,
       "hbm_bytes_per_launch_uncorrected": fetch + write,
       "dispatches": len(f_plan),
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/pmc.sh); "
                 "KB units; corrected by the 8-B/lane calibration dispatch", "round": os.environ.get("PMC_ROUND", "r03")}
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_lookahead.json")
try:
    d = json.load(open(path))
except (OSError, ValueError):
    d = {}
d[key] = out
json.dump(d, open(path, "w"), indent=1)
print(json.dumps({key: out}, indent=1))
json.dump({key: out}, open(os.path.join(sys.argv[1], "pmc_lookahead_entry.json"), "w"), indent=1)
