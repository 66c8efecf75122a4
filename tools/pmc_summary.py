"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: mean counter value per dispatch."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
pats = sys.argv[2].split(",") if len(sys.argv) > 2 else ["plan_kernel", "merge"]   # kernel-name filters
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        name = r.get("Counter_Name", "?")
        try:
            v = float(r.get("Counter_Value", "nan"))
        except ValueError:
            continue
        vals[k][(name, r.get("Dispatch_Id"))].append(v)
for k, d in vals.items():
    if not any(p in k for p in pats):
        continue
    per = defaultdict(list)
    for (name, disp), v in d.items():
        per[name].append(sum(v))          # sum over instances/dimensions of one dispatch
    print(k[:110])
    for name in sorted(per):
        xs = per[name]
        print(f"   {name:28s} mean/dispatch {sum(xs)/len(xs):16.1f}   dispatches {len(xs)}")
