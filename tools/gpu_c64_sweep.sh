#!/bin/bash
# C=64 N-sweep of the throughput layouts: launch_plan's choice (default), 4-wave and 8-wave
# work queue forced (LLAMPC_WQ_WAVES) and the static block-per-models layout (LLAMPC_NO_WQ=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
OUT=${1:?out dir}; mkdir -p $OUT
NS=${NS:-1000 1500 2000 3000 4000 5000 10000 20000}
A="--steps 40 --warmup 5 --C 64 --cpu-max 0 --n $NS"
timeout -k 10 300 python -u tools/nsweep.py $A > $OUT/auto.jsonl 2> $OUT/auto.err || exit $?
LLAMPC_WQ_WAVES=4 timeout -k 10 300 python -u tools/nsweep.py $A > $OUT/wq4.jsonl 2> $OUT/wq4.err || exit $?
LLAMPC_WQ_WAVES=8 timeout -k 10 300 python -u tools/nsweep.py $A > $OUT/wq8.jsonl 2> $OUT/wq8.err || exit $?
LLAMPC_NO_WQ=1 timeout -k 10 300 python -u tools/nsweep.py $A > $OUT/static.jsonl 2> $OUT/static.err || exit $?
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
ks = ("auto", "static", "wq4", "wq8")
rows = {k: {d["N"]: d["device_ms_per_tick"] * 1e3 for d in map(json.loads, open(f"{o}/{k}.jsonl"))} for k in ks}
print("N      " + "  ".join(f"{k:>8s}" for k in ks) + "   (us per tick, C = 64, H = 20)")
for n in sorted(rows["auto"]):
    print(f"{n:6d} " + "  ".join(f"{rows[k].get(n, float('nan')):8.1f}" for k in ks))
PY
