#!/bin/bash
# Round 6: alternating A/B of library builds on the NLP solve latency (same box, same command).
# usage (gpurun): bash tools/gpu_r06_abnlp.sh gpurun_out/<tag> "libA libB ..." [reps]
set -o pipefail
OUT=${1:?out dir}
LIBS=${2:?libs}
REPS=${3:-3}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
for rep in $(seq 1 $REPS); do
  for lib in $LIBS; do
    echo "[$(date +%T)] $lib rep $rep"
    LLAMPC_HIP_LIB=$L/$lib timeout -k 10 120 python -u -c "
import sys, json, argparse; sys.argv=['bench.py']; import bench
print(json.dumps(bench.solve_latency(argparse.Namespace())))" > "$OUT/nlp_${lib}_$rep.json" 2> "$OUT/nlp_${lib}_$rep.err" || exit $?
  done
done
python3 - "$OUT" $LIBS <<'PY' | tee "$OUT/abnlp_summary.txt"
import json, sys, glob
out = sys.argv[1]
for lib in sys.argv[2:]:
    r = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/nlp_{lib}_*.json"))]
    print(f"{lib:28s} p50", [round(x["p50"], 1) for x in r], "p99", [round(x["p99"], 1) for x in r],
          "kernel", [round(x["kernel_us_avg"], 1) for x in r])
PY
