#!/bin/bash
# Round 6: alternating A/B of library builds on the headline tick (same box, same command).
# usage (gpurun): bash tools/gpu_r06_ablibs.sh gpurun_out/<tag> "libA libB ..." [reps] [bench args]
# (libs: names under lla-mpc_amd/llampc/_lib/, e.g. libllampc_hip.so)
set -o pipefail
OUT=${1:?out dir}
LIBS=${2:?libs}
REPS=${3:-3}
shift 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
for rep in $(seq 1 $REPS); do
  for lib in $LIBS; do
    echo "[$(date +%T)] $lib rep $rep"
    LLAMPC_HIP_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-call-latency "$@" \
      > "$OUT/ab_${lib}_$rep.json" 2> "$OUT/ab_${lib}_$rep.err" || exit $?
  done
done
python3 - "$OUT" $LIBS <<'PY' | tee "$OUT/ab_summary.txt"
import json, sys, glob
out = sys.argv[1]
for lib in sys.argv[2:]:
    r = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/ab_{lib}_*.json"))]
    print(f"{lib:28s} us/tick", [round(x["ms_per_step"] * 1e3, 2) for x in r], "kernel", [round(x["roofline"]["kernel_avg_us"], 2) for x in r])
PY
