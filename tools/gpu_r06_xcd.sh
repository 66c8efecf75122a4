#!/bin/bash
# Round 6 (verdict r05 #8): the plan kernel's XCD-aligned look-back and two-word C = 1 results.
# The whole GPU suite, then the C = 1 PMC passes with the layout on and off (LLAMPC_LB_XCD=0),
# an alternating A/B of the tick (K = 200, three pairs), and the one-device 2-rank rehearsal.
# usage (gpurun): bash tools/gpu_r06_xcd.sh gpurun_out/<tag> [skiptests]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
if [ "$2" != "skiptests" ]; then
  step "gpu tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputest.log" 2>&1
  rc=$?
  tail -3 "$OUT/gputest.log"
  [ $rc -eq 0 ] || { step "pytest rc=$rc: stopping"; exit $rc; }
fi
step "PMC C=1, XCD-aligned"
PMC_ROUND="r06 XCD-aligned look-back" PMC_OUT=$OUT/pmc_on bash tools/pmc.sh --steps 40 --warmup 10 > "$OUT/pmc_on.txt" 2>&1 || { tail -5 "$OUT/pmc_on.txt"; exit 1; }
step "PMC C=1, contiguous"
LLAMPC_LB_XCD=0 PMC_ROUND="r06 contiguous look-back" PMC_OUT=$OUT/pmc_off bash tools/pmc.sh --steps 40 --warmup 10 > "$OUT/pmc_off.txt" 2>&1 || { tail -5 "$OUT/pmc_off.txt"; exit 1; }
grep -E "FETCH_SIZE|WRITE_SIZE" "$OUT/pmc_on.txt" "$OUT/pmc_off.txt"
for rep in 1 2 3; do
  for v in on off; do
    step "A/B $v rep $rep"
    if [ $v = off ]; then export LLAMPC_LB_XCD=0; else unset LLAMPC_LB_XCD; fi
    timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-call-latency > "$OUT/ab_${v}_$rep.json" 2> "$OUT/ab_${v}_$rep.err" || exit $?
  done
done
unset LLAMPC_LB_XCD
python3 - "$OUT" <<'PY' | tee "$OUT/ab_summary.txt"
import json, sys, glob
out = sys.argv[1]
for v in ("on", "off"):
    r = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/ab_{v}_*.json"))]
    print(v, "us/tick", [round(x["ms_per_step"] * 1e3, 2) for x in r], "kernel", [round(x["roofline"]["kernel_avg_us"], 2) for x in r])
PY
step "bench 2 ranks, self-spawned, one device"
LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline \
  > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err" || exit $?
step "done"
