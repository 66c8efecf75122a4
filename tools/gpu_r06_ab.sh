#!/bin/bash
# Round 6: alternating A/B of the shipped library against round 5's (same box, same bench
# command; libllampc_r05.so built from e70587a, git-ignored), the NLP phase stamps, and the
# default bench line (extras included).
# usage (gpurun): bash tools/gpu_r06_ab.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
step() { echo "[$(date +%T)] $*"; }
L=$PWD/lla-mpc_amd/llampc/_lib
for rep in 1 2 3; do
  for v in r06 r05; do
    lib=$L/libllampc_hip.so; [ $v = r05 ] && lib=$L/libllampc_r05.so
    step "A/B $v rep $rep"
    LLAMPC_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --no-call-latency \
      > "$OUT/ab_${v}_$rep.json" 2> "$OUT/ab_${v}_$rep.err" || exit $?
    LLAMPC_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline \
      --no-call-latency > "$OUT/ab20_${v}_$rep.json" 2> "$OUT/ab20_${v}_$rep.err" || exit $?
  done
done
python3 - "$OUT" <<'PY' | tee "$OUT/ab_summary.txt"
import json, sys, glob
out = sys.argv[1]
for pre in ("ab", "ab20"):
    for v in ("r06", "r05"):
        r = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{out}/{pre}_{v}_*.json"))]
        print(pre, v, "us/tick", [round(x["ms_per_step"] * 1e3, 2) for x in r], "kernel", [round(x["roofline"]["kernel_avg_us"], 2) for x in r])
PY
step "NLP phase stamps"
timeout -k 10 120 python -u tools/diag/nlp_phases.py > "$OUT/nlp_phases.txt" 2>&1 || exit $?
step "bench (default, extras)"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
step "done"
