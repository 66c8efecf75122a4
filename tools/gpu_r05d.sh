#!/bin/bash
# Round 5: the conditioning-aware parity tests, the accuracy diagnostic over every shape, then
# tools/gpu_r05b.sh (the driver's command, stamps timelines, controller / NLP traces and PMC).
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT"
echo "[$(date +%T)] conditioning-aware tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  -k "config_scenario or ctl_closed_loop or near_ties or lean_cores" > "$OUT/gputest_cond.log" 2>&1 || { tail -30 "$OUT/gputest_cond.log"; exit 1; }
tail -3 "$OUT/gputest_cond.log"
echo "[$(date +%T)] accuracy headroom (every shape)"
timeout -k 10 600 python -u tools/diag/accuracy_headroom.py "$OUT/accuracy.json" > "$OUT/accuracy.log" 2>&1 || { tail -5 "$OUT/accuracy.log"; exit 1; }
bash tools/gpu_r05b.sh "$OUT" || exit $?
echo "[$(date +%T)] all done"
