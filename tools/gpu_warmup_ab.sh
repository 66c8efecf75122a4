#!/bin/bash
# Headline bench at several warmup/step counts on one box (does a short timed region read
# slow because the clocks are still ramping?).  usage (gpurun): bash tools/gpu_warmup_ab.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in "20 200" "2000 2000" "20 200" "200 1000" "5000 200" "20 200" "2000 2000"; do
  set -- $cfg
  echo "[$(date +%T)] warmup $1 steps $2"
  timeout -k 10 120 python -u bench.py --warmup $1 --steps $2 --no-extra --no-cpu-baseline --no-call-latency \
    >> "$OUT/warm_ab.jsonl" 2>> "$OUT/warm_ab.err" || exit $?
done
echo "[$(date +%T)] done"
