#!/bin/bash
# Round 5, second half of the check: the driver's command, the controller / NLP kernel traces
# and PMC passes (tools/gpu_r05_prof.sh), the stamps timelines (C = 1 plan tick, controller
# phases).  usage (gpurun): bash tools/gpu_r05b.sh gpurun_out/<tag> [noprof]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1
mkdir -p "$OUT"
echo "[$(date +%T)] driver's command"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || exit $?
echo "[$(date +%T)] stamps: C=1 timeline, controller phases"
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_c1.txt" 2>&1 || exit $?
timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > "$OUT/ctl_phases.txt" 2>&1 || exit $?
if [ "$2" != "noprof" ]; then
  bash tools/gpu_r05_prof.sh "$OUT/prof5" || exit $?
fi
echo "[$(date +%T)] done"
