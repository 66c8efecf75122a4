#!/bin/bash
# Round-5 GPU check: tests + smoke + default bench + 2-rank rehearsal + bench kernel trace
# (tools/gpu_check.sh), the driver's command (--steps 20 --warmup 5), then the controller / NLP
# kernel traces and PMC passes (tools/gpu_r05_prof.sh).
# usage (gpurun): bash tools/gpu_r05.sh gpurun_out/<tag> [noprof] [pytest -k expr]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1
mkdir -p "$OUT"
bash tools/gpu_check.sh "$OUT" "$3" || exit $?
echo "[$(date +%T)] driver's command"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || exit $?
echo "[$(date +%T)] accuracy headroom"
timeout -k 10 300 python -u tools/diag/accuracy_headroom.py "$OUT/accuracy.json" > "$OUT/accuracy.log" 2>&1 || exit $?
if [ "$2" != "noprof" ]; then
  bash tools/gpu_r05_prof.sh "$OUT/prof5" || exit $?
fi
echo "[$(date +%T)] all done"
