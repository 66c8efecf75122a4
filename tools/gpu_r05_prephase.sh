#!/bin/bash
# Round 5: controller phases (stamps build) launched vs armed (llampc_ctl_set_prelaunch).
# usage (gpurun): bash tools/gpu_r05_prephase.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 6 > "$OUT/phases_launched.txt" 2>&1 || { echo "phases failed"; tail -5 "$OUT/phases_launched.txt"; exit 1; }
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 6 prelaunch > "$OUT/phases_armed.txt" 2>&1 || { echo "phases armed failed"; tail -5 "$OUT/phases_armed.txt"; exit 1; }
cat "$OUT/phases_launched.txt" "$OUT/phases_armed.txt"
