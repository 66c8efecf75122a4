#!/bin/bash
# Kernel trace of host-pointer ticks paced at 1 ms and at 100 us, and back to back.
# usage (gpurun): bash tools/gpu_paced_trace.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/$OUT"
export TMPDIR=/tmp
cd /tmp
for p in 1000 100 0; do
  echo "[$(date +%T)] period $p us"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/p$p" -o run -- \
    python3 "$R/tools/diag/paced_ticks.py" $p 400 > "$R/$OUT/p$p.txt" 2>&1 || exit $?
  cat "$R/$OUT/p$p.txt" | grep period
done
echo "[$(date +%T)] done"
