#!/bin/bash
# Round 5: lb_final's wave-register ranking — all GPU tests, the C = 1 timeline (lb_final's
# phases), the armed controller phases and the paced two-track step (armed, spec).
# usage (gpurun): bash tools/gpu_r05_lbf2.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/gputest.log"; exit 1; }
tail -2 "$OUT/gputest.log"
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_c1.txt" 2>&1 || { echo "timeline failed"; tail -5 "$OUT/timeline_c1.txt"; exit 1; }
grep -E "^lb_final|^final_select" "$OUT/timeline_c1.txt"
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 4 prelaunch > "$OUT/phases_armed.txt" 2>&1 || { echo "phases failed"; tail -5 "$OUT/phases_armed.txt"; exit 1; }
cut -c1-200 "$OUT/phases_armed.txt" | tail -4
for rep in 1 2; do
  timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 600 plant prelaunch > "$OUT/two.$rep.txt" 2>&1 || { echo "two-track failed"; tail -5 "$OUT/two.$rep.txt"; exit 1; }
  tail -1 "$OUT/two.$rep.txt"
done
