#!/bin/bash
# Round 5: the controller completion's stores spread over the waves — controller GPU tests, the
# armed phases (with the spec blocks' stamps) and the paced two-track step.
# usage (gpurun): bash tools/gpu_r05_tail.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/ctltest.log" 2>&1 || { echo "ctl tests failed"; tail -30 "$OUT/ctltest.log"; exit 1; }
tail -1 "$OUT/ctltest.log"
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 4 prelaunch > "$OUT/phases_armed.txt" 2>&1 || { echo "phases failed"; tail -5 "$OUT/phases_armed.txt"; exit 1; }
tail -3 "$OUT/phases_armed.txt" | cut -c1-330
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 600 plant prelaunch > "$OUT/two.$rep.txt" 2>&1 || { echo "two-track failed"; tail -5 "$OUT/two.$rep.txt"; exit 1; }
  tail -1 "$OUT/two.$rep.txt"
done
