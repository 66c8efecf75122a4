#!/bin/bash
# Round 5: armed controller ticks (llampc_ctl_set_prelaunch) — the controller GPU tests, the
# stamps phases launched vs armed, then the paced two-track step launched vs armed, alternating,
# with the device RK6 plant.
# usage (gpurun): bash tools/gpu_r05_pre.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py tests/test_sharded_ctl_gpu.py -x -v --timeout 120 --timeout-method thread > "$OUT/ctltest.log" 2>&1 || { echo "ctl tests failed"; tail -40 "$OUT/ctltest.log"; exit 1; }
tail -3 "$OUT/ctltest.log"
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 4 prelaunch > "$OUT/phases_armed.txt" 2>&1 || { echo "phases armed failed"; tail -5 "$OUT/phases_armed.txt"; exit 1; }
cat "$OUT/phases_armed.txt"
for rep in 1 2 3; do
  for mode in plant "plant prelaunch"; do
    timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 600 $mode > "$OUT/two.$rep.${mode// /_}.txt" 2>&1 || { echo "two-track $mode failed"; tail -5 "$OUT/two.$rep.${mode// /_}.txt"; exit 1; }
    tail -1 "$OUT/two.$rep.${mode// /_}.txt"
  done
done
