#!/bin/bash
# Round 5: the speculative look-ahead of armed controller ticks — the controller GPU tests, the
# stamps phases (armed), then the paced two-track step launched / armed without spec / armed
# with spec, alternating, with the device RK6 plant.
# usage (gpurun): bash tools/gpu_r05_spec.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_ctl_gpu.py tests/test_sharded_ctl_gpu.py -x -v --timeout 120 --timeout-method thread > "$OUT/ctltest.log" 2>&1 || { echo "ctl tests failed"; tail -40 "$OUT/ctltest.log"; exit 1; }
tail -3 "$OUT/ctltest.log"
timeout -k 10 120 python -u tools/diag/ctl_phases.py 10000 4 prelaunch > "$OUT/phases_armed.txt" 2>&1 || { echo "phases armed failed"; tail -5 "$OUT/phases_armed.txt"; exit 1; }
cat "$OUT/phases_armed.txt"
for rep in 1 2 3; do
  for mode in plant "plant prelaunch" "plant prelaunch nospec"; do
    tag=${mode// /_}
    if [[ "$mode" == *nospec ]]; then export LLAMPC_CTL_NO_SPEC=1; m="plant prelaunch"; else unset LLAMPC_CTL_NO_SPEC; m="$mode"; fi
    timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 600 $m > "$OUT/two.$rep.$tag.txt" 2>&1 || { echo "two-track $mode failed"; tail -5 "$OUT/two.$rep.$tag.txt"; exit 1; }
    echo "$mode: $(tail -1 $OUT/two.$rep.$tag.txt)"
  done
done
