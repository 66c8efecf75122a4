#!/bin/bash
# Round 5: the paced two-track step with 64 / 32 / 96 spec models (LLAMPC_CTL_SPEC_N), alternating.
# usage (gpurun): bash tools/gpu_r05_specn.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
for rep in 1 2; do
  for n in ${SPEC_NS:-64 32 96}; do
    LLAMPC_CTL_SPEC_N=$n timeout -k 10 120 python -u tools/diag/ctl_two_tracks.py 10000 1000 plant prelaunch > "$OUT/two.$n.$rep.txt" 2>&1 || { echo "two-track $n failed"; tail -5 "$OUT/two.$n.$rep.txt"; exit 1; }
    echo "spec $n: $(tail -1 $OUT/two.$n.$rep.txt)"
  done
done
