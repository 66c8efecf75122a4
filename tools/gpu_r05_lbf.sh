#!/bin/bash
# Round 5 diagnostic: lb_final cold vs warm (stamps build with -DLLAMPC_LBF_TWICE runs it twice,
# the stamps keep the second run's phases) on the C = 1 tick, three processes each.
# usage (gpurun): bash tools/gpu_r05_lbf.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
L=$PWD/lla-mpc_amd/llampc/_lib
for rep in 1 2 3; do
  for s in libllampc_hip_stamps lbf_twice; do
    LLAMPC_HIP_LIB=$L/$s.so timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_$s.$rep.txt" 2>&1 || { echo "timeline $s failed"; tail -5 "$OUT/timeline_$s.$rep.txt"; exit 1; }
    echo "$s rep $rep: $(grep -E '^lb_final' $OUT/timeline_$s.$rep.txt)"
  done
done
