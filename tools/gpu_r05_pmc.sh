#!/bin/bash
# Round 5: the plan kernel's PMC passes on the shipped library (C = 1 and C = 64), their
# corrected HBM traffic into profiles/pmc_lookahead.json (tools/pmc.sh, tools/pmc_traffic.py).
# usage (gpurun): bash tools/gpu_r05_pmc.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$OUT"
PMC_ROUND="r05 (8-term lean cores, shipped library)" PMC_OUT=$OUT/c1 PMC_KEY=ETHZ_N10000_H20_C1 bash tools/pmc.sh --steps 40 --warmup 5 > "$OUT/c1.txt" 2>&1 || { echo "c1 failed"; tail -5 "$OUT/c1.txt"; exit 1; }
PMC_ROUND="r05 (8-term lean cores, shipped library)" PMC_OUT=$OUT/c64 PMC_KEY=ETHZ_N10000_H20_C64 bash tools/pmc.sh --steps 10 --warmup 2 --C 64 > "$OUT/c64.txt" 2>&1 || { echo "c64 failed"; tail -5 "$OUT/c64.txt"; exit 1; }
cp profiles/pmc_lookahead.json "$OUT/pmc_lookahead.json"
tail -20 "$OUT/c1.txt"
echo "[$(date +%T)] done"
