#!/bin/bash
# Round-3 check of the shipped library: tests, smoke, headline bench, 2-rank self-spawned bench,
# rocprofv3 kernel trace, config-3 bench, PMC passes at C=1 and C=64.
# usage (gpurun): bash tools/gpu_final_r03.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_check.sh "$OUT" || exit $?
echo "[$(date +%T)] config 3 bench"
timeout -k 10 600 python -u bench.py --track ETHZMobil --H 40 --no-extra > "$OUT/bench_config3.json" 2> "$OUT/bench_config3.err" || exit $?
echo "[$(date +%T)] PMC C=1"
PMC_OUT=$OUT/pmc_c1 bash tools/pmc.sh --steps 40 --warmup 5 > "$OUT/pmc_c1.log" 2>&1 || exit $?
echo "[$(date +%T)] PMC C=64"
PMC_OUT=$OUT/pmc_c64 bash tools/pmc.sh --C 64 --steps 10 --warmup 2 > "$OUT/pmc_c64.log" 2>&1 || exit $?
echo "[$(date +%T)] done"
