#!/bin/bash
# Round-3 (session 2) check of the shipped library: tests, smoke, headline bench, 2-rank
# self-spawned bench, rocprofv3 kernel trace, config-3 bench, PMC passes at C=1 and C=64, and
# the stamps diagnostics (C=1 timeline, work-queue units at C=64).
# usage (gpurun): bash tools/gpu_final_r03s2.sh gpurun_out/<tag>
# (the stamps diagnostics need libllampc_hip_stamps.so: `make -C lla-mpc_amd/csrc stamps` first)
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
echo "[$(date +%T)] stamps: C=1 timeline, C=64 work-queue units"
timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_c1.txt" 2>&1 || exit $?
timeout -k 10 120 python -u tools/diag/wq_units.py 10000 64 > "$OUT/wq_units_c64.txt" 2>&1 || exit $?
echo "[$(date +%T)] done"
