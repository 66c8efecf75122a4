#!/bin/bash
# Round-4 check of the shipped library: GPU tests + smoke + default bench + 2-rank rehearsal +
# rocprofv3 kernel trace of the bench (tools/gpu_check.sh), the driver's K = 20 / W = 5 bench,
# config 3, PMC passes at C = 1 and C = 64, and the stamps diagnostics (C = 1 timeline,
# controller and NLP phases; needs `make -C lla-mpc_amd/csrc stamps` first).
# usage (gpurun): bash tools/gpu_final_r04.sh gpurun_out/<tag> [quick]
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1
mkdir -p "$OUT"
if [ "$2" != "pmc" ]; then
  bash tools/gpu_check.sh "$OUT" || exit $?
  echo "[$(date +%T)] driver's command"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_k20.json" 2> "$OUT/bench_k20.err" || exit $?
  echo "[$(date +%T)] config 3 bench"
  timeout -k 10 300 python -u bench.py --track ETHZMobil --H 40 --no-extra --no-cpu-baseline > "$OUT/bench_config3.json" 2> "$OUT/bench_config3.err" || exit $?
fi
echo "[$(date +%T)] PMC C=1"
PMC_OUT=$OUT/pmc_c1 bash tools/pmc.sh --steps 40 --warmup 5 > "$OUT/pmc_c1.log" 2>&1 || exit $?
echo "[$(date +%T)] PMC C=64"
PMC_OUT=$OUT/pmc_c64 bash tools/pmc.sh --C 64 --steps 10 --warmup 2 > "$OUT/pmc_c64.log" 2>&1 || exit $?
if [ "$2" != "pmc" ]; then
  echo "[$(date +%T)] stamps: C=1 timeline, controller and NLP phases"
  timeout -k 10 120 python -u tools/diag_timeline.py 10000 > "$OUT/timeline_c1.txt" 2>&1 || exit $?
  timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > "$OUT/ctl_phases.txt" 2>&1 || exit $?
  timeout -k 10 120 python -u tools/diag/nlp_phases.py > "$OUT/nlp_phases.txt" 2>&1 || exit $?
fi
echo "[$(date +%T)] done"
