#!/bin/bash
# Round-6 rocprof evidence for the controller and the NLP kernels (verdict r05 #4: the NLP wait share): a kernel
# trace (--kernel-trace --stats) of the paced two-track controller (tools/diag/ctl_two_tracks.py)
# and of setupNLP.solve (tools/diag/nlp_solve.py), then PMC passes on both programs, each counter
# group its own run, summarised per kernel (ctl_kernel / nlp_kernel).
# usage (gpurun): bash tools/gpu_r05_prof.sh gpurun_out/<tag>
set -o pipefail
OUT=${1:?out dir}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HIP_FORCE_DEV_KERNARG=1 TMPDIR=/tmp
mkdir -p "$OUT" "$OUT/pmc_ctl" "$OUT/pmc_nlp"
echo "[$(date +%T)] kernel trace: the default bench line's plan launches"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_bench" -o run -- \
  python3 bench.py --no-extra --no-cpu-baseline --no-call-latency > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
echo "[$(date +%T)] kernel trace: controller"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ctl" -o run -- \
  python3 tools/diag/ctl_two_tracks.py 10000 300 > "$OUT/trace_ctl.log" 2>&1 || exit $?
echo "[$(date +%T)] kernel trace: NLP"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_nlp" -o run -- \
  python3 tools/diag/nlp_solve.py 200 > "$OUT/trace_nlp.log" 2>&1 || exit $?
i=0
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "[$(date +%T)] PMC pass $i: $group"
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc_ctl/p$i" -o run -- \
    python3 tools/diag/ctl_two_tracks.py 10000 120 > "$OUT/pmc_ctl/p$i.log" 2>&1 || { echo "ctl pass $i failed"; tail -5 "$OUT/pmc_ctl/p$i.log"; exit 1; }
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc_nlp/p$i" -o run -- \
    python3 tools/diag/nlp_solve.py 60 > "$OUT/pmc_nlp/p$i.log" 2>&1 || { echo "nlp pass $i failed"; tail -5 "$OUT/pmc_nlp/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT/pmc_ctl" ctl_kernel > "$OUT/pmc_ctl/summary.txt" 2>&1
python3 tools/pmc_summary.py "$OUT/pmc_nlp" nlp_kernel > "$OUT/pmc_nlp/summary.txt" 2>&1
cat "$OUT/pmc_ctl/summary.txt" "$OUT/pmc_nlp/summary.txt"
echo "[$(date +%T)] done"
