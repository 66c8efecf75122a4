#!/bin/bash
# PMC passes on the plan kernel (each pass its own rocprofv3 run; counters only with
# --kernel-trace-free --pmc; no sys/runtime traces).  Usage: tools/pmc.sh [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUTD=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUTD
ARGS="${@:---steps 40 --warmup 5}"
rocprofv3 -L > $OUTD/counters_list.txt 2>&1 || true
i=0
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
             "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH" \
             "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d $OUTD/p$i -o run -- \
     python3 bench.py $ARGS --no-cpu-baseline --no-extra --no-timing --no-call-latency > $OUTD/p$i.log 2>&1 || { echo "pass $i failed: $group"; tail -5 $OUTD/p$i.log; exit 1; }
done
# calibration dispatch for the 8-B/lane FETCH/WRITE counters (tools/pmc_calib.py)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $OUTD/cal_$c -o run -- \
     python3 tools/pmc_calib.py > $OUTD/cal_$c.log 2>&1 || { echo "calibration $c failed"; tail -5 $OUTD/cal_$c.log; exit 1; }
done
python3 tools/pmc_summary.py $OUTD > $OUTD/summary.txt 2>&1; cat $OUTD/summary.txt
if [ -n "$PMC_KEY" ]; then python3 tools/pmc_traffic.py $OUTD "$PMC_KEY"; fi
