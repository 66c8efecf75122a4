#!/bin/bash
# SQ issue/wait counters (two rocprofv3 --pmc passes) of the bench's plan kernel for each
# library named.  usage: PMC_OUT=dir tools/pmc_sq.sh "libA.so libB.so" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUTD=${PMC_OUT:-gpurun_out/pmc_sq}; mkdir -p $OUTD
LIBS=$1; shift
ARGS="${@:---C 64 --steps 10 --warmup 2}"
for lib in $LIBS; do
  i=0
  for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
               "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    LLAMPC_HIP_LIB=$PWD/lla-mpc_amd/llampc/_lib/$lib timeout -k 10 120 rocprofv3 --pmc $group --output-format csv \
      -d $OUTD/$lib.p$i -o run -- python3 bench.py $ARGS --no-cpu-baseline --no-extra --no-timing --no-call-latency \
      > $OUTD/$lib.p$i.log 2>&1 || { echo "pass $i failed: $lib $group"; tail -5 $OUTD/$lib.p$i.log; exit 1; }
  done
  mkdir -p $OUTD/$lib; cp -r $OUTD/$lib.p1 $OUTD/$lib/p1; cp -r $OUTD/$lib.p2 $OUTD/$lib/p2
  echo "== $lib"; python3 tools/pmc_summary.py $OUTD/$lib 2>&1 | grep -A14 "plan_kernel" | head -16
done
