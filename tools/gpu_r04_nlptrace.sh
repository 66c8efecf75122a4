#!/bin/bash
# Kernel trace of back-to-back setupNLP solves (the H2D blit, the one-launch rounds, the gaps).
# usage: tools/gpu_r04_nlptrace.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $R/tools/diag/nlp_solve.py 60 > $OUT/solve.log 2>&1 || { tail -20 $OUT/solve.log; exit 1; }
tail -2 $OUT/solve.log
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
