#!/bin/bash
# rocprofv3 kernel traces (csv) of the two-track controller step and of setupNLP solves.
# usage: tools/gpu_r04_ctlprof.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ctl -o run -- python3 $R/tools/diag/ctl_two_tracks.py 10000 300 plant > $OUT/ctl.log 2>&1 || { tail -20 $OUT/ctl.log; exit 1; }
grep two-track $OUT/ctl.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nlp -o run -- python3 $R/tools/diag/nlp_solve.py 100 > $OUT/nlp.log 2>&1 || { tail -20 $OUT/nlp.log; exit 1; }
tail -1 $OUT/nlp.log
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -c1-180 "$f"; done
export HIP_FORCE_DEV_KERNARG=1
cd $R && timeout -k 10 180 python -u tools/diag/ctl_phases.py 10000 4 > $OUT/ctl_phases.txt 2>&1 || { tail -5 $OUT/ctl_phases.txt; exit 1; }
cut -c1-360 $OUT/ctl_phases.txt | grep tick
