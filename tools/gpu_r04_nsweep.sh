#!/bin/bash
# N-sweep of the tick (tools/nsweep.py) with the round's last library, CPU oracle up to N=2000.
# usage: tools/gpu_r04_nsweep.sh <tag>
set -o pipefail
T=${1:?tag}
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
timeout -k 10 600 python -u tools/nsweep.py --steps 200 --cpu-max 2000 > $OUT/nsweep.jsonl 2> $OUT/nsweep.err || { tail -10 $OUT/nsweep.err; exit 1; }
cut -c1-220 $OUT/nsweep.jsonl
