#!/bin/bash
# Alternating A/B of two library builds: the headline (C = 1, K = 200) and C = 64 (K = 50),
# three pairs each.  usage: tools/gpu_ab_r04.sh <tag> <libA.so> <libB.so>
set -o pipefail
T=${1:?tag}; A=$2; B=$3
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export HIP_FORCE_DEV_KERNARG=1
for rep in 1 2 3; do
  for lib in $A $B; do
    for cfg in "--C 1 --steps 200 --warmup 20" "--C 64 --steps 50 --warmup 5"; do
      tag=$(echo "$lib $cfg" | tr ' -' '__')
      LLAMPC_HIP_LIB=$R/lla-mpc_amd/llampc/_lib/$lib timeout -k 10 120 python -u bench.py $cfg --no-extra --no-cpu-baseline --no-call-latency > $OUT/$tag.$rep.json 2> $OUT/$tag.$rep.err || { echo "FAIL $lib $cfg"; tail -5 $OUT/$tag.$rep.err; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/$tag.$rep.json').read().strip().splitlines()[-1]);print('$rep $lib $cfg', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['kernel_us']['plan'],2))" | tee -a $OUT/ab.log
    done
  done
done
