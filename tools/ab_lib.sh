#!/bin/bash
# A/B of library builds x lane splits on the headline shape (one GPU call).
# usage: tools/ab_lib.sh "libA libB ..." "lpmA lpmB ..."  (libs under lla-mpc_amd/llampc/_lib/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for lib in $1; do
  for L in $2; do
    LLAMPC_HIP_LIB=$PWD/lla-mpc_amd/llampc/_lib/$lib LLAMPC_LPM=$L timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-extra --no-call-latency ${BENCH_ARGS} > gpurun_out/ab/$lib.$L.json 2>gpurun_out/ab/$lib.$L.err || { echo "FAIL $lib $L"; tail -3 gpurun_out/ab/$lib.$L.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab/$lib.$L.json').read().strip().splitlines()[-1]);print('$lib lpm=$L', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2), d['result_check'])"
  done
done
