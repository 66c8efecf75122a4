#!/bin/bash
# A/B of HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/kernarg
for v in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python bench.py --steps 1000 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/kernarg/b$v.json 2> gpurun_out/kernarg/b$v.err || { echo fail $v; tail -3 gpurun_out/kernarg/b$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/kernarg/b$v.json').read().strip().splitlines()[-1]);print('HIP_FORCE_DEV_KERNARG=$v', round(d['ms_per_step']*1e3,2), 'us/tick; plan_us', round(d['kernel_us']['plan'],2), 'plan_call p50', round(d.get('plan_call_us',{}).get('p50',0),1), 'sync p50', round(d.get('sync_plan_latency_us',{}).get('p50',0),1))"
done
