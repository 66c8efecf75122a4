#!/bin/bash
# Diagnostic: rocprofv3 kernel stats of the N>1 tick path (plan + all-gather + device merge)
# on ONE GPU via a forced exchange on a 1-rank RCCL group.  usage: prof_exchange.sh TAG [LIB]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1
[ -n "$2" ] && export LLAMPC_HIP_LIB=$PWD/lla-mpc_amd/llampc/_lib/$2
LLAMPC_FORCE_EXCHANGE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profx_$tag -o run -- \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-timing > gpurun_out/profx_$tag.log 2>&1 || exit 1
python3 - "$tag" <<'PY'
import csv, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/profx_{tag}/run_kernel_trace.csv")))
for name in ("plan_kernel", "merge_kernel"):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if name in r["Kernel_Name"])
    if d:
        print(f"{tag} {name}: n={len(d)} min {d[0]:.2f} median {d[len(d)//2]:.2f} p90 {d[int(len(d)*0.9)]:.2f} us")
PY
