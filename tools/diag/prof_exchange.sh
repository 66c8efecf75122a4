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
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    return "plan" if "plan_kernel" in n else "merge" if "merge_kernel" in n else ("rccl" if "ncclDevKernel" in n or "nccl" in n.lower() else n[:40])
seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
dur, gap = {}, {}
for i, (n, a, b) in enumerate(seq):
    dur.setdefault(n, []).append((b - a) / 1000)
    if i:
        p = seq[i - 1]
        gap.setdefault(f"{p[0]}->{n}", []).append((a - p[2]) / 1000)
med = lambda v: sorted(v)[len(v) // 2]
for n, v in dur.items():
    print(f"{tag} {n}: n={len(v)} median {med(v):.2f} us")
for n, v in gap.items():
    if len(v) > 20:
        print(f"{tag} gap {n}: n={len(v)} median {med(v):.2f} us")
PY
