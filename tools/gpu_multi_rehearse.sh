#!/bin/bash
# The N > 1 bench flow on a one-GPU box, with the extras (C=64 ticks on every rank): 2 ranks on
# one device over a gloo group (peer transport: IPC mailboxes within the device), and 1 rank
# with the exchange forced on an nccl group.  && stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/multi
O=gpurun_out/multi
LLAMPC_DIST_BACKEND=gloo LLAMPC_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29583 bench.py --gpus 2 --steps 500 --warmup 20 \
  --no-cpu-baseline > $O/rehearse2.json 2> $O/rehearse2.err && \
LLAMPC_FORCE_EXCHANGE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29584 bench.py --gpus 1 --steps 1000 --warmup 20 --no-cpu-baseline \
  > $O/force1.json 2> $O/force1.err
rc=$?
for f in $O/rehearse2 $O/force1; do
  python -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step']*1e3,2),'us/tick', d['exchange'], d['result_check'], 'C64', d.get('C64',{}).get('ms_per_step'))" || tail -5 $f.err
done
exit $rc
