"""Diagnostic: device time per tick of the plan launch's parts (look-back only, look-ahead
only, both; polled vs ticket completion) at a few (N, H), resident inputs, events around
200 back-to-back launches.  usage: python tools/diag/tick_parts.py [N ...]"""
import os
import sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat
from llampc.mpc import generate_bank
from llampc.mpc.sharded import ShardedBank

d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
dev = torch.device("cuda", 0)
Ns = [int(a) for a in sys.argv[1:]] or [10, 10000]


def run(sb, pin, reps=200):
    st = sb.stream
    for _ in range(20):
        sb.launch(pin, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
        for _ in range(reps):
            sb.launch(pin, st)
        e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for N in Ns:
    for H in (1, 20):
        sb = ShardedBank(generate_bank(N, 0), 0, 1, 0, W=10)
        U = np.tile(u[:, 1], (H, 1))[None]
        pack = np.concatenate([s[:, 0], u[:, 0], s[:, 1], u[:, 0], s[:2, :H + 1].ravel(), U.ravel()])
        pk = torch.from_numpy(pack).to(dev)
        res = {}
        for name, lb, la, env in (("lb+la poll", 1, 1, {}), ("lb+la ticket", 1, 1, {"LLAMPC_NO_POLL": "1"}),
                                  ("la only", 0, 1, {}), ("lb only", 1, 0, {})):
            os.environ.update(env)
            pin = sb.make_plan_in(pk, 1, H, do_lookback=bool(lb))
            pin.do_lookahead = la
            res[name] = run(sb, pin)
            for k in env:
                del os.environ[k]
        print(f"N={N} H={H}: " + ", ".join(f"{k} {v:.2f}" for k, v in res.items()) + " us/tick", flush=True)
        sb.close()
