"""Diagnostic: run bench.py's extras alone, in a given order, to find interactions between them
(e.g. which earlier extra slows the two-track controller step).
usage: python tools/diag/bench_extra.py config5,config3,controller"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
order = sys.argv[1].split(",") if len(sys.argv) > 1 else ["controller"]
sys.argv = [sys.argv[0]]
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
args = bench.parse()
state = {}


def headline(args):
    """main()'s headline setup: the sharded bank (world 1), its resident ticks, 50 launches"""
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank
    ticks = bench.make_ticks(args, 16)
    packs = torch.from_numpy(ticks).to(torch.device("cuda", 0))
    sb = ShardedBank(generate_bank(args.n_per_gpu, seed=0), 0, 1, 0, W=args.W)
    pins = [sb.make_plan_in(packs[i], args.C, args.H, K=args.K, current_model=0) for i in range(16)]
    for i in range(50):
        sb.launch(pins[i % 16], sb.stream)
    torch.cuda.synchronize()
    state.update(sb=sb, ticks=ticks)
    return {}


def call(args):
    return bench.plan_call_latency(args, state["sb"], state["sb"].stream, state["ticks"], 1)


def extras(args):
    r = bench.extras(args, state["sb"], state["sb"].stream, 1, 0) if hasattr(bench, "extras") else {}
    return r.get("controller_tick_us", {})


def c64(args):
    """extras()'s C=64 leg on the headline bank"""
    a2 = bench.argparse.Namespace(**vars(args))
    a2.C = 64
    t64 = bench.make_ticks(a2, 8)
    sb = state["sb"]
    p64 = torch.from_numpy(t64).to(torch.device("cuda", 0))
    torch.cuda.synchronize()
    pins = [sb.make_plan_in(p64[i], 64, args.H, K=args.K) for i in range(8)]
    for i in range(55):
        sb.launch(pins[i % 8], sb.stream)
    torch.cuda.synchronize()
    return {}


def sync(args):
    """extras()'s host-pointer plan_raw legs (back to back, then paced)"""
    pk = bench.make_ticks(args, 1)[0]
    H, C = args.H, args.C
    xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
    U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
    for i in range(1050):
        state["sb"].bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=args.K)
    return {}


def bank(args):
    """one more open bank whose stream has run a tick (another HIP stream in use)"""
    from llampc.mpc import ModelBank, generate_bank
    b = ModelBank(generate_bank(64, seed=3), W=2, device=0)
    from llampc.mpc import plan
    x = np.array([0.1, 0.1, 0.0, 1.0, 0.0, 0.0])
    plan(b, x, np.zeros(2), x, np.zeros((2, args.H + 1)), np.zeros((1, args.H, 2)), do_lookback=False)
    state.setdefault("banks", []).append(b)
    return {}


fns = {"bank": bank, "headline": headline, "call": call, "extras": extras, "c64": c64, "sync": sync, "config5": bench.concurrent_tracks, "config3": bench.config3, "controller": bench.controller_ticks,
       "solve": bench.solve_latency}
for name in order:
    r = fns[name](args)
    keep = {k: r[k] for k in ("p50", "p99", "p50_us", "p99_us", "ms_per_step", "host_split_us_p50", "kernel_us_avg")
            if k in r}
    print(name, json.dumps(keep), flush=True)
