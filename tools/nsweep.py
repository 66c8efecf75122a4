#!/usr/bin/env python3
"""N-sweep of the tick time, mirroring the reference's computation-time study
(llampc/mpc/plot_comp_time.py:71-83: N_MODELS in [10 ... 20000], H = 20, Ts = 0.02).

For every N: the device tick on resident inputs (llampc_plan_device, ms/tick over `--steps`
ticks after warm-up), the synchronous host-pointer tick (llampc_plan incl. H2D/D2H; p50/p99),
and — for N <= --cpu-max — the CPU oracle plan (the reference's NumPy functions composed,
one core).  One JSON line per N on stdout.  Usage:
    python tools/nsweep.py [--steps 200] [--C 1] [--H 20] [--track ETHZ] > profiles/nsweep.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]

import bench  # noqa: E402  (make_ticks, the tick inputs of the bench scenario)

N_LIST = [10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 7000, 10000, 13000, 17000, 20000]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--H", type=int, default=20)
    ap.add_argument("--C", type=int, default=1)
    ap.add_argument("--W", type=int, default=10)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--track", default="ETHZ", choices=["ETHZ", "ETHZMobil"])
    ap.add_argument("--cpu-max", type=int, default=2000, help="largest N timed on the CPU oracle")
    ap.add_argument("--n", type=int, nargs="*", default=N_LIST)
    args = ap.parse_args()
    import torch
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank
    from oracle import llampc_oracle as O

    targs = argparse.Namespace(track=args.track, H=args.H, C=args.C)
    ticks = bench.make_ticks(targs, 16)
    dev = torch.device("cuda", 0)
    packs = torch.from_numpy(ticks).to(dev)
    torch.cuda.synchronize()
    H, C = args.H, args.C
    for N in args.n:
        bank = generate_bank(N, seed=0)
        sb = ShardedBank(bank, 0, 1, 0, W=args.W)
        pins = [sb.make_plan_in(packs[i], C, H, K=min(args.K, N)) for i in range(len(ticks))]
        s = sb.stream
        for i in range(args.warmup):
            sb.launch(pins[i % len(pins)], s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            sb.launch(pins[i % len(pins)], s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        pk = ticks[0]
        xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
        U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
        lat = []
        for i in range(args.steps + args.warmup):
            t1 = time.perf_counter()
            sb.bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=min(args.K, N))
            lat.append(time.perf_counter() - t1)
        lat = np.array(lat[args.warmup:]) * 1e6
        line = {"N": N, "H": H, "C": C, "track": args.track, "device_ms_per_tick": ms,
                "rollout_steps_per_s": (N * C * H + N) / (ms / 1e3),
                "sync_latency_us": {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99))}}
        if N <= args.cpu_max:
            p = O.orca_params()
            shared = {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
            win = O.LookbackWindow(N, args.W, min(args.K, N))
            Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
            reps, t2 = 0, time.perf_counter()
            while reps < 3 or (time.perf_counter() - t2 < 1.0 and reps < 200):
                O.plan_cpu(shared, bank, win, pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], 0.02, Q, R, P)
                reps += 1
            line["cpu_oracle_ms_per_tick"] = (time.perf_counter() - t2) / reps * 1e3
        print(json.dumps(line), flush=True)
        sb.close()


if __name__ == "__main__":
    main()
