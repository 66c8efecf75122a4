"""Diagnostic (verdict r05 #5): what armed controller launches cost the other work on the chip.

Two controllers (ETHZ + ETHZMobil, N models each, H = 40, C = 64; the bench's config-5 loop)
tick paced at 1 kHz.  After each step — while armed launches (if any) sit on their CUs waiting for
the next doorbell — a co-tenant workload runs on its own torch stream and is timed by HIP events:
  matmul  torch fp64 GEMM 2048^3 (one library kernel over the whole chip)
  plant   the device RK6 plant (Dynamic.sim_continuous: the closed loop's own co-tenant)
  plan    a plan() tick of a third bank (N = 10^4, C = 64: every CU for ~380 us)
Modes: disarmed (launched ticks), armed without the speculative blocks (LLAMPC_CTL_NO_SPEC=1 is
read at controller create), armed (the default: 32 spec blocks per controller).  Prints one JSON
line per mode: the co-tenant's p50 / p99 and the controllers' step p50 / p99.
usage: python tools/diag/cotenant.py [N] [steps] [out.json]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 300
OUT = sys.argv[3] if len(sys.argv) > 3 else None

import torch  # noqa: E402
from llampc.models import Dynamic  # noqa: E402
from llampc.mpc import LLAMPC, ModelBank, generate_bank  # noqa: E402
from llampc.mpc.scenarios import scenario_ticks  # noqa: E402
from llampc.params import ORCA  # noqa: E402
from llampc.tracks import ETHZ, ETHZMobil, dyn_slice  # noqa: E402

dev = torch.device("cuda", 0)
side = torch.cuda.Stream(device=dev)
A = torch.randn(2048, 2048, dtype=torch.float64, device=dev)
B = torch.randn(2048, 2048, dtype=torch.float64, device=dev)
plant = Dynamic(**ORCA(), device=0)
third = ModelBank(generate_bank(10000, seed=5), W=10, device=0)
pk = scenario_ticks("ETHZ", 20, 64, 1, device=0)[0]
H3 = 20
xref3, U3 = pk[16:16 + 2 * (H3 + 1)].reshape(2, H3 + 1), pk[16 + 2 * (H3 + 1):].reshape(64, H3, 2)
x_pl = dyn_slice()["states"][:, 0].copy()


def cotenant(kind):
    """Time one co-tenant job on its own stream (HIP events around it)."""
    if kind == "plan":                   # the library's own host-pointer call (blocking)
        t0 = time.perf_counter()
        third.plan_raw(pk[0:6], pk[6:8], pk[8:14], U3, xref3, pk[14:16], K=10)
        return (time.perf_counter() - t0) * 1e6
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(side):
        e0.record(side)
        if kind == "matmul":
            torch.matmul(A, B)
        e1.record(side)
    if kind == "plant":
        t0 = time.perf_counter()
        plant.sim_continuous(x_pl, np.array([[0.5], [0.1]]), [0, 0.02])
        return (time.perf_counter() - t0) * 1e6
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3


def run(mode):
    os.environ.pop("LLAMPC_CTL_NO_SPEC", None)
    if mode == "armed_no_spec":
        os.environ["LLAMPC_CTL_NO_SPEC"] = "1"
    setups = []
    for seed, tr in ((0, ETHZ('optimal', True)), (1, ETHZMobil('optimal', True))):
        b = ModelBank(generate_bank(N, seed=seed), W=10, device=0)
        b.set_concurrency(2)
        ctl = LLAMPC(b, tr, H=40, C=64, K=10, mode="device", prelaunch=mode != "disarmed")
        x = dyn_slice()["states"][:, 0].copy() if tr.name == "ETHZ" else \
            np.array([tr.x_init, tr.y_init, tr.psi_init, 1.0, 0.0, 0.0])
        setups.append([b, ctl, x])
    lat, co = [], {"matmul": [], "plant": [], "plan": []}
    kinds = list(co)
    try:
        nxt = time.perf_counter()
        for i in range(T):
            nxt += 1e-3
            while time.perf_counter() < nxt:
                pass
            t0 = time.perf_counter()
            for s in setups:
                s[1].tick_begin(s[2])
            res = [s[1].tick_end() for s in setups]
            lat.append((time.perf_counter() - t0) * 1e6)
            co[kinds[i % 3]].append(cotenant(kinds[i % 3]))    # while the next launches are armed
            for s, r in zip(setups, res):
                xn, _ = plant.sim_continuous(s[2], r.u_seq[:, 0].reshape(2, 1), [0, 0.02])
                s[2] = xn[:, -1]
    finally:
        for s in setups:
            s[1].close()
            s[0].close()
    q = lambda a: {"p50": float(np.percentile(a[10:], 50)), "p99": float(np.percentile(a[10:], 99))}  # noqa: E731
    return {"mode": mode, "N": N, "steps": T, "controller_step_us": q(lat),
            **{f"{k}_us": q(v) for k, v in co.items()}}


for _ in range(3):                        # warm the clocks and the code objects
    cotenant("matmul")
    cotenant("plan")
res = [run(m) for m in ("disarmed", "armed_no_spec", "armed", "disarmed")]
for r in res:
    print(json.dumps(r), flush=True)
if OUT:
    json.dump(res, open(OUT, "w"), indent=1)
