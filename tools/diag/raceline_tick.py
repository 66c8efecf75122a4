"""Diagnostic: host-pointer tick latency with the shared xref vs the device raceline lookup
(xref_mode RACELINE, per-model ConstantSpeed with mu_n) at N models, H, C = 1 (p50 of 300
ticks after 30 warm-up; look-back + look-ahead).  usage: raceline_tick.py [N] [H]"""
import os
import sys
import time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc.mpc import ModelBank, generate_bank
from llampc.mpc.planner import ConstantSpeed, raceline_start
from llampc.tracks import ETHZ

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
H = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tr = ETHZ('optimal', True)
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
x0 = s[:, 30]
U = np.tile(u[:, 30], (H, 1))[None]
s0, _ = raceline_start(x0, tr, 0)
xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, H, 0.02, 0)
with ModelBank(generate_bank(N, 0), W=10, device=0) as b:
    b.set_raceline(tr)
    for mode in ("shared", "raceline", "shared", "raceline"):
        kw = dict(raceline_start=(s0, float(x0[3]), 0.9)) if mode == "raceline" else {}
        lat = []
        for i in range(330):
            t0 = time.perf_counter()
            b.plan_raw(s[:, 29], u[:, 29], x0, U, xref, u[:, 29], K=10, **kw)
            lat.append(time.perf_counter() - t0)
        print(f"{mode:9s} N={N} H={H}: p50 {np.percentile(np.array(lat[30:]) * 1e6, 50):.1f} us", flush=True)
