"""Diagnostic (stamps build): the spread of the look-ahead blocks' rollout times at the
headline shape — per block: start, staged, rolled out (us from the first start), rollout
shader cycles, the implied clock, and the block's XCD (blockIdx % 8, the dispatcher's
round-robin) — to tell slow CUs/XCDs (clock) from slow blocks (cycles).
usage: python tools/diag/block_spread.py [N]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LLAMPC_HIP_LIB", os.path.join(REPO, "lla-mpc_amd/llampc/_lib/libllampc_hip_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat  # noqa: E402
from llampc.mpc import ModelBank, generate_bank  # noqa: E402

lib = nat.load()
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N, H = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 20
b = ModelBank(generate_bank(N, 0), W=10, device=0)
U = np.tile(u[:, 0], (H, 1))[None]
rows = []
for rep in range(6):
    b.plan_raw(s[:, rep], u[:, rep], s[:, rep + 1], U, s[:2, :H + 1], u[:, rep])
    ALL = (ctypes.c_ulonglong * (1024 * 4 * 2))()
    lib.llampc_debug_la_all.argtypes = [ctypes.c_void_p]
    lib.llampc_debug_la_all(ALL)
    Z = np.frombuffer(ALL, dtype=np.uint64).reshape(1024, 4, 2).astype(np.int64)
    nb = (N + 63) // 64
    Z = Z[:nb]
    t0 = Z[:, 0, 1].min()
    cyc = Z[:, 2, 0] - Z[:, 1, 0]
    us = (Z[:, 2, 1] - Z[:, 1, 1]) / 100.0
    rows.append((Z, t0, cyc, us))
for rep, (Z, t0, cyc, us) in enumerate(rows[2:]):
    clk = cyc / us / 1e3
    end = (Z[:, 2, 1] - t0) / 100.0
    print(f"tick {rep}: rollout us min/med/max {us.min():.2f}/{np.median(us):.2f}/{us.max():.2f}; cycles "
          f"{cyc.min()}/{int(np.median(cyc))}/{cyc.max()}; clock GHz {clk.min():.2f}/{np.median(clk):.2f}/{clk.max():.2f}; "
          f"rolled-out end max {end.max():.2f} at block {int(end.argmax())}")
    xcd = np.arange(len(us)) % 8
    print("   per XCD (blk % 8) median rollout us:", " ".join(f"{np.median(us[xcd == x]):.2f}" for x in range(8)),
          "| clock:", " ".join(f"{np.median(clk[xcd == x]):.2f}" for x in range(8)))
    slow = np.argsort(-end)[:6]
    print("   latest blocks (blk: start, staged, rolled out us; cycles; GHz):",
          "; ".join(f"{k}: {(Z[k,0,1]-t0)/100:.2f} {(Z[k,1,1]-t0)/100:.2f} {end[k]:.2f} {cyc[k]} {clk[k]:.2f}" for k in slow))
b.close()
