"""Diagnostic (stamps build with -DLLAMPC_LB_TWICE): the look-back block's RK4 step run twice —
cycles of the first (cold code, operand loads) vs the second (warm) — on the C = 1 plan tick.
usage: LLAMPC_HIP_LIB=<lb_twice.so> python tools/diag/lb_twice.py [N]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat  # noqa: E402
from llampc.mpc import ModelBank, generate_bank  # noqa: E402

lib = nat.load()
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N, H = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 20
b = ModelBank(generate_bank(N, 0), W=10, device=0)
U = np.tile(u[:, 0], (H, 1))[None]
for t in range(1, 30):
    b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, s[:2, t:t + H + 1], u[:, t - 1])
lb = (ctypes.c_ulonglong * (8 * 8 * 2))()
lib.llampc_debug_lb_stamps.argtypes = [ctypes.c_void_p]
lib.llampc_debug_lb_stamps(lb)
B = np.frombuffer(lb, dtype=np.uint64).reshape(8, 8, 2).astype(np.int64)
for k in range(8):
    c = B[k, :, 0]
    print(f"look-back block {k}: first step {c[4] - c[0]} cycles (entry -> after step 1), second step "
          f"{c[5] - c[4]} cycles, rest of the models' loop {c[1] - c[5]}")
