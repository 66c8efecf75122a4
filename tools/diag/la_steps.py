"""Diagnostic (stamps build): shader cycles of each rollout step of the C = 1 plan tick's
look-ahead blocks (thread 0, s_memtime before every step) — is the first step (cold
instruction cache: every launch starts with the code uncached) slower than the warm ones?
usage: python tools/diag/la_steps.py [N]"""
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
lib.llampc_debug_la_step.argtypes = [ctypes.c_void_p]
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N, H = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 20
b = ModelBank(generate_bank(N, 0), W=10, device=0)
xref = s[:2, :H + 1]
U = np.tile(u[:, 0], (H, 1))[None]
buf = (ctypes.c_ulonglong * (1024 * 25))()
for rep in range(3):
    for t in range(1, 30):
        b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
    lib.llampc_debug_la_step(buf)
    Z = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 25).astype(np.int64)
    rows = Z[(Z[:, 0] > 0) & (Z[:, H - 1] > 0)]
    dz = np.diff(rows[:, :H], axis=1)                 # step k = stamp k+1 - stamp k, k < H - 1
    first, rest = dz[:, 0], dz[:, 1:]
    print(f"rep {rep}: {rows.shape[0]} blocks; step 0 {int(np.median(first))} cycles (min {int(first.min())}, "
          f"max {int(first.max())}); step 1 {int(np.median(dz[:, 1]))}; steps 2..{H - 2} median "
          f"{int(np.median(rest[:, 1:]))}, max {int(rest[:, 1:].max())}", flush=True)
b.close()
