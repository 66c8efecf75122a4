"""Diagnostic (stamps build): the work-queue layout's per-unit phases at (N, C) — per wave and
unit: take -> Pacejka row loaded, row -> rolled out, rolled out -> unit done (argmin, tagged
stores), done -> next take — and each wave's idle time at the end of the launch (last unit
done -> the launch's last unit done).  usage: python tools/diag/wq_units.py [N] [C]"""
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
lib.llampc_debug_wq_units.argtypes = [ctypes.c_void_p]
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H = 20
rng = np.random.RandomState(2)
U = np.repeat(np.tile(u[:, 0], (H, 1))[None], C, axis=0)
U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
b = ModelBank(generate_bank(N, 0), W=10, device=0)
q = lambda v: f"{np.min(v):.2f}/{np.median(v):.2f}/{np.mean(v):.2f}/{np.max(v):.2f}"
for rep in range(4):
    lib.llampc_debug_wq_reset()
    b.plan_raw(s[:, rep], u[:, rep], s[:, rep + 1], U, s[:2, :H + 1], u[:, rep])
    if rep < 2:
        continue
    A = (ctypes.c_ulonglong * (256 * 8 * 16 * 4 * 2))()
    lib.llampc_debug_wq_units(A)
    Z = np.frombuffer(A, dtype=np.uint64).reshape(256, 8, 16, 4, 2).astype(np.int64)
    used = Z[:, :, :, 0, 1] > 0                       # (block, wave, unit) stamped
    nunits = used.sum(axis=2)
    w = nunits > 0
    # per-wave shader clock from its first take to its last unit done (memtime / realtime)
    first = np.where(w, Z[:, :, 0, 0, 1], 0)
    lastj = np.maximum(nunits - 1, 0)
    bi, wi = np.nonzero(w)
    f_mhz = []
    for B, W_ in zip(bi, wi):
        j = lastj[B, W_]
        dc = Z[B, W_, j, 3, 0] - Z[B, W_, 0, 0, 0]
        dr = Z[B, W_, j, 3, 1] - Z[B, W_, 0, 0, 1]
        f_mhz.append(100.0 * dc / dr if dr > 0 else np.nan)
    f_mhz = np.array(f_mhz)
    fmed = np.nanmedian(f_mhz)
    us = lambda cyc: cyc / fmed                        # shader cycles -> us (median clock)
    ph = {k: [] for k in ("row", "roll", "fin", "gap")}
    for B, W_ in zip(bi, wi):
        n = nunits[B, W_]
        for j in range(n):
            t = Z[B, W_, j, :, 0]
            ph["row"].append(us(t[1] - t[0]))
            ph["roll"].append(us(t[2] - t[1]))
            ph["fin"].append(us(t[3] - t[2]))
            if j + 1 < n:
                ph["gap"].append(us(Z[B, W_, j + 1, 0, 0] - t[3]))
    t0 = Z[:, :, 0, 0, 1][w].min()
    end = np.array([Z[B, W_, lastj[B, W_], 3, 1] for B, W_ in zip(bi, wi)])
    start = np.array([Z[B, W_, 0, 0, 1] for B, W_ in zip(bi, wi)])
    idle = (end.max() - end) / 100.0
    print(f"tick {rep}: N={N} C={C}: {len(bi)} waves stamped, units/wave {q(nunits[w])}, "
          f"clock MHz {q(f_mhz)}")
    for k, v in ph.items():
        v = np.array(v)
        print(f"  {k:5s} us min/med/mean/max {q(v)}  total per wave {v.sum() / len(bi):.1f}")
    print(f"  first take after launch's first take (us) {q((start - t0) / 100.0)}; "
          f"last unit done (us) {q((end - t0) / 100.0)}; end idle per wave (us) {q(idle)}")
b.close()
