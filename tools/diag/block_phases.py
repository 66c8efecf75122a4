"""Diagnostic (stamps build): per-block phase durations of the look-ahead blocks at a given
(N, C) — start -> staged (prologue: loads, staging, barrier), staged -> rolled out, rolled out
-> reduced — over the first 1024 blocks of one launch, and the gap between consecutive blocks
in block order (how long the dispatcher leaves a CU idle is not visible here; the lifetime
share of the prologue is).  usage: python tools/diag/block_phases.py [N] [C]"""
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
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
C = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H = 20
rng = np.random.RandomState(2)
U = np.repeat(np.tile(u[:, 0], (H, 1))[None], C, axis=0)
U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
b = ModelBank(generate_bank(N, 0), W=10, device=0)
q = lambda v: f"{np.min(v):.2f}/{np.median(v):.2f}/{np.max(v):.2f}"
for rep in range(4):
    b.plan_raw(s[:, rep], u[:, rep], s[:, rep + 1], U, s[:2, :H + 1], u[:, rep])
    ALL = (ctypes.c_ulonglong * (1024 * 4 * 2))()
    lib.llampc_debug_la_all.argtypes = [ctypes.c_void_p]
    lib.llampc_debug_la_all(ALL)
    Z = np.frombuffer(ALL, dtype=np.uint64).reshape(1024, 4, 2).astype(np.int64)
    if rep < 2:
        continue
    t = Z[:, :, 1] / 100.0
    t = t - t[:, 0].min()
    pro, roll, red = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    life = t[:, 3] - t[:, 0]
    print(f"tick {rep}: blocks 0..1023 (min/med/max us): prologue {q(pro)}, rollouts {q(roll)}, "
          f"reduce {q(red)}, lifetime {q(life)}; prologue share {pro.sum() / life.sum():.3f}, "
          f"reduce share {red.sum() / life.sum():.3f}; first-round starts {q(t[:256, 0])}")
b.close()
