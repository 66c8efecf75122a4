"""Diagnostic (stamps build): phases of the setupNLP.solve CEM round — per stamp the earliest
and latest block (µs from the first block's round start, s_memrealtime): mean / std in, samples
formed, rate-clipped, staged, rolled out, list published; then every block's completion
(round 6): wave 0's four lists in, every group in, merged, elite loads issued, elite mean, next
mean / std — for the last round of a few solves.
usage: python tools/diag/nlp_phases.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LLAMPC_HIP_LIB", os.path.join(REPO, "lla-mpc_amd/llampc/_lib/libllampc_hip_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat  # noqa: E402
from llampc.models import Dynamic  # noqa: E402
from llampc.mpc.nmpc import setupNLP  # noqa: E402
from llampc.mpc.planner import ConstantSpeed  # noqa: E402
from llampc.params import ORCA  # noqa: E402
from llampc.tracks import ETHZ  # noqa: E402

lib = nat.load()
lib.llampc_debug_nlp_stamps.argtypes = [ctypes.c_void_p]
H = 20
from llampc.tracks import dyn_slice  # noqa: E402
d = dyn_slice()
s, u = d["states"], d["inputs"]
tr = ETHZ('optimal', True)
p = ORCA(control="pwm")
nlp = setupNLP(H, 0.02, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, Dynamic(**p, device=0), tr, device=0)
buf = (ctypes.c_ulonglong * (32 * 16))()
projidx = 0
for t in range(10, 16):
    xref, projidx, _ = ConstantSpeed(s[:2, t], s[3, t], tr, H, 0.02, projidx)
    nlp.solve(s[:, t].copy(), xref, u[:, t - 1].copy())
    lib.llampc_debug_nlp_stamps(buf)
    Z = np.frombuffer(buf, dtype=np.uint64).reshape(32, 16).astype(np.int64)
    nb = nlp.samples // 64
    base = Z[:nb, 0].min()
    us = lambda v: (v - base) / 100.0  # noqa: E731
    row = [f"{k}: {us(Z[:nb, k]).min():.1f}/{us(Z[:nb, k]).max():.1f}" for k in (10, 1, 2, 15, 9, 3, 12, 11, 4, 13, 5, 6, 14, 8)]
    print(f"solve {t}: ms/formed/clipped/cand-stored/staged/rolled0/rolled/published/own4/all-in/merged/elite-issued/"
          f"mean/next-ms (min/max) "
          f"{' '.join(row)}", flush=True)
nlp.close()
