"""Diagnostic (stamps build): where the controller tick's time goes.  Runs LLAMPC (device
mode, ETHZ, H = 40, C = 64, K = 10, W = 10) on an N-model bank and prints, per tick, the
phase boundaries of every block of the launch relative to the first block's entry (µs,
s_memrealtime at 100 MHz): look-ahead blocks — staged (tables + candidates), walk done
(thread 0), walk barrier, selection known, rolled out, published; the look-back ticket winner
— scored, lb_final done, slots polled, record stores issued (thread 0), record
written (after the system fence) — plus the host's own split of the
tick (tick_begin, the wait, the result).  Paced at 1 ms and back to back.
"prelaunch": armed ticks (llampc_ctl_set_prelaunch), times from the first block's doorbell.
usage: python tools/diag/ctl_phases.py [N] [ticks] [prelaunch]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LLAMPC_HIP_LIB", os.path.join(REPO, "lla-mpc_amd/llampc/_lib/libllampc_hip_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat  # noqa: E402
from llampc.models import Dynamic  # noqa: E402
from llampc.mpc import LLAMPC, ModelBank, generate_bank  # noqa: E402
from llampc.params import ORCA  # noqa: E402
from llampc.tracks import ETHZ  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 6
PRE = "prelaunch" in sys.argv[3:]
lib = nat.load()
lib.llampc_debug_ctl_stamps.argtypes = [ctypes.c_void_p]
tr = ETHZ('optimal', True)
b = ModelBank(generate_bank(N, seed=0), W=10, device=0)
ctl = LLAMPC(b, tr, H=40, C=64, K=10, mode="device", prelaunch=PRE)
plant = Dynamic(**ORCA(), device=0)
x = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))["states"][:, 0].copy()
nb_lb = None
NAMES = {17: "walk-loop", 18: "walk-loop-end", 16: "door", 0: "entry", 14: "bracket", 15: "tables", 1: "staged", 10: "walked", 2: "walk-bar", 3: "selected", 4: "rolled", 5: "published"}


def step(paced_until=None):
    global x
    if paced_until is not None:
        while time.perf_counter() < paced_until:
            pass
    t0 = time.perf_counter()
    ctl.tick_begin(x)
    t1 = time.perf_counter()
    o = ctl._ctl.wait()
    t2 = time.perf_counter()
    r = ctl._finish_device(o, ctl._pending_x)
    t3 = time.perf_counter()
    xn, _ = plant.sim_continuous(x, np.array(r.u0).reshape(2, 1), [0, 0.02])
    x = xn[:, -1]
    return (t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6


for i in range(40):
    step()
buf = (ctypes.c_ulonglong * (64 * 24))()
for mode in ("paced", "back-to-back"):
    nxt = time.perf_counter()
    for i in range(T):
        nxt += 1e-3
        hb, hw, hr = step(nxt if mode == "paced" else None)
        lib.llampc_debug_ctl_stamps(buf)
        Z = np.frombuffer(buf, dtype=np.uint64).reshape(64, 24).astype(np.int64)
        live = Z[:, 0] > 0
        base = Z[live, 16].min() if PRE else Z[live, 0].min()
        us = lambda v: (v - base) / 100.0  # noqa: E731
        win = int(np.argmax(np.where(live, Z[:, 9], 0)))      # the completing block
        la = [k for k in range(64) if live[k] and Z[k, 5] >= base and Z[k, 1] >= base]
        parts = [f"{mode} tick: host begin {hb:.1f} wait {hw:.1f} result {hr:.1f} us |"]
        parts.append(f"lb(block {win}): scored {us(Z[win, 6]):.1f} lb_final {us(Z[win, 7]):.1f} "
                     f"polled {us(Z[win, 8]):.1f} seq {us(Z[win, 12]):.1f} words {us(Z[win, 13]):.1f} "
                     f"stored {us(Z[win, 11]):.1f} record {us(Z[win, 9]):.1f} |")
        # spec blocks (armed ticks, CtlLaunch.n_spec): 19 doorbell seen, 20 rolled out, 21 published
        sp = [k for k in range(64) if Z[k, 21] >= base and Z[k, 19] >= base]
        if PRE and sp:
            for slot, nm in ((19, "spec-door"), (20, "spec-rolled"), (21, "spec-published")):
                v = np.array([us(Z[k, slot]) for k in sp])
                parts.append(f"{nm} {v.min():.1f}/{v.max():.1f}")
            parts.append("|")
        for slot in ((16, 0, 14, 15, 1, 17, 18, 10, 2, 3, 4, 5) if PRE else (0, 14, 15, 1, 17, 18, 10, 2, 3, 4, 5)):
            v = np.array([us(Z[k, slot]) for k in la])
            if v.size:                   # armed ticks whose selection the spec blocks covered
                parts.append(f"{NAMES[slot]} {v.min():.1f}/{v.max():.1f}")   # roll nothing more
        print(" ".join(parts), flush=True)
ctl.close()
b.close()
