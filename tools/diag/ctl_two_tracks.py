"""Diagnostic: the bench's two-track controller step (ETHZ + ETHZMobil, H = 40, C = 64, N models
each, tick_begin on both then tick_end) for a kernel trace: do the two controllers' launches
overlap on the GPU?  Prints the host split per step; run under rocprofv3 --kernel-trace and
read the trace with tools/diag/trace_overlap.py.  "prelaunch": armed ticks (llampc_ctl_set_prelaunch).
usage: python tools/diag/ctl_two_tracks.py [N] [ticks] [timing] [plant] [prelaunch]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc.mpc import LLAMPC, ModelBank, generate_bank  # noqa: E402
from llampc.tracks import ETHZ, ETHZMobil  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
TIMING = "timing" in sys.argv[3:]
PLANT = "plant" in sys.argv[3:]
PRE = "prelaunch" in sys.argv[3:]
EXTRA = int(next((a[8:] for a in sys.argv[3:] if a.startswith("streams=")), "0"))
import torch  # noqa: E402
_extra = [torch.cuda.Stream(device=0) for _ in range(EXTRA)]   # other streams created first
from llampc import _native as nat  # noqa: E402
from llampc.models import Dynamic  # noqa: E402
from llampc.params import ORCA  # noqa: E402
plant = Dynamic(**ORCA(), device=0)
setups = []
for seed, tr in ((0, ETHZ('optimal', True)), (1, ETHZMobil('optimal', True))):
    b = ModelBank(generate_bank(N, seed=seed), W=10, device=0)
    b.set_concurrency(2)            # the two controllers' banks: a hardware queue each
    ctl = LLAMPC(b, tr, H=40, C=64, K=10, mode="device", prelaunch=PRE)
    if tr.name == "ETHZ":
        x = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))["states"][:, 0].copy()
    else:
        x = np.array([tr.x_init, tr.y_init, tr.psi_init, 1.0, 0.0, 0.0])
    setups.append([b, ctl, x])
    if TIMING:
        nat.check(nat.load().llampc_bank_timing(b.handle, 1, T + 8))
lat = []
nxt = time.perf_counter()
for i in range(T):
    nxt += 1e-3
    while time.perf_counter() < nxt:
        pass
    t0 = time.perf_counter()
    for s in setups:
        s[1].tick_begin(s[2])
    res = [s[1].tick_end() for s in setups]
    lat.append(time.perf_counter() - t0)
    for s, r in zip(setups, res):
        if PLANT:
            xn, _ = plant.sim_continuous(s[2], r.u_seq[:, 0].reshape(2, 1), [0, 0.02])
            s[2] = xn[:, -1]
lat = np.array(lat[20:]) * 1e6
print(f"timing={TIMING} plant={PLANT} prelaunch={PRE} extra streams={EXTRA}: two-track step us p50 {np.median(lat):.1f} p99 {np.percentile(lat, 99):.1f}")
for s in setups:
    s[1].close()
    s[0].close()
