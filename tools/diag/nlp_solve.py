"""Diagnostic: setupNLP.solve back to back on DYN-slice states (bench.py solve_latency's
cases) for a kernel trace of the CEM rounds.  usage: python tools/diag/nlp_solve.py [solves]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc.models import Dynamic  # noqa: E402
from llampc.mpc.nmpc import setupNLP  # noqa: E402
from llampc.mpc.planner import ConstantSpeed  # noqa: E402
from llampc.params import ORCA  # noqa: E402
from llampc.tracks import ETHZ  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
H = 20
d = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))
s, u = d["states"], d["inputs"]
tr = ETHZ('optimal', True)
p = ORCA(control="pwm")
nlp = setupNLP(H, 0.02, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, Dynamic(**p, device=0), tr, device=0)
cases, projidx = [], 0
for t in range(10, 50):
    xref, projidx, _ = ConstantSpeed(s[:2, t], s[3, t], tr, H, 0.02, projidx)
    cases.append((s[:, t].copy(), xref, u[:, t - 1].copy()))
lat = []
for i in range(n):
    x0, xref, up = cases[i % len(cases)]
    t0 = time.perf_counter()
    nlp.solve(x0, xref, up)
    lat.append(time.perf_counter() - t0)
nlp.close()
lat = np.array(lat[10:]) * 1e6
print(f"solve us p50 {np.median(lat):.1f} p99 {np.percentile(lat, 99):.1f} min {lat.min():.1f}")
