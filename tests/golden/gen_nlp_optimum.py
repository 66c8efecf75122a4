"""Local optima of the restated NLP (test fixture generator; test infrastructure).

The reference's per-tick NLP (llampc/mpc/nmpc.py:14-203: the Euler transcription of
Dynamic.casadi, nmpc.py:58-60 / dynamic.py:195-226, the objective nmpc.py:44-111, the input
bounds and the steering-rate bound nmpc.py:102-105) is restated in oracle/llampc_oracle.py
(rollout_euler_nlp + mpc_cost).  IPOPT (casadi 3.5.1) is absent here, so this script finds a
local optimum of that restatement with scipy's SLSQP (bounds + the rate constraints as
linear inequalities, started from uprev held, ftol 1e-12) on three DYN-slice ticks with the
ConstantSpeed reference of the packaged ETHZ raceline, and writes them to nlp_optimum.npz.
tests/test_gpu_parity.py::test_setupnlp_within_5pct_of_local_optimum asserts the device
solver's fval <= 1.05 x these.  Run: python tests/golden/gen_nlp_optimum.py
"""
import os
import sys

import numpy as np
import scipy
from scipy.optimize import minimize

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from oracle import llampc_oracle as O  # noqa: E402
from llampc.mpc.planner import ConstantSpeed  # noqa: E402
from llampc.tracks import ETHZ  # noqa: E402

H, TS = 20, 0.02
TICKS = (10, 25, 60)


def main():
    p = O.orca_params()
    shared = {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
    b6 = tuple(np.array([p[k]]) for k in O.BANK_ORDER)
    d = np.load(os.path.join(HERE, "dyn_slice.npz"))
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    Q, R, P = np.eye(2), np.diag([5e-3, 1.0]), np.zeros((2, 2))
    umin, umax, r = np.array(p["min_inputs"]), np.array(p["max_inputs"]), p["max_rates"][1] * TS
    out = {k: [] for k in ("x0", "uprev", "xref", "fstar", "ustar", "tick")}
    for t in TICKS:
        x0, up = s[:, t].copy(), u[:, t - 1].copy()
        xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, H, TS, 0)
        A = np.zeros((H, 2 * H))
        for k in range(H):
            A[k, 2 * k + 1] = 1.0
            if k:
                A[k, 2 * (k - 1) + 1] = -1.0
        c = np.zeros(H)
        c[0] = up[1]
        cons = [{"type": "ineq", "fun": lambda z: r - (A @ z - c)}, {"type": "ineq", "fun": lambda z: r + (A @ z - c)}]
        J = lambda z: O.mpc_cost(O.rollout_euler_nlp(shared, b6, x0, z.reshape(1, H, 2), TS), z.reshape(1, H, 2),
                                 xref, up, Q, R, P)[0]
        res = minimize(J, np.tile(up, H), method="SLSQP", constraints=cons,
                       bounds=[(umin[i % 2], umax[i % 2]) for i in range(2 * H)], options={"maxiter": 500, "ftol": 1e-12})
        assert res.success, res.message
        for k, v in (("x0", x0), ("uprev", up), ("xref", xref), ("fstar", res.fun), ("ustar", res.x.reshape(H, 2)),
                     ("tick", t)):
            out[k].append(v)
        print(f"tick {t}: local optimum {res.fun:.6f} ({res.nit} SLSQP iterations)")
    np.savez(os.path.join(HERE, "nlp_optimum.npz"), scipy_version=np.array(scipy.__version__),
             **{k: np.array(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
