import sys
sys.path[:0] = ["/root/repo", "/root/repo/lla-mpc_amd"]
import numpy as np
from llampc.mpc import ModelBank, generate_bank, plan
from llampc.mpc.planner import raceline_start
from llampc.tracks import ETHZ
mode, N, C, sig = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
tr = ETHZ('optimal', True)
H = 20
p = generate_bank(N, seed=21, sigma=sig)
d = np.load("/root/repo/tests/golden/dyn_slice.npz")
x0 = d["states"][:, 30].copy()
rng = np.random.RandomState(4)
U = np.stack([rng.uniform(0.2, 0.8, (C, H)), rng.uniform(-0.2, 0.2, (C, H))], axis=-1)
s0, _ = raceline_start(x0, tr, 0)
with ModelBank(p, device=0) as b:
    if mode != "plain":
        b.set_raceline(tr)
    kw = dict(raceline_start=(s0, float(x0[3]), 0.9)) if mode == "raceline" else {}
    res = plan(b, x0, U[0, 0], x0, np.zeros((2, H + 1)), U, uprev=U[0, 0], do_lookback=False, return_costs=True, **kw)
    c = np.where(np.isnan(res.costs), np.inf, res.costs)
    print(mode, N, C, sig, "global_best", res.global_best, "argmin", divmod(int(np.argmin(c)), C), "nonfinite", res.n_nonfinite, flush=True)
