"""Accuracy headroom of the look-ahead (verdict r04 #5): the largest relative error of the HIP
path's rollout costs against the oracle (oracle/llampc_oracle.py, pinned to the reference) per
shape, and of the final states where an API returns them, with the worst pair's conditioning —
how much its cost moves when x0 moves by one ulp in the oracle itself (so an error that the
arithmetic order alone can produce is told apart from a wrong kernel).

  c1_h20 / c1_h40   plan(): N = 10^4, C = 1, H = 20 / 40 (the headline path, LPM 4)
  c64_h20           plan(): N = 10^4, C = 64, H = 20 (the work-queue layout, LPM 1)
  ctl_h40           LLAMPC.tick (device mode): N = 10^4, C = 64, H = 40, 14 closed-loop ticks,
                    every rolled-out slot's best cost vs ControllerOracle
  wide              the sigma = 2 bank (tests/golden/rollout_wide.npz): costs (plan) and final
                    states (llampc_integrate_batch, RK4) vs the reference's own x_final

  c2_scenario / c3_scenario  plan() on configs 2 / 3's own scenario states (llampc.mpc.scenarios)

usage: python tools/diag/accuracy_headroom.py [out.json] [case,case,...]   (GPU)"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from oracle import llampc_oracle as O  # noqa: E402

TS = 0.02
Q, R, P = np.eye(2), np.diag([5e-3, 1.0]), np.zeros((2, 2))
p0 = O.orca_params()
SHARED = {k: p0[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}


def relerr(got, want):
    got, want = np.asarray(got, dtype=np.float64).ravel(), np.asarray(want, dtype=np.float64).ravel()
    fin = np.isfinite(want) & np.isfinite(got)
    assert np.array_equal(np.isfinite(got), np.isfinite(want)), "finiteness differs"
    r = np.abs(got[fin] - want[fin]) / np.maximum(np.abs(want[fin]), 1e-300)
    idx = np.flatnonzero(fin)
    j = int(np.argmax(r)) if r.size else 0
    return {"max": float(r.max()) if r.size else 0.0, "p99_9": float(np.quantile(r, 0.999)) if r.size else 0.0,
            "median": float(np.median(r)) if r.size else 0.0, "n": int(r.size), "worst_index": int(idx[j]) if r.size else -1}


def conditioning(bank, flat_index, C, x0, U, xref, uprev):
    """Relative cost change of pair `flat_index` (model n = i // C, candidate c = i % C) when x0
    is perturbed by one ulp per component in the oracle: the error the arithmetic order alone
    can produce, to compare the kernel's error with."""
    n, c = divmod(flat_index, C)
    cols = tuple(bank[:, [n]])
    Uc = U[c:c + 1]
    base = O.mpc_cost(O.rollout_rk4(SHARED, cols, x0, Uc, TS), Uc, xref, uprev, Q, R, P)[0]
    worst = 0.0
    for j in range(6):
        xp = x0.copy()
        xp[j] = np.nextafter(xp[j], np.inf)
        cj = O.mpc_cost(O.rollout_rk4(SHARED, cols, xp, Uc, TS), Uc, xref, uprev, Q, R, P)[0]
        worst = max(worst, abs(cj - base) / abs(base))
    return {"model": int(n), "cand": int(c), "cost": float(base), "ulp_x0_rel_change": worst}


def plan_case(name, N, C, H, seed=0):
    from llampc.mpc import CandidateGenerator, ModelBank, generate_bank, plan
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    d = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    bank = generate_bank(N, seed=seed)
    gen = CandidateGenerator(C, H, seed=2)
    W = 10
    with ModelBank(bank, W=W, device=0) as b:
        for t in range(1, W + 2):
            x_t = s[:, t]
            xref, _, _ = ConstantSpeed(x_t[:2], x_t[3], tr, H, TS, 0, curr_mu=0.9, scale=0.9)
            U = gen(None, u[:, t]) if C > 1 else np.tile(u[:, t], (H, 1))[None]
            res = plan(b, x_t, u[:, t - 1], s[:, t - 1], xref, U, Ts=TS, K=10, return_costs=(t == W + 1))
    x0, uprev = s[:, W + 1], u[:, W]
    t0 = time.time()
    cref = O.mpc_cost(O.rollout_rk4(SHARED, tuple(bank), x0, U, TS), U, xref, uprev, Q, R, P)
    out = {"shape": name, "N": N, "C": C, "H": H, "cost": relerr(res.costs.ravel(), cref),
           "oracle_s": time.time() - t0}
    out["worst_conditioning"] = conditioning(bank, out["cost"]["worst_index"], C, x0, U, xref, uprev)
    return out


def scenario_case(name, track, H, seed, N=10000, C=1, W=10, K=10):
    """Configs 2 / 3 on their own scenario states (llampc.mpc.scenarios, the test's inputs):
    every full-window tick's N costs."""
    from llampc.mpc import ModelBank, generate_bank, plan
    from llampc.mpc.scenarios import scenario_ticks, unpack
    ticks = scenario_ticks(track, H, C, W + 3, device=0)
    bank = generate_bank(N, seed=seed)
    got, want, worst = [], [], None
    with ModelBank(bank, W=W, device=0) as b:
        for t, pk in enumerate(ticks):
            f = unpack(pk, H, C)
            last = t >= W - 1
            res = plan(b, f["x_now"], f["u_prev"], f["x_prev"], f["xref"], f["U"], uprev=f["uprev"], Ts=TS, K=K,
                       return_costs=last)
            if not last:
                continue
            cref = O.mpc_cost(O.rollout_rk4(SHARED, tuple(bank), f["x_now"], f["U"], TS), f["U"], f["xref"],
                              f["uprev"], Q, R, P)
            r = relerr(res.costs.ravel(), cref)
            if worst is None or r["max"] > worst[0]["max"]:
                worst = (r, f)
            got.append(res.costs.ravel())
            want.append(cref)
    out = {"shape": name, "N": N, "C": C, "H": H, "cost": relerr(np.concatenate(got), np.concatenate(want))}
    r, f = worst
    out["worst_conditioning"] = conditioning(bank, r["worst_index"], C, f["x_now"], f["U"], f["xref"], f["uprev"])
    out["worst_conditioning"]["err"] = r["max"]
    return out


def ctl_case(N=10000, C=64, H=40, W=10, K=10, ticks=14):
    from llampc.mpc import LLAMPC, ModelBank, generate_bank
    from llampc.tracks import ETHZ
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td["ETHZ_x"], td["ETHZ_y"], td["ETHZ_speeds"], td["ETHZ_mus"])
    tr = ETHZ('optimal', True)
    bank = generate_bank(N, seed=0)
    orc = O.ControllerOracle(SHARED, bank, ref, tr.lap_projidx, H=H, C=C, K=K, W=W, Ts=TS)
    plant = O.Vehicle.from_params(p0)
    x = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))["states"][:, 0].copy()
    got, want = [], []
    with ModelBank(bank, W=W, device=0) as b, LLAMPC(b, tr, H=H, C=C, K=K) as ctl:
        for t in range(ticks):
            res = ctl.tick(x)
            o = orc.tick(x)
            got.append(res.cost)
            want.append(o["cost"])
            if not o["warm"]:
                got.extend(np.asarray(res.raw.plan.topk_cost[:K]))
                want.extend(o["topk_cost"])
            plant.Df *= 1 - 1 / 260.0
            plant.Dr *= 1 - 1 / 260.0
            xn, _ = O.sim_continuous(plant, x, res.u_seq[:, 0].reshape(2, 1), [0, TS])
            x = xn[:, -1]
    return {"shape": "ctl_h40", "N": N, "C": C, "H": H, "ticks": ticks, "cost": relerr(got, want)}


def wide_case():
    from llampc import _native as nat
    from llampc.models import Dynamic
    from llampc.mpc import ModelBank, plan
    g = np.load(os.path.join(REPO, "tests", "golden", "rollout_wide.npz"))
    p, x0, U = g["params"], g["x0"], g["U"]
    N, H = p.shape[1], U.shape[1]
    xref = np.vstack([x0[0] + 0.03 * np.arange(H + 1), x0[1] + 0.01 * np.arange(H + 1)])
    uprev = U[0, 0]
    with ModelBank(p, W=1, device=0) as b:
        res = plan(b, x0, uprev, x0, xref, U, uprev=uprev, Ts=TS, K=10, do_lookback=False, return_costs=True)
    with np.errstate(all="ignore"):
        cref = O.mpc_cost(O.rollout_rk4(SHARED, tuple(p), x0, U, TS), U, xref, uprev, Q, R, P)
    m = Dynamic(**{**p0, **{k: p[i] for i, k in enumerate(O.BANK_ORDER)}})
    xf = m._native_integrate(np.tile(x0, (N, 1)), np.tile(U, (N, 1, 1)), np.full(H, TS), nat.RK4, final_only=True)
    return {"shape": "wide", "N": N, "C": 1, "H": H, "cost": relerr(res.costs.ravel(), cref),
            "final_state_integrate_api": relerr(xf, g["x_final"])}


def nlp_case():
    """setupNLP's objective against the committed SLSQP local optima (tests/golden/nlp_optimum.npz):
    fval / f* per case (the test bounds it by 1.05)."""
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.tracks import ETHZ
    g = np.load(os.path.join(REPO, "tests", "golden", "nlp_optimum.npz"))
    ratios = []
    for i in range(len(g["fstar"])):
        nlp = setupNLP(int(g["xref"][i].shape[1] - 1), TS, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p0,
                       Dynamic(**p0, device=0), ETHZ('optimal', True), device=0)
        try:
            _, fval, _, _ = nlp.solve(g["x0"][i], g["xref"][i], g["uprev"][i])
        finally:
            nlp.close()
        ratios.append(fval / float(g["fstar"][i]))
    return {"shape": "nlp_vs_slsqp", "fval_over_fstar": ratios, "max": float(max(ratios))}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    cases = [("c2_scenario", lambda: scenario_case("c2_scenario", "ETHZ", 20, 0)),
             ("c3_scenario", lambda: scenario_case("c3_scenario", "ETHZMobil", 40, 1)),
             ("c1_h20", lambda: plan_case("c1_h20", 10000, 1, 20)), ("c1_h40", lambda: plan_case("c1_h40", 10000, 1, 40)),
             ("wide", wide_case), ("ctl_h40", ctl_case), ("nlp", nlp_case),
             ("c64_h20", lambda: plan_case("c64_h20", 10000, 64, 20))]
    rows = [fn() for name, fn in cases if only is None or name in only]
    for r in rows:
        print(json.dumps(r), flush=True)
    if out:
        json.dump(rows, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
