"""Generate the golden fixtures by running the REFERENCE (tianhao-stan-wu/LLA-MPC) itself.

Run in the build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [/root/reference]

The reference imports ``casadi`` at module level (llampc/models/dynamic.py:17) but never
calls it on the hot path; casadi 3.5.1 is not installed here, so an empty stub module is
injected before import.  Nothing from the reference is copied: only input/output arrays
are written (``tests/golden/*.npz``) plus a repacked raceline/track data file for the
package (``lla-mpc_amd/llampc/tracks/data/tracks.npz``, data only).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
_ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
REF = _ARGS[0] if _ARGS else "/root/reference"

sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.modules.setdefault("casadi", types.ModuleType("casadi"))

from llampc.models import Dynamic                                   # noqa: E402
from llampc.params import ORCA                                      # noqa: E402
from llampc.mpc.evaluate_models_vectorized import evaluate_models_vectorized  # noqa: E402
from llampc.mpc.planner import ConstantSpeed                        # noqa: E402
from llampc.tracks import ETHZ, ETHZMobil                           # noqa: E402

VARIATION_ORDER = ("Br", "Cr", "Dr", "Bf", "Cf", "Df")
TS = 0.02
W, K = 10, 10


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path)} B")


def ref_bank(n, seed, sigma):
    """rt.py:161-177 loop, driven with the reference's ORCA()/Dynamic objects and the
    global NumPy RNG seeded with ``seed`` (the reference itself is unseeded)."""
    params = ORCA(control='pwm')
    np.random.seed(seed)
    bank = []
    for _ in range(n):
        pv = params.copy()
        for name in VARIATION_ORDER:
            pv[name] *= (1 + sigma[name] * np.random.randn())
        bank.append(Dynamic(**pv))
    arr = np.array([[getattr(m, k) for m in bank] for k in ("Bf", "Cf", "Df", "Br", "Cr", "Dr")])
    return bank, arr


def batch_model(shared, params6):
    Bf, Cf, Df, Br, Cr, Dr = params6
    return Dynamic(Bf=Bf, Cf=Cf, Df=Df, Br=Br, Cr=Cr, Dr=Dr, mass=shared.mass, lf=shared.lf,
                   lr=shared.lr, Iz=shared.Iz, Cm1=shared.Cm1, Cm2=shared.Cm2, Cr0=shared.Cr0,
                   Cr2=shared.Cr2, input_acc=False)


def config1(states, inputs, first):
    """BASELINE config 1 exactly as SURVEY.md §8(d) states it, computed by the reference:
    ETHZ, N = 100 (rt.py bank, seed 0), H = 20, C = 1, W = 10, K = 10, nominal friction.
    Look-back over DYN states[:, 490:501] / inputs[:, 490:500] (evaluate_models_vectorized +
    the rt.py:347-366 window logic), x0 = states[:, 500], U = inputs[:, 500:520],
    xref = ConstantSpeed(x0, vx0, ETHZ, 20, 0.02, projidx, curr_mu=0.9092, scale=0.9) with
    projidx the raceline point nearest x0 minus 2 (the reference's warm-start hint; "auto"),
    then H x _integrate_batch of every model under U (rk6.py:50-68 via model.py:32-40)."""
    params = ORCA(control='pwm')
    nominal = Dynamic(**params)
    rt_sigma = {"Br": 0.2, "Cr": 0.1, "Dr": 0.5, "Bf": 0.2, "Cf": 0.1, "Df": 0.5}
    N, H = 100, 20
    models, bank = ref_bank(N, 0, rt_sigma)
    p6 = tuple(bank)
    i0 = 490 - first
    s = states[:, i0:i0 + 11]
    u = inputs[:, i0:i0 + 10]
    win = np.zeros((N, W))
    errs = []
    for t in range(W):
        pred = evaluate_models_vectorized(models, N, s[:, t], u[:, t], TS, p6)
        e = np.mean((pred - s[0:4, t + 1]) ** 2, axis=1)
        win = np.roll(win, -1, axis=1)
        win[:, -1] = e
        errs.append(e)
    avg = np.mean(win, axis=1)
    x0 = states[:, 500 - first]
    U = inputs[:, 500 - first:520 - first].T[None].copy()
    tr = ETHZ(reference='optimal', longer=True)
    rl = np.asarray(tr.raceline)
    near = int(np.argmin(np.hypot(rl[0] - x0[0], rl[1] - x0[1])))
    pin = max(near - 2, 0)
    xref, pout, vr = ConstantSpeed(x0=x0[:2], v0=x0[3], track=tr, N=H, Ts=TS, projidx=pin, scale=0.9, curr_mu=0.9092)
    bm = batch_model(nominal, p6)
    xb = np.tile(x0, (N, 1))
    traj = [xb]
    for k in range(H):
        xb = bm._integrate_batch(xb, np.tile(U[0, k], (N, 1)), 0, TS)
        traj.append(xb)
    save("config1.npz", bank=bank, seed=np.array(0), states=s, inputs=u, x0=x0, U=U, uprev=u[:, -1].copy(),
         xref=xref, projidx_in=np.array(pin), projidx_out=np.array(pout), vr=np.array(vr), mu=np.array(0.9092),
         scale=np.array(0.9), errors=np.array(errs), window_mean=avg, best=np.array(np.argmin(avg)),
         topk=avg.argsort()[:K], traj=np.array(traj), W=np.array(W), K=np.array(K), H=np.array(H))


def main():
    if "--only-config1" in sys.argv:
        dyn = np.load(os.path.join(REF, "llampc/data/DYN-GPMPC-NOCONS-with_var_speedsETHZ.npz"))
        config1(np.asarray(dyn["states"][:6], dtype=np.float64), np.asarray(dyn["inputs"], dtype=np.float64), 0)
        return
    params = ORCA(control='pwm')
    nominal = Dynamic(**params)
    rt_sigma = {"Br": 0.2, "Cr": 0.1, "Dr": 0.5, "Bf": 0.2, "Cf": 0.1, "Df": 0.5}

    # ---------------- track data (package data, repacked) ----------------
    tracks = {}
    for name, cls in (("ETHZ", ETHZ), ("ETHZMobil", ETHZMobil)):
        t = cls(reference='optimal', longer=True)
        sub = "" if name == "ETHZ" else "Mobil"
        raw = np.load(os.path.join(REF, "llampc/tracks/src", f"ethz{sub}_raceline_long_.npz"))
        tracks[f"{name}_x"] = np.asarray(raw["x"], dtype=np.float64)
        tracks[f"{name}_y"] = np.asarray(raw["y"], dtype=np.float64)
        tracks[f"{name}_speeds"] = np.asarray(raw["speeds"], dtype=np.float64)
        tracks[f"{name}_mus"] = np.asarray(raw["mus"], dtype=np.float64)
        tracks[f"{name}_init"] = np.array([t.x_init, t.y_init, t.psi_init, t.vx_init])
        tracks[f"{name}_s"] = np.asarray(t.spline.s, dtype=np.float64)
        tracks[f"{name}_track_width"] = np.array(t.track_width)
        # the boundary / centre lines (ethz.py:20-42), read the reference's way
        for line in ("inner", "center", "outer"):
            tracks[f"{name}_{line}"] = np.asarray(getattr(t, line), dtype=np.float64)
    # the short optimal ETHZ raceline (ethz.py:62-65 with longer=False; no Mobil counterpart)
    raw = np.load(os.path.join(REF, "llampc/tracks/src", "ethz_raceline_.npz"))
    for k in ("x", "y", "speeds", "mus"):
        tracks[f"ETHZ_short_{k}"] = np.asarray(raw[k], dtype=np.float64)
    dpath = os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data")
    os.makedirs(dpath, exist_ok=True)
    np.savez_compressed(os.path.join(dpath, "tracks.npz"), **tracks)
    print("wrote package tracks.npz")

    # ---------------- real closed-loop trajectory slice (data) ----------------
    dyn = np.load(os.path.join(REF, "llampc/data/DYN-GPMPC-NOCONS-with_var_speedsETHZ.npz"))
    states = np.asarray(dyn["states"][:6], dtype=np.float64)
    inputs = np.asarray(dyn["inputs"], dtype=np.float64)
    lo, hi = 470, 620
    save("dyn_slice.npz", states=states[:, lo:hi + 1], inputs=inputs[:, lo:hi], first_index=np.array(lo))
    # the same bytes as package data: the scenario generator and the bench read it from there
    import shutil
    shutil.copyfile(os.path.join(HERE, "dyn_slice.npz"), os.path.join(dpath, "dyn_slice.npz"))
    config1(states, inputs, 0)

    # ---------------- bank generation: rt.py loop vs randn(N,6) ----------------
    bank_models, bank = ref_bank(1000, 0, rt_sigma)
    save("bank_rt_seed0_n1000.npz", bank=bank, seed=np.array(0))
    _, bank_wide = ref_bank(512, 7, {k: 2.0 for k in VARIATION_ORDER})
    save("bank_wide_seed7_n512.npz", bank=bank_wide, seed=np.array(7), sigma=np.array(2.0))

    # ---------------- batched dynamics on random states (a1-a3) ----------------
    rng = np.random.RandomState(11)
    n = 256
    x = np.column_stack([rng.uniform(-2, 2, n), rng.uniform(-2, 2, n), rng.uniform(-4, 4, n),
                         rng.uniform(-0.5, 3.5, n), rng.uniform(-0.5, 0.5, n), rng.uniform(-6, 6, n)])
    x[:4, 3] = [0.0, -0.0, 1e-9, -2.0]               # |vx| edge cases (atan2 at 0, reverse)
    u = np.column_stack([rng.uniform(-0.1, 1.0, n), rng.uniform(-0.35, 0.35, n)])
    p6 = tuple(bank[:, :n])
    bm = batch_model(nominal, p6)
    with np.errstate(all="ignore"):
        Ffy, Frx, Fry, af, ar = bm.calc_forces_batch(x, u, return_slip=True)
        dx = bm._diffequation_batch(None, x, u)
        x1 = bm._integrate_batch(x, u, 0, TS)
    # scalar-param model broadcast over a batch (Dynamic(**ORCA) used batch-wise)
    dx_nom = nominal._diffequation_batch(None, x, u)
    x1_nom = nominal._integrate_batch(x, u, 0, TS)
    # approx (linear tire) and input_acc variants
    apx = Dynamic(lf=params['lf'], lr=params['lr'], mass=params['mass'], Iz=params['Iz'],
                  Cf=params['Cf'], Cr=params['Cr'])
    xs = x.copy()
    xs[:4, 3] = [0.5, -0.7, 1.0, 2.0]
    dx_apx = apx._diffequation_batch(None, xs, u)
    acc = Dynamic(**{**params, "input_acc": True})
    dx_acc = acc._diffequation_batch(None, x, u)
    save("dynamics_batch.npz", x=x, u=u, params=bank[:, :n], Ffy=Ffy, Frx=Frx, Fry=Fry, alphaf=af,
         alphar=ar, dxdt=dx, x_rk4=x1, dxdt_nominal=dx_nom, x_rk4_nominal=x1_nom, x_apx=xs,
         dxdt_approx=dx_apx, dxdt_input_acc=dx_acc)

    # ---------------- look-back over real transitions (a5-a6) ----------------
    # rt.py:347-366 semantics with the reference functions, ticks over the DYN slice.
    N = 1000
    p6 = tuple(bank)
    win = np.zeros((N, W))
    count = 0
    T = 24
    errs, avgs, best, topk, preds = [], [], [], [], []
    for t in range(T):
        i = t  # transition slice index -> states[:, i] --inputs[:, i]--> states[:, i+1]
        pred = evaluate_models_vectorized(bank_models, N, states[:, lo + i], inputs[:, lo + i], TS, p6)
        e = np.mean((pred - states[0:4, lo + i + 1]) ** 2, axis=1)
        win = np.roll(win, -1, axis=1)
        win[:, -1] = e
        count = min(count + 1, W)
        errs.append(e)
        if t < 3:
            preds.append(pred)
        if count >= W:
            a = np.mean(win, axis=1)
            avgs.append(a)
            best.append(np.argmin(a))
            topk.append(a.argsort()[:K])
    save("lookback_n1000.npz", errors=np.array(errs), window_mean=np.array(avgs), best=np.array(best),
         topk=np.array(topk), pred=np.array(preds), W=np.array(W), K=np.array(K), ticks=np.array(T))

    # ---------------- look-ahead RK4 bank rollouts (a10) ----------------
    # H successive reference _integrate_batch steps for every (model, candidate)
    Nr, C, H = 64, 4, 40
    x0 = states[:, lo + 30]
    rngc = np.random.RandomState(2)
    U = np.empty((C, H, 2))
    base = inputs[:, lo + 30: lo + 30 + H].T
    U[0] = base
    for c in range(1, C):
        U[c, :, 0] = np.clip(base[:, 0] + 0.05 * rngc.randn(H), -0.1, 1.0)
        U[c, :, 1] = np.clip(base[:, 1] + 0.02 * rngc.randn(H), -0.35, 0.35)
    rp = tuple(np.repeat(bank[i, :Nr], C) for i in range(6))
    bmr = batch_model(nominal, rp)
    xb = np.tile(x0, (Nr * C, 1))
    traj = [xb]
    for k in range(H):
        ub = np.tile(U[:, k, :], (Nr, 1))
        xb = bmr._integrate_batch(xb, ub, 0, TS)
        traj.append(xb)
    traj = np.array(traj)
    save("rollout_rk4.npz", x0=x0, U=U, params=bank[:, :Nr], traj=traj, uprev=inputs[:, lo + 29])

    # wide (sigma=2) bank: non-finite rollouts, NaN handling
    Nw, Hw = 512, 20
    x0w = states[:, lo + 60]
    Uw = inputs[:, lo + 60: lo + 60 + Hw].T[None]
    bmw = batch_model(nominal, tuple(bank_wide))
    xb = np.tile(x0w, (Nw, 1))
    with np.errstate(all="ignore"):
        for k in range(Hw):
            xb = bmw._integrate_batch(xb, np.tile(Uw[:, k, :], (Nw, 1)), 0, TS)
        pw = evaluate_models_vectorized([nominal] * Nw, Nw, states[:, lo + 60], inputs[:, lo + 60], TS, tuple(bank_wide))
    save("rollout_wide.npz", x0=x0w, U=Uw, params=bank_wide, x_final=xb, lookback_pred=pw,
         x_next=states[:, lo + 61])

    # ---------------- RK6 plant (dynamic.py:59-74) with friction changes ----------------
    plant = Dynamic(**params)
    xs6 = [states[:, lo]]
    dfs, drs = [], []
    for k in range(40):
        if k >= 20:
            plant.Df -= plant.Df / 22.
            plant.Dr -= plant.Dr / 22.
        dfs.append(plant.Df)
        drs.append(plant.Dr)
        xn, _ = plant.sim_continuous(xs6[-1], inputs[:, lo + k].reshape(-1, 1), [0, TS])
        xs6.append(xn[:, -1])
    xs_multi, dxs_multi = Dynamic(**params).sim_continuous(states[:, lo], inputs[:, lo:lo + 10],
                                                            np.arange(11) * TS)
    save("plant_rk6.npz", x=np.array(xs6), u=inputs[:, lo:lo + 40], Df=np.array(dfs), Dr=np.array(drs),
         x_multi=xs_multi, dxdt_multi=dxs_multi)

    # ---------------- planner ConstantSpeed (planner.py:12-67) ----------------
    out = {}
    for name, cls in (("ETHZ", ETHZ), ("ETHZMobil", ETHZMobil)):
        t = cls(reference='optimal', longer=True)
        cases = []
        xrefs = []
        for j, (pi, mu, scale, H_) in enumerate([(0, 1.0, 1.0, 20), (5, 0.45, 0.9, 20), (100, 0.6, 0.9, 40),
                                                 (200, 0.9092265, 0.9, 20), (300, 1.0, 0.9, 40),
                                                 (350, 1.2, 0.9, 20), (480, 0.777, 0.9, 40)]):
            pi = min(pi, t.raceline.shape[1] - 12)
            px = t.raceline[:, pi + 3] + np.array([0.01, -0.02])
            v0 = 1.0 + 0.1 * j
            xr, pidx, vr = ConstantSpeed(x0=px, v0=v0, track=t, N=H_, Ts=TS, projidx=pi, scale=scale, curr_mu=mu)
            cases.append([px[0], px[1], v0, pi, mu, scale, H_, pidx, vr])
            xrefs.append(np.pad(xr, ((0, 0), (0, 41 - xr.shape[1])), constant_values=np.nan))
        out[f"{name}_cases"] = np.array(cases)
        out[f"{name}_xref"] = np.array(xrefs)
    save("planner.npz", **out)

    # ---------------- track loaders (ethz.py:15-138, track.py:12-160) ----------------
    tr = {}
    rng_t = np.random.RandomState(17)
    for name, cls in (("ETHZ", ETHZ), ("ETHZMobil", ETHZMobil)):
        t = cls()                                   # the reference's defaults: reference='center'
        tr[f"{name}_center_s"] = np.asarray(t.spline.s, dtype=np.float64)
        tr[f"{name}_center_raceline"] = np.asarray(t.raceline, dtype=np.float64)
        tr[f"{name}_center_init"] = np.array([t.x_init, t.y_init, t.psi_init, t.vx_init])
        tr[f"{name}_track_length"] = np.array(t.track_length)
        tr[f"{name}_theta_track"] = np.asarray(t.theta_track, dtype=np.float64)
        thetas = np.concatenate([[0.0, 1e-3], rng_t.uniform(0, t.track_length, 30), [t.theta_track[-1] - 1e-6]])
        tr[f"{name}_thetas"] = thetas
        tr[f"{name}_param_to_xy"] = np.array([t.param_to_xy(th) for th in thetas])
        idx = rng_t.randint(0, t.center.shape[1], 30)
        pts = t.center[:, idx].T + rng_t.uniform(-0.1, 0.1, (30, 2))
        mid_close = 0.5 * (t.center[:, -1] + t.center[:, 0])          # on the closing segment
        pts = np.vstack([pts, mid_close + [0.001, -0.001]])
        tr[f"{name}_xy_points"] = pts
        tr[f"{name}_xy_to_param"] = np.array([t.xy_to_param(px, py) for px, py in pts])
        proj = [t.project(px, py, t.center_line) for px, py in pts]
        tr[f"{name}_project_xy"] = np.array([p[0] for p in proj])
        tr[f"{name}_project_idx"] = np.array([p[1] for p in proj])
        try:                                        # no speed profiles on the centre line
            ConstantSpeed(x0=t.raceline[:, 5], v0=1.0, track=t, N=5, Ts=TS, projidx=0)
            tr[f"{name}_center_constantspeed_error"] = np.array("")
        except Exception as e:                      # noqa: BLE001
            tr[f"{name}_center_constantspeed_error"] = np.array(type(e).__name__)
    ts = ETHZ(reference='optimal', longer=False)
    tr["ETHZ_short_s"] = np.asarray(ts.spline.s, dtype=np.float64)
    tr["ETHZ_short_mus"] = np.asarray(ts.mus, dtype=np.float64)
    cases, xrefs = [], []
    for j, (pi, mu, scale, H_) in enumerate([(0, 1.0, 1.0, 20), (120, 0.55, 0.9, 40), (300, 0.8, 0.9, 20),
                                             (480, 0.95, 0.9, 40)]):
        px = ts.raceline[:, pi + 3] + np.array([0.01, -0.02])
        xr, pidx, vr = ConstantSpeed(x0=px, v0=1.0 + 0.2 * j, track=ts, N=H_, Ts=TS, projidx=pi, scale=scale,
                                     curr_mu=mu)
        cases.append([px[0], px[1], 1.0 + 0.2 * j, pi, mu, scale, H_, pidx, vr])
        xrefs.append(np.pad(xr, ((0, 0), (0, 41 - xr.shape[1])), constant_values=np.nan))
    tr["ETHZ_short_cases"] = np.array(cases)
    tr["ETHZ_short_xref"] = np.array(xrefs)
    try:
        ETHZMobil(reference='optimal', longer=False)
        tr["ETHZMobil_short_error"] = np.array("")
    except Exception as e:                          # noqa: BLE001
        tr["ETHZMobil_short_error"] = np.array(type(e).__name__)
    save("tracks_center.npz", **tr)

    # ---------------- closed-loop look-back + mu-hat emulation (rt.py:269-366) ----------------
    # Plant: reference RK6 with a gradual friction drop; controls: recorded DYN inputs
    # (IPOPT is not available).  Records the reference tick logic's outputs.
    Nc = 400
    bank_c_models, bank_c = ref_bank(Nc, 3, rt_sigma)
    p6c = tuple(bank_c)
    plant = Dynamic(**params)
    pr = dict(params)
    x_cur = states[:, lo].copy()
    winc = np.zeros((Nc, W))
    cnt = 0
    cur = 0
    drs_p, dfs_p, mu_pred_hist, mu_log, cur_hist, topk_hist, xs_hist = [], [], [], [], [], [], [x_cur]
    smooth = None
    ind_best = None
    mu_pred = None
    n_ticks = 60
    for idt in range(n_ticks):
        if idt > 5:                                          # gradual drop from tick 6 on
            plant.Df -= plant.Df / 260.
            plant.Dr -= plant.Dr / 260.
            pr['Df'], pr['Dr'] = plant.Df, plant.Dr
        u_t = inputs[:, lo + idt]
        xn, _ = plant.sim_continuous(x_cur, u_t.reshape(-1, 1), [0, TS])
        x_next = xn[:, -1]
        if idt <= W:
            drs_p.append(1.0 * params['mass'] * 9.8 * params['lr'] / (params['lf'] + params['lr']))
            dfs_p.append(1.0 * params['mass'] * 9.8 * params['lf'] / (params['lf'] + params['lr']))
            mu_log.append(1.0)
        else:
            drs_p.append(np.mean([bank_c_models[b].Dr for b in ind_best]))
            dfs_p.append(np.mean([bank_c_models[b].Df for b in ind_best]))
            mu_pred = (np.mean(np.array(drs_p)[-20:]) + np.mean(np.array(dfs_p)[-20:])) / (9.81 * params['mass'])
            smooth = mu_pred if smooth is None else 0.08 * mu_pred + (1 - 0.08) * smooth
            mu_log.append(smooth * .95)
        mu_pred_hist.append(np.nan if mu_pred is None else mu_pred)
        if idt > 0:
            e = np.mean((evaluate_models_vectorized(bank_c_models, Nc, x_cur, u_t, TS, p6c) - x_next[0:4]) ** 2, axis=1)
            winc = np.roll(winc, -1, axis=1)
            winc[:, -1] = e
            cnt = min(cnt + 1, W)
            if cnt >= W:
                a = np.mean(winc, axis=1)
                cur = np.argmin(a)
                ind_best = a.argsort()[:10]
        cur_hist.append(cur)
        topk_hist.append(ind_best if ind_best is not None else np.full(10, -1))
        x_cur = x_next
        xs_hist.append(x_cur)
    save("closed_loop.npz", bank=bank_c, seed=np.array(3), x=np.array(xs_hist), u=inputs[:, lo:lo + n_ticks],
         current=np.array(cur_hist), topk=np.array(topk_hist), mu_pred=np.array(mu_pred_hist),
         mu_logged=np.array(mu_log), drop_after=np.array(5), drop_div=np.array(260.0))

    # ---------------- friction schedule known answers (results/**/MUs.npy) ----------------
    mus = {}
    for case in ("LLA/CASE 2 (GRAD AFTER)", "LLA/CASE 4 (SUDD AFTER) - 22", "LLA/CASE 5 (CONSTANT)",
                 "LLA T2/CASE 2 (GRAD AFTER)", "LLA/CASE 3 (SUDD BEG) - 22"):
        a = np.load(os.path.join(REF, "results", case, "MUs.npy"), allow_pickle=False)
        key = case.replace("/", "_").replace(" ", "").replace("(", "").replace(")", "").replace("-", "_")
        mus[key] = np.asarray(a, dtype=np.float64)
    save("mus_known_answers.npz", **mus)


if __name__ == "__main__":
    main()
