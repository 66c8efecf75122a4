"""GPU parity tests: the HIP path (through the C ABI) against the pinned oracle and the
reference-generated golden vectors.  Tolerances: fp64 values 1e-9 relative for one
integration step (the fast cores vs NumPy's libm differ by ulps), 1e-7 for H-step rollouts and
their costs (the look-ahead's 8-term lean cores: the largest error measured on a well-conditioned
shape is 1e-10, profiles/r05/accuracy_lean.txt; north star bound: 1e-5); indices exact
(tie-tolerant only where stated).  Ill-conditioned rollouts (a one-ulp change of x0 moves the
cost visibly in the oracle itself) are held to their core-error bound — the lean cores'
measured errors propagated through the oracle's rollout (conftest.core_error_bound) — in
tests/test_configs_gpu.py, tests/test_ctl_gpu.py and the wide-sigma argmin test here."""
import os

import numpy as np
import pytest

from conftest import core_error_bound, golden
from oracle import llampc_oracle as O

pytestmark = pytest.mark.gpu

TS = 0.02
RTOL_STEP = 1e-9
RTOL_ROLL = 1e-7


@pytest.fixture(scope="module")
def nat():
    from llampc import _native
    _native.load()
    if _native.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    return _native


def shared():
    p = O.orca_params()
    return {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}


def close(a, b, rtol, scale=None):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    fin = np.isfinite(b)
    np.testing.assert_array_equal(np.isfinite(a), fin)
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    sc = np.max(np.abs(b[fin])) if scale is None and fin.any() else (scale or 1.0)
    np.testing.assert_allclose(a[fin], b[fin], rtol=rtol, atol=rtol * 1e-3 * sc)


# ----------------------------------------------------------------- Dynamic API (a1-a3)
def test_dynamic_batch_forces_deriv_rk4(nat):
    from llampc.models import Dynamic
    g = golden("dynamics_batch.npz")
    p = O.orca_params()
    Bf, Cf, Df, Br, Cr, Dr = g["params"]
    m = Dynamic(**{**p, "Bf": Bf, "Cf": Cf, "Df": Df, "Br": Br, "Cr": Cr, "Dr": Dr})
    Ffy, Frx, Fry, af, ar = m.calc_forces_batch(g["x"], g["u"], return_slip=True)
    for a, k in ((Ffy, "Ffy"), (Frx, "Frx"), (Fry, "Fry"), (af, "alphaf"), (ar, "alphar")):
        close(a, g[k], RTOL_STEP)
    close(m._diffequation_batch(None, g["x"], g["u"]), g["dxdt"], RTOL_STEP)
    close(m._integrate_batch(g["x"], g["u"], 0, TS), g["x_rk4"], RTOL_STEP)
    nom = Dynamic(**p)
    close(nom._diffequation_batch(None, g["x"], g["u"]), g["dxdt_nominal"], RTOL_STEP)
    close(nom._integrate_batch(g["x"], g["u"], 0, TS), g["x_rk4_nominal"], RTOL_STEP)


def test_dynamic_approx_and_input_acc(nat):
    from llampc.models import Dynamic
    g = golden("dynamics_batch.npz")
    p = O.orca_params()
    apx = Dynamic(lf=p["lf"], lr=p["lr"], mass=p["mass"], Iz=p["Iz"], Cf=p["Cf"], Cr=p["Cr"])
    assert apx.approx
    close(apx._diffequation_batch(None, g["x_apx"], g["u"]), g["dxdt_approx"], RTOL_STEP)
    acc = Dynamic(**{**p, "input_acc": True})
    close(acc._diffequation_batch(None, g["x"], g["u"]), g["dxdt_input_acc"], RTOL_STEP)


def test_sim_continuous_rk6_plant(nat):
    from llampc.models import Dynamic
    g = golden("plant_rk6.npz")
    p = O.orca_params()
    x = g["x"][0]
    for k in range(g["u"].shape[1]):
        m = Dynamic(**{**p, "Df": g["Df"][k], "Dr": g["Dr"][k]})
        xn, _ = m.sim_continuous(x, g["u"][:, k:k + 1], [0, TS])
        x = xn[:, -1]
        close(x, g["x"][k + 1], RTOL_ROLL)
    xm, dm = Dynamic(**p).sim_continuous(g["x"][0], g["u"][:, :10], np.arange(11) * TS)
    close(xm, g["x_multi"], RTOL_ROLL)
    close(dm, g["dxdt_multi"], RTOL_ROLL)
    f = Dynamic(**p).calc_forces(g["x"][0], g["u"][:, 0])
    fo = O.calc_forces(O.Vehicle.from_params(p), g["x"][0], g["u"][:, 0])
    close(np.array(f), np.array(fo), RTOL_STEP)


def test_evaluate_models_vectorized_dropin(nat):
    from llampc.models import Dynamic
    from llampc.mpc import evaluate_models_vectorized
    g = golden("lookback_n1000.npz")
    d = golden("dyn_slice.npz")
    bank = golden("bank_rt_seed0_n1000.npz")["bank"]
    models = [Dynamic(**O.orca_params())] * bank.shape[1]
    for t in range(3):
        pred = evaluate_models_vectorized(models, len(models), d["states"][:, t], d["inputs"][:, t], TS, tuple(bank))
        close(pred, g["pred"][t], RTOL_STEP)


# ----------------------------------------------------------------- look-back (a5-a6)
def test_lookback_window_argmin_topk_vs_golden(nat):
    from llampc.mpc import ModelBank
    g = golden("lookback_n1000.npz")
    d = golden("dyn_slice.npz")
    bank = golden("bank_rt_seed0_n1000.npz")["bank"]
    s, u = d["states"], d["inputs"]
    full = 0
    with ModelBank(bank, W=int(g["W"]), device=0) as b:
        for t in range(int(g["ticks"])):
            r = b.lookback(s[:, t], u[:, t], s[:, t + 1], Ts=TS, K=int(g["K"]), return_errors=True,
                           return_window_mean=True)
            close(r["errors"], g["errors"][t], RTOL_STEP)
            if r["full"]:
                close(r["window_mean"], g["window_mean"][full], RTOL_STEP)
                assert r["best"] == g["best"][full]
                np.testing.assert_array_equal(r["topk"], g["topk"][full])
                np.testing.assert_allclose(r["topk_val"], g["window_mean"][full][g["topk"][full]], rtol=RTOL_STEP)
                full += 1
        assert full == len(g["best"])
        ring = b.window()
        np.testing.assert_allclose(ring[:, -1], g["errors"][-1], rtol=RTOL_STEP)
        np.testing.assert_allclose(ring[:, 0], g["errors"][-int(g["W"])], rtol=RTOL_STEP)


@pytest.mark.parametrize("N,W,K", [(1, 1, 1), (5, 3, 10), (257, 10, 10), (1000, 8, 32), (3001, 17, 7),
                                   (700, 16, 5)])
def test_lookback_edge_shapes(nat, N, W, K):
    """Ragged N (not a multiple of 256), N < K (padding with -1), W below/above 8 (both
    pairwise-sum branches; W = 8 and 16: the newest error is the last term of the 8th partial
    sum, the other W the sequential tail's last add — win_pre / win_finish), K up to KMAX."""
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    p = generate_bank(N, seed=N)
    win = O.LookbackWindow(N, W, K)
    with ModelBank(p, W=W, device=0) as b:
        for t in range(W + 2):
            r = b.lookback(s[:, t], u[:, t], s[:, t + 1], Ts=TS, K=K, return_errors=True, return_window_mean=True)
            e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, t], u[:, t], TS), s[:, t + 1])
            close(r["errors"], e, RTOL_STEP)
            assert win.push(e) == r["full"]
            if r["full"]:
                close(r["window_mean"], win.avg, RTOL_STEP)
                assert r["best"] == win.current
                kk = min(K, N)
                np.testing.assert_array_equal(r["topk"][:kk], win.best_k[:kk])
                assert np.all(r["topk"][kk:] == -1)


def test_lookback_nan_semantics(nat):
    """np.argmin returns the first NaN (rt.py:359); argsort puts NaN last (rt.py:360)."""
    from llampc.mpc import ModelBank
    g = golden("rollout_wide.npz")
    p = g["params"]
    x0, u0 = g["x0"], g["U"][0, 0]
    with np.errstate(all="ignore"):
        e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), x0, u0, TS), g["x_next"])
    p = p.copy()
    p[2, 7] = np.nan          # a NaN model (Df) -> NaN error
    p[2, 300] = np.nan
    with np.errstate(all="ignore"):
        e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), x0, u0, TS), g["x_next"])
    assert np.isnan(e[7]) and np.isnan(e[300])
    for policy in (0, 1):
        with ModelBank(p, W=1, device=0) as b:
            r = b.lookback(x0, u0, g["x_next"], Ts=TS, K=10, nan_policy=policy, return_errors=True)
            close(r["errors"], e, RTOL_STEP)
            if policy == 0:
                assert r["best"] == int(np.argmin(e)) == 7
            else:
                assert r["best"] == int(np.nanargmin(e))
            np.testing.assert_array_equal(r["topk"], e.argsort(kind="stable")[:10])


@pytest.mark.parametrize("N,K", [(200_000, 10), (200_000, 1), (60_000, 32)])
def test_lookback_selection_ties_nans_many_lists(nat, N, K):
    """The look-back selection at sizes where each lane ranks several models (R > 1) and
    lb_final merges hundreds of per-wave lists (up to its 512-list cap at K = 1), with exact
    ties (duplicated models: equal errors -> lower index first, the stable argsort) and NaN
    models (argmin: first NaN under NaN-first; argsort: NaN last).  Expected indices come from
    the kernel's own errors (the selection is exact); the errors match the oracle."""
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    p = generate_bank(N, seed=5)
    e0 = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, 0], u[:, 0], TS), s[:, 1])
    best = int(np.argmin(e0))
    dup = np.array([i for i in (best + 7, best + 3001, best + 45_000, N - 1, 3) if 0 <= i < N and i != best])
    p[:, dup] = p[:, [best]]                      # exact ties with the best model
    p[2, [11, N // 2]] = np.nan                  # NaN models
    with np.errstate(all="ignore"):
        e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, 0], u[:, 0], TS), s[:, 1])
    for policy in (0, 1):
        with ModelBank(p, W=1, device=0) as b:
            r = b.lookback(s[:, 0], u[:, 0], s[:, 1], Ts=TS, K=K, nan_policy=policy, return_errors=True)
        g = r["errors"]
        close(g, e, RTOL_STEP)
        assert np.array_equal(np.isnan(g), np.isnan(e))
        assert np.all(g[dup] == g[best])
        if policy == 0:
            assert r["best"] == int(np.argmin(g)) == 11
        else:
            assert r["best"] == int(np.nanargmin(g))
        np.testing.assert_array_equal(r["topk"][:K], g.argsort(kind="stable")[:K])


@pytest.mark.parametrize("case", ["all_equal", "mostly_nan", "few_finite"])
def test_lookback_topk_degenerate_banks(nat, case):
    """lb_final's threshold merge (T = the K-th smallest block head) on degenerate banks:
    every model identical (every key ties across all block lists: the top-K is indices
    0..K-1), 6 of 7 models NaN (the NaN entries fill the lists' tails and, under NaN-first,
    the argmin is the first NaN), and fewer finite models than K (NaN entries enter the
    top-K in index order, np.argsort's NaN-last order)."""
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, K = 3000, 10
    p = generate_bank(N, seed=8)
    if case == "all_equal":
        p[:] = p[:, [17]]
    elif case == "mostly_nan":
        p[2, np.arange(N) % 7 != 3] = np.nan
    else:
        p[2, np.arange(N) % 600 != 599] = np.nan          # 5 finite models
    for policy in (0, 1):
        with ModelBank(p, W=2, device=0) as b:
            for t in range(2):
                r = b.lookback(s[:, t], u[:, t], s[:, t + 1], Ts=TS, K=K, nan_policy=policy,
                               return_errors=True, return_window_mean=True)
        wm = r["window_mean"]
        with np.errstate(all="ignore"):
            e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, 1], u[:, 1], TS), s[:, 2])
        close(r["errors"], e, RTOL_STEP)
        np.testing.assert_array_equal(r["topk"], wm.argsort(kind="stable")[:K])
        if policy == 0:
            assert r["best"] == int(np.argmin(wm))
        else:
            assert r["best"] == (int(np.nanargmin(wm)) if np.isfinite(wm).any() else 0)
        if case == "all_equal":
            np.testing.assert_array_equal(r["topk"], np.arange(K))


# ----------------------------------------------------------------- look-ahead (a8-a10)
def test_lookahead_rk4_rollout_and_cost_vs_golden(nat):
    from llampc import _native
    from llampc.mpc import ModelBank
    g = golden("rollout_rk4.npz")
    U, x0, p = g["U"], g["x0"], g["params"]
    N, C_ = p.shape[1], U.shape[0]
    Q, R, P = np.diag([1, 1]), np.diag([5e-3, 1]), np.diag([0, 0])
    for H in (20, 40):
        xref = np.vstack([g["traj"][:H + 1, 0, 0] + 0.01, g["traj"][:H + 1, 0, 1] - 0.02])
        cref = O.mpc_cost(g["traj"][:H + 1], U[:, :H], xref, g["uprev"], Q, R, P)
        with ModelBank(p, device=0) as b:
            r = b.lookahead(x0, U[:, :H], xref, g["uprev"], Ts=TS, return_costs=True, return_best_cand=True)
        close(r["costs"].ravel(), cref, RTOL_ROLL)
        cm = cref.reshape(N, C_)
        np.testing.assert_array_equal(r["best_cand_per_model"], np.argmin(cm, axis=1))
        assert (r["best_model"], r["best_cand"]) == divmod(int(np.argmin(cref)), C_)
    # the final states through the raw integrate API (rk4, per-lane controls)
    from llampc.models import Dynamic
    rp = np.repeat(p, C_, axis=1)
    m = Dynamic(**{**O.orca_params(), **{k: rp[i] for i, k in enumerate(O.BANK_ORDER)}})
    u = np.tile(U, (N, 1, 1))
    traj = m._native_integrate(np.tile(x0, (N * C_, 1)), u, np.full(40, TS), _native.RK4, final_only=False)
    close(traj, g["traj"], RTOL_ROLL)


@pytest.mark.parametrize("C,H,N", [(1, 20, 300), (3, 7, 300), (64, 20, 300), (100, 5, 300),
                                   (130, 40, 300), (1000, 12, 3)])
def test_lookahead_candidate_group_shapes(nat, C, H, N):
    """C=1 (lane per model), non-power-of-two C, C = 64 (one model per wave), 64 < C <= 256
    (a model spans 2 or 4 waves: per-model argmin across waves in LDS), C > 256 (lanes loop
    over candidates), LDS staging on (small C*H) and off (C*H*16 > 48 KB)."""
    from llampc.mpc import ModelBank, generate_bank
    p = generate_bank(N, seed=C)
    rng = np.random.RandomState(C)
    x0 = np.array([0.2, 0.1, -0.7, 1.5, 0.02, 0.3])
    U = np.stack([rng.uniform(-0.1, 1.0, (C, H)), rng.uniform(-0.35, 0.35, (C, H))], axis=-1)
    xref = np.vstack([0.2 + 0.03 * np.arange(H + 1), 0.1 - 0.02 * np.arange(H + 1)])
    uprev = np.array([0.3, 0.0])
    with np.errstate(all="ignore"):
        traj = O.rollout_rk4(shared(), tuple(p), x0, U, TS)
        cref = O.mpc_cost(traj, U, xref, uprev, np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2)))
    with ModelBank(p, device=0) as b:
        r = b.lookahead(x0, U, xref, uprev, Ts=TS, return_costs=True, return_best_cand=True)
    close(r["costs"].ravel(), cref, RTOL_ROLL)
    cm = np.where(np.isnan(cref), np.inf, cref).reshape(N, C)
    np.testing.assert_array_equal(r["best_cand_per_model"], np.argmin(cm, axis=1))
    assert r["best_model"] * C + r["best_cand"] == int(np.argmin(cm.ravel()))


@pytest.mark.parametrize("Q,P", [(np.diag([2.0, 0.5]), np.diag([3.0, 0.25])),       # split quads
                                 (np.array([[1.0, 0.3], [0.2, 2.0]]), np.array([[0.5, -0.1], [0.4, 1.0]]))])
def test_lookahead_weighted_cost(nat, Q, P):
    """nmpc.py:44-111 with other Q and terminal P than rt.py's: diagonal weights take the
    position split of the LPM-4 quads (each lane one position component), full matrices the
    unsplit path; both against the oracle's cost on the reference rollouts."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    N, C, H = 500, 3, 20
    p = generate_bank(N, seed=21)
    rng = np.random.RandomState(21)
    x0 = np.array([0.3, -0.2, 0.9, 1.7, -0.03, 0.5])
    U = np.stack([rng.uniform(-0.1, 1.0, (C, H)), rng.uniform(-0.3, 0.3, (C, H))], axis=-1)
    xref = np.vstack([0.3 + 0.02 * np.arange(H + 1), -0.2 + 0.03 * np.arange(H + 1)])
    uprev = np.array([0.4, 0.05])
    R = np.diag([5e-3, 1.0])
    with np.errstate(all="ignore"):
        traj = O.rollout_rk4(shared(), tuple(p), x0, U, TS)
        cref = O.mpc_cost(traj, U, xref, uprev, Q, R, P)
    cost = _native.cost_struct(Q=Q, R=R, P=P)
    with ModelBank(p, device=0) as b:
        r = b.lookahead(x0, U, xref, uprev, Ts=TS, cost=cost, return_costs=True, return_best_cand=True)
    close(r["costs"].ravel(), cref, RTOL_ROLL)
    cm = np.where(np.isnan(cref), np.inf, cref).reshape(N, C)
    np.testing.assert_array_equal(r["best_cand_per_model"], np.argmin(cm, axis=1))


def test_lookahead_feasibility_mask(nat):
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    N, C, H = 64, 6, 10
    p = generate_bank(N, seed=1)
    U = np.zeros((C, H, 2))
    U[:, :, 0] = 0.5
    U[1, 3, 1] = 0.2          # steering jump 0.2 > 5*Ts -> infeasible
    U[2, 0, 0] = 1.2          # pwm above max -> infeasible
    U[3, :, 1] = np.linspace(0, 0.09, H)   # within rate
    xref = np.zeros((2, H + 1))
    ok = O.candidates_feasible(U, np.zeros(2), [-0.1, -0.35], [1.0, 0.35], 5.0, TS)
    assert list(ok) == [True, False, False, True, True, True]
    cost = _native.cost_struct(enforce_bounds=True)
    x0 = np.array([0, 0, 0, 1.0, 0, 0])
    with ModelBank(p, device=0) as b:
        r = b.lookahead(x0, U, xref, np.zeros(2), Ts=TS, cost=cost, return_costs=True)
    assert np.all(np.isinf(r["costs"][:, ~ok])) and np.all(np.isfinite(r["costs"][:, ok]))


def test_lookahead_euler_nlp_and_rk6(nat):
    """NLP-form Euler (dynamic.py:195-226 + nmpc.py:58-60; restated, parity unpinned) and
    RK6 look-ahead integrators against the oracle restatements."""
    from llampc.mpc import ModelBank, generate_bank
    N, C, H = 200, 2, 20
    p = generate_bank(N, seed=4)
    x0 = np.array([0.1, 0.2, 0.3, 0.03, 0.01, 0.2])      # vx < vmin: exercises the clamp
    U = np.zeros((C, H, 2))
    U[:, :, 0] = [[0.6], [0.9]]
    U[:, :, 1] = 0.05
    xref = np.zeros((2, H + 1))
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    with ModelBank(p, device=0) as b:
        r = b.lookahead(x0, U, xref, np.zeros(2), Ts=TS, integrator="euler_nlp", return_costs=True)
        traj = O.rollout_euler_nlp(shared(), tuple(p), x0, U, TS)
        close(r["costs"].ravel(), O.mpc_cost(traj, U, xref, np.zeros(2), Q, R, P), RTOL_ROLL)
        x0b = np.array([0.1, 0.2, 0.3, 1.0, 0.01, 0.2])
        r6 = b.lookahead(x0b, U, xref, np.zeros(2), Ts=TS, integrator="rk6", return_costs=True)
    # Dynamic.casadi always uses the pwm motor model and the Pacejka tires
    # (dynamic.py:214-218): the NLP-form look-ahead ignores input_acc / approx
    for flags in ({"input_acc": True}, {"approx": True}):
        with ModelBank(p, device=0, **flags) as b2:
            r2 = b2.lookahead(x0, U, xref, np.zeros(2), Ts=TS, integrator="euler_nlp", return_costs=True)
        np.testing.assert_array_equal(r2["costs"], r["costs"], err_msg=str(flags))
    # RK6 reference: the oracle's scalar odeintRK6 restatement per model (first 20 models)
    for n in range(20):
        v = O.Vehicle.from_params(O.orca_params(), **{k: p[i, n] for i, k in enumerate(O.BANK_ORDER)})
        for c in range(C):
            xs, _ = O.sim_continuous(v, x0b, U[c].T, np.arange(H + 1) * TS)
            cc = O.mpc_cost(xs.T[:, None, :], U[c:c + 1], xref, np.zeros(2), Q, R, P)[0]
            np.testing.assert_allclose(r6["costs"][n, c], cc, rtol=RTOL_ROLL)


# ----------------------------------------------------------------- fused tick + merge
def test_plan_fused_tick_vs_oracle(nat):
    from llampc.mpc import ModelBank, generate_bank, plan
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, W, K, H, C = 2000, 10, 10, 20, 8
    p = generate_bank(N, seed=0)
    win = O.LookbackWindow(N, W, K)
    rng = np.random.RandomState(2)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    with ModelBank(p, W=W, device=0) as b:
        for t in range(1, W + 4):
            U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
            U[1:] += rng.randn(C - 1, H, 2) * [0.05, 0.02]
            xref = s[:2, t:t + H + 1] + 0.01
            res = plan(b, s[:, t], u[:, t - 1], s[:, t - 1], xref, U, uprev=u[:, t - 1], Ts=TS, K=K,
                       current_model=3, return_errors=True, return_window_mean=True, return_costs=True)
            e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, t - 1], u[:, t - 1], TS), s[:, t])
            win.push(e)
            close(res.lookback_err, e, RTOL_STEP)
            traj = O.rollout_rk4(shared(), tuple(p), s[:, t], U, TS)
            cref = O.mpc_cost(traj, U, xref, u[:, t - 1], Q, R, P).reshape(N, C)
            close(res.costs, cref, RTOL_ROLL)
            sel = win.current if win.count >= W else 3
            assert res.best_model == sel
            assert res.best_cand == int(np.argmin(cref[sel]))
            np.testing.assert_array_equal(res.u_seq, U[res.best_cand].T)
            if win.count >= W:
                np.testing.assert_array_equal(res.topk, win.best_k)
                np.testing.assert_array_equal(res.topk_Df, p[2][win.best_k])
                np.testing.assert_array_equal(res.topk_Dr, p[5][win.best_k])
                np.testing.assert_array_equal(res.raw.topk_cand[:K], np.argmin(cref[win.best_k], axis=1))
            assert res.global_best[0] * C + res.global_best[1] == int(np.argmin(cref.ravel()))


@pytest.mark.parametrize("G", [1, 4, 8, 32])
def test_merge_device_equals_host_and_unsharded(nat, G):
    """Shard a bank G ways on one GPU (G up to the merge's 32): device merge == host merge
    == unsharded tick."""
    import ctypes
    import torch
    from llampc.mpc import ModelBank, generate_bank, shard_range
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, W, H, C = 3000, 3, 20, 4
    p = generate_bank(N, seed=9)
    U = np.repeat(u[:, 5:5 + H].T[None], C, axis=0)
    U[:, :, 1] += np.linspace(-0.02, 0.02, C)[:, None]
    xref = s[:2, 5:5 + H + 1]
    banks = [ModelBank(p[:, lo:hi], W=W, device=0, global_offset=lo)
             for lo, hi in (shard_range(N, g, G) for g in range(G))]
    full = ModelBank(p, W=W, device=0)
    try:
        for t in range(1, W + 2):
            outs = [b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1], K=10)[0] for b in banks]
            ref = full.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1], K=10)[0]
            host = nat.merge(outs)
            raw = b"".join(ctypes.string_at(ctypes.addressof(o), nat.PLAN_OUT_BYTES) for o in outs)
            dparts = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
            dm = torch.empty(nat.PLAN_OUT_BYTES, dtype=torch.uint8, device="cuda")
            nat.check(nat.load().llampc_merge_device(dparts.data_ptr(), G, 0, dm.data_ptr(), 0, None))
            torch.cuda.synchronize()
            dev = nat.PlanOut.from_buffer_copy(dm.cpu().numpy().tobytes())
            for o in (host, dev):
                a, r = nat.plan_out_to_dict(o), nat.plan_out_to_dict(ref)
                for k in ("window_count", "window_full", "lb_best", "sel_model", "sel_cand",
                          "la_best_model", "la_best_cand", "n_nonfinite"):
                    assert a[k] == r[k], (k, a[k], r[k])
                for k in ("topk", "topk_cand"):
                    np.testing.assert_array_equal(a[k], r[k])
                for k in ("topk_val", "topk_Df", "topk_Dr", "topk_cost"):
                    np.testing.assert_array_equal(a[k], r[k])
    finally:
        for b in banks + [full]:
            b.close()


# ----------------------------------------------------------------- closed loop + full size
def test_closed_loop_lookback_and_mu_vs_golden(nat):
    """The reference tick logic (rt.py:269-366) over 60 ticks: model selection, top-K and
    mu-hat sequences through ModelBank + MuEstimator."""
    from llampc.mpc import ModelBank, MuEstimator
    g = golden("closed_loop.npz")
    p = O.orca_params()
    x, u = g["x"], g["u"]
    bank = g["bank"]
    mu = MuEstimator(mass=p["mass"], lf=p["lf"], lr=p["lr"])
    cur, topk = 0, None
    with ModelBank(bank, W=10, device=0) as b:
        for idt in range(u.shape[1]):
            if idt <= 10:
                mu.warmup()
            else:
                mu.update(bank[5][topk], bank[2][topk])
                np.testing.assert_allclose(mu.mu_pred, g["mu_pred"][idt], rtol=1e-12)
            np.testing.assert_allclose(mu.mu_logged[-1], g["mu_logged"][idt], rtol=1e-12)
            if idt > 0:
                r = b.lookback(x[idt], u[:, idt], x[idt + 1], Ts=TS, K=10)
                if r["full"]:
                    cur, topk = r["best"], r["topk"]
                    np.testing.assert_array_equal(topk, g["topk"][idt])
            assert cur == g["current"][idt]


@pytest.mark.parametrize("N", [300, 6])
def test_llampc_controller_closed_loop_vs_oracle(nat, monkeypatch, N):
    """mode="host" (the device mode: tests/test_ctl_gpu.py).  The LLAMPC tick loop in closed loop with an RK6 plant (friction dropping): while the
    window fills (tick <= W) every tick plans with the NOMINAL model (the reference's
    nlp_initial, rt.py:207, 300-301), afterwards with the look-back's selection
    (nlp_bank[current_model_idx], rt.py:303).  Each tick's chosen candidate and cost equal
    the oracle's (rollout_rk4 + mpc_cost + feasibility on the same xref and candidates);
    mu-hat follows the oracle window's top-K.  N = 6 < K checks that the -1 padding of
    top-K never enters mu-hat (argsort()[:K] has n entries, rt.py:360)."""
    import llampc.mpc.controller as ctl_mod
    from llampc.mpc import LLAMPC, ModelBank, generate_bank
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    p = O.orca_params()
    C, H, W, K = 8, 20, 4, 10
    bank_p = generate_bank(N, seed=21)
    nominal = np.array([[p[k]] for k in O.BANK_ORDER])
    xrefs, Us = [], []
    cs = ctl_mod.ConstantSpeed
    monkeypatch.setattr(ctl_mod, "ConstantSpeed", lambda *a, **k: (lambda r: (xrefs.append(r[0]), r)[1])(cs(*a, **k)))
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    plant = O.Vehicle.from_params(p)
    win = O.LookbackWindow(N, W, K)
    x = d["states"][:, 0].copy()
    cur = 0
    with ModelBank(bank_p, W=W, device=0) as b, LLAMPC(b, ETHZ('optimal', True), H=H, C=C, K=K, mode="host") as ctl:
        gen = ctl.gen
        ctl.gen = lambda prev, up: (lambda U: (Us.append(U), U)[1])(gen(prev, up))
        x_prev = u_prev = None
        for t in range(W + 6):
            l0 = b.launches + ctl.nominal_bank.launches
            res = ctl.tick(x)
            # after the warm-up one fused launch per tick (rt.py:300-366 in one plan kernel);
            # while the window fills, the bank's look-back plus the nominal look-ahead
            assert b.launches + ctl.nominal_bank.launches - l0 == (1 if (t > W or t < 2) else 2), t
            if t >= 2:                                   # oracle look-back on (x_{t-1}, u_{t-1}) -> x_t
                pred = O.evaluate_models_vectorized(shared(), tuple(bank_p), x_prev, u_prev, TS)
                win.push(O.lookback_errors(pred, x))
                if win.count >= W:
                    cur = win.current
                    kk = min(N, K)
                    np.testing.assert_array_equal(res.topk, win.best_k[:kk])
            assert res.nominal == (t <= W)
            cols = nominal if t <= W else bank_p[:, cur:cur + 1]
            U, xref = Us[-1], xrefs[-1]
            uprev = np.zeros(2) if u_prev is None else u_prev
            cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(cols), x, U, TS), U, xref, uprev, Q, R, P)
            ok = O.candidates_feasible(U, uprev, [-0.1, -0.35], [1.0, 0.35], 5.0, TS)
            cref = np.where(ok & ~np.isnan(cref), cref, np.inf)
            assert res.best_cand == int(np.argmin(cref)), (t, res.best_cand, cref)
            np.testing.assert_allclose(res.cost, cref[res.best_cand], rtol=RTOL_ROLL)
            if t > W:
                assert res.best_model == cur
                np.testing.assert_allclose(ctl.mu.dr_hist[-1], np.mean(bank_p[5][win.best_k[:min(N, K)]]), rtol=1e-12)
            u = res.u_seq[:, 0]
            np.testing.assert_array_equal(u, U[res.best_cand, 0])
            plant.Df *= 1 - 1 / 260.0
            plant.Dr *= 1 - 1 / 260.0
            xn, _ = O.sim_continuous(plant, x, u.reshape(2, 1), [0, TS])
            x_prev, u_prev, x = x, u.copy(), xn[:, -1]


@pytest.mark.parametrize("N,H,track", [(10000, 20, "ETHZ"), (80000, 20, "ETHZ")])
def test_baseline_sizes_properties(nat, N, H, track):
    """BASELINE.json sizes on the DYN recording (ETHZ: configs 2 and 4's track): errors/costs vs
    the oracle on every model (numpy handles these sizes in seconds), selection consistent with
    the returned arrays, top-K sorted.  Config 3 (ETHZMobil) runs on its own synthetic Mobil
    states in tests/test_configs_gpu.py."""
    from llampc.mpc import ModelBank, generate_bank, plan
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ, ETHZMobil
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True) if track == "ETHZ" else ETHZMobil('optimal', True)
    p = generate_bank(N, seed=0 if track == "ETHZ" else 1)
    W, K = 10, 10
    with ModelBank(p, W=W, device=0) as b:
        for t in range(1, W + 2):
            x_t = s[:, t]
            xref, _, _ = ConstantSpeed(x_t[:2], x_t[3], tr, H, TS, 0)
            U = np.repeat(np.tile(u[:, t], (H, 1))[None], 1, axis=0)
            res = plan(b, x_t, u[:, t - 1], s[:, t - 1], xref, U, Ts=TS, K=K, return_errors=True,
                       return_window_mean=True, return_costs=True)
        e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, W], u[:, W], TS), s[:, W + 1])
        close(res.lookback_err, e, RTOL_STEP)
        wm = res.window_mean
        assert res.best_model == int(np.argmin(wm))
        assert np.all(np.diff(wm[res.topk]) >= 0) and set(res.topk) == set(np.argsort(wm, kind="stable")[:K])
        traj = O.rollout_rk4(shared(), tuple(p), s[:, W + 1], U, TS)
        cref = O.mpc_cost(traj, U, xref, u[:, W], np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2)))
        close(res.costs.ravel(), cref, RTOL_ROLL)
        assert res.global_best[0] == int(np.argmin(np.where(np.isnan(cref), np.inf, cref)))


def test_c64_work_queue_full_size_vs_oracle(nat):
    """The bench's C = 64 throughput shape at full size — N = 10^4, C = 64, H = 20, where
    launch_plan takes the 8-wave work-queue layout (10^4 units >= 4 per wave slot of 255
    CUs) — against the oracle: all 640,000 (model, candidate) costs at 1e-6, the selected and
    top-K models' best candidates and the global argmin exact, the look-back selection exact."""
    from llampc.mpc import CandidateGenerator, ModelBank, generate_bank, plan
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    N, C, H, W, K = 10000, 64, 20, 10, 10
    p = generate_bank(N, seed=0)
    gen = CandidateGenerator(C, H, seed=2)
    win = O.LookbackWindow(N, W, K)
    with ModelBank(p, W=W, device=0) as b:
        for t in range(1, W + 2):
            x_t = s[:, t]
            xref, _, _ = ConstantSpeed(x_t[:2], x_t[3], tr, H, TS, 0, curr_mu=0.9, scale=0.9)
            U = gen(None, u[:, t])
            res = plan(b, x_t, u[:, t - 1], s[:, t - 1], xref, U, Ts=TS, K=K, return_costs=(t == W + 1))
            win.push(O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), s[:, t - 1], u[:, t - 1], TS),
                                       x_t))
    assert res.window_full and res.best_model == win.current
    np.testing.assert_array_equal(res.topk, win.best_k)
    traj = O.rollout_rk4(shared(), tuple(p), s[:, W + 1], U, TS)
    cref = O.mpc_cost(traj, U, xref, u[:, W], np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2)))
    del traj
    close(res.costs.ravel(), cref, RTOL_ROLL)
    cm = np.where(np.isnan(cref), np.inf, cref).reshape(N, C)
    assert res.best_cand == int(np.argmin(cm[win.current]))
    np.testing.assert_array_equal(res.raw.topk_cand[:K], [int(np.argmin(cm[m])) for m in win.best_k])
    g = int(np.argmin(cm.ravel()))
    assert res.global_best[:2] == (g // C, g % C)


# ----------------------------------------------------------------- model transcendentals
def _math(nat, fn, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty_like(a)
    nat.check(nat.load().llampc_math_batch(fn, a.ctypes.data, None if bb is None else bb.ctypes.data,
                                           a.size, out.ctypes.data, 0))
    return out


def _ulp(got, want):
    fin = np.isfinite(want)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(got[~fin], want[~fin])
    return np.max(np.abs(got[fin] - want[fin]) / np.spacing(np.maximum(np.abs(want[fin]), 1e-300)))


def test_fast_transcendentals_ulp_vs_libm(nat):
    """csrc/fastmath.hpp vs NumPy (libm): <= 4 ulp over the model's argument ranges and
    wide random ranges; C99 special cases exactly."""
    rng = np.random.RandomState(0)
    n = 1 << 20
    y = np.concatenate([rng.uniform(-3, 3, n), rng.standard_cauchy(n), [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 5.0, 0.0]])
    x = np.concatenate([rng.uniform(0, 4, n), np.abs(rng.standard_cauchy(n)), [0.0, 0.0, 0.0, 0.0, np.inf, np.inf, 1.0, np.inf, 3.0]])
    assert _ulp(_math(nat, 0, y, x), np.arctan2(y, x)) <= 4
    z = np.concatenate([rng.uniform(-2, 2, n), rng.standard_cauchy(n) * 10, [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e300, 1e-300]])
    assert _ulp(_math(nat, 1, z), np.arctan(z)) <= 4
    a = np.concatenate([rng.uniform(-4, 4, n), rng.uniform(-300, 300, n), rng.uniform(-3e6, 3e6, 1000),
                        [0.0, -0.0, np.pi / 2, np.pi, 1e-300, np.inf, -np.inf, np.nan, 1e20]])
    s, c = _math(nat, 2, a), _math(nat, 3, a)
    # absolute error near the zeros of sin/cos (reduction), relative elsewhere
    for got, want in ((s, np.sin(a)), (c, np.cos(a))):
        fin = np.isfinite(want)
        np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
        err = np.abs(got[fin] - want[fin])
        assert np.all(err <= 4 * np.spacing(np.maximum(np.abs(want[fin]), 1e-16))), err.max()


def test_fast_cores_ulp_on_domain(nat):
    """The branch-free cores of the rollout stage (fastmath.hpp, math fn 4-9) on their
    domains vs NumPy (libm): atan2/atan <= 4 ulp, sin_wide <= 4 ulp for |a| <= 2 and
    <= 2^-49 absolute up to 3 (no reduction: a + a s P(s) cancels as sin(3) ~ 0.14),
    sincos <= 4 ulp / absolute near zeros, a / 6 bit-exact."""
    rng = np.random.RandomState(1)
    n = 1 << 20
    y = np.concatenate([rng.uniform(-3, 3, n), rng.standard_cauchy(n), [0.0, -0.0, 1.0, -1.0, 1e-300, 5.0]])
    x = np.concatenate([rng.uniform(0, 4, n), np.abs(rng.standard_cauchy(n)), [1.0, 1.0, 0.0, 0.0, 0.0, 3.0]])
    ok = (np.abs(y) + x >= 2.0 ** -1000) & (np.abs(y) + x <= 2.0 ** 1000)
    assert _ulp(_math(nat, 4, y[ok], x[ok]), np.arctan2(y[ok], x[ok])) <= 4
    z = np.concatenate([rng.uniform(-2, 2, n), rng.standard_cauchy(n) * 10, [0.0, -0.0, 1.0, -1.0, 1e300, -1e-300]])
    assert _ulp(_math(nat, 5, z), np.arctan(z)) <= 4
    a = rng.uniform(-2, 2, n)
    assert _ulp(_math(nat, 6, a), np.sin(a)) <= 4
    a = np.concatenate([rng.uniform(-3, 3, n), [3.0, -3.0, 0.0, -0.0, 1e-300]])
    err = np.abs(_math(nat, 6, a) - np.sin(a))
    assert np.all(err <= 4 * np.spacing(np.abs(np.sin(a))) + 2.0 ** -49), err.max()
    a = np.concatenate([rng.uniform(-4, 4, n), rng.uniform(-300, 300, n), rng.uniform(-1.6e6, 1.6e6, 1000),
                        [0.0, -0.0, np.pi / 2, np.pi, 1e-300]])
    for fn, want in ((7, np.sin(a)), (8, np.cos(a))):
        err = np.abs(_math(nat, fn, a) - want)
        assert np.all(err <= 4 * np.spacing(np.maximum(np.abs(want), 1e-16))), err.max()
    v = np.concatenate([rng.standard_normal(n) * 10.0 ** rng.randint(-300, 300, n), [0.0, -0.0, 6.0, 1e308, 5e-324]])
    np.testing.assert_array_equal(_math(nat, 9, v), v / 6.0)


def test_lean_cores_accuracy_on_domain(nat):
    """The look-ahead's lean cores (math fn 10-12: 8-term atan and sin_wide, division without
    its residual step) on the same domains vs NumPy: atan2 / atan within 2^11 ulp (~4.5e-13
    relative; the fit's own error is 1.1e-13), sin_wide within 2^12 ulp for |a| <= 2 and 2^-40
    absolute up to 3 (the fit: 2.6e-13)."""
    rng = np.random.RandomState(2)
    n = 1 << 20
    y = np.concatenate([rng.uniform(-3, 3, n), rng.standard_cauchy(n), [0.0, -0.0, 1.0, -1.0, 1e-300, 5.0]])
    x = np.concatenate([rng.uniform(0, 4, n), np.abs(rng.standard_cauchy(n)), [1.0, 1.0, 0.0, 0.0, 0.0, 3.0]])
    ok = (np.abs(y) + x >= 2.0 ** -1000) & (np.abs(y) + x <= 2.0 ** 1000)
    u_a2 = _ulp(_math(nat, 10, y[ok], x[ok]), np.arctan2(y[ok], x[ok]))
    z = np.concatenate([rng.uniform(-2, 2, n), rng.standard_cauchy(n) * 10, [0.0, -0.0, 1.0, -1.0, 1e300, -1e-300]])
    u_a = _ulp(_math(nat, 11, z), np.arctan(z))
    a = rng.uniform(-2, 2, n)
    u_s = _ulp(_math(nat, 12, a), np.sin(a))
    print(f"lean cores: atan2 {u_a2:.1f} ulp, atan {u_a:.1f} ulp, sin_wide |a|<=2 {u_s:.1f} ulp")
    assert u_a2 <= 2 ** 11 and u_a <= 2 ** 11 and u_s <= 2 ** 12
    a = np.concatenate([rng.uniform(-3, 3, n), [3.0, -3.0, 0.0, -0.0, 1e-300]])
    err = np.abs(_math(nat, 12, a) - np.sin(a))
    assert np.all(err <= 16 * np.spacing(np.abs(np.sin(a))) + 2.0 ** -40), err.max()
    # the paired cores of the LPM-1 look-ahead lane (math fn 13/14: front and rear division
    # through one reciprocal, partner = element n-1-i) on their domain (Dom::ok_paired:
    # atan2 divisors max(|y|, x) in [2^-500, 2^499], atan divisor products <= 2^499)
    ok2 = ok & (np.maximum(np.abs(y), x) >= 2.0 ** -500) & (np.maximum(np.abs(y), x) <= 2.0 ** 499)
    yy, xx = y[ok2], x[ok2]
    part = np.maximum(np.abs(yy[::-1]), xx) >= 2.0 ** -500
    got = _math(nat, 13, yy, xx)
    u_p2 = _ulp(got[part], np.arctan2(yy, xx)[part])
    zz = z[np.abs(z) <= 2.0 ** 240]
    u_p = _ulp(_math(nat, 14, zz), np.arctan(zz))
    print(f"paired cores: atan2 {u_p2:.1f} ulp, atan {u_p:.1f} ulp")
    assert u_p2 <= 2 ** 11 and u_p <= 2 ** 11


def test_lookahead_out_of_domain_fallback(nat):
    """Rollouts whose operands leave the fast cores' domains take the general evaluation
    (dyn.hpp rhs_fast): models with |C| > 1.9, a yaw beyond 2^20 pi/2, a standing start
    (|y| + |vx| = 0), and a linear-tire bank — all against the oracle, in waves that mix
    fast and fallback lanes (LPM = 1, the lane-pair split and the quad with folded sincos)."""
    from llampc.mpc import ModelBank, generate_bank
    N, C, H = 640, 3, 12
    p = generate_bank(N, seed=11)
    p[1, 5::37] = 2.6          # Cf beyond the sin_wide bound
    p[4, 9::41] = -2.2         # Cr
    rng = np.random.RandomState(3)
    U = np.stack([rng.uniform(0.1, 0.9, (C, H)), rng.uniform(-0.3, 0.3, (C, H))], axis=-1)
    xref = np.vstack([np.linspace(0, 0.5, H + 1), np.linspace(0, -0.2, H + 1)])
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    cases = [np.array([0.2, 0.1, -0.7, 1.5, 0.02, 0.3]),
             np.array([0.2, 0.1, 3.0e6, 1.5, 0.02, 0.3]),           # huge yaw: sincos fallback
             np.array([0.0, 0.0, 0.4, 0.0, 0.0, 0.0]),              # standing start
             np.array([0.2, 0.1, -0.7, 2.5, 0.1, 40.0])]            # spinning start
    for x0 in cases:
        with np.errstate(all="ignore"):
            traj = O.rollout_rk4(shared(), tuple(p), x0, U, TS)
            cref = O.mpc_cost(traj, U, xref, np.zeros(2), Q, R, P)
        for lpm in ("1", "2", "4"):
            os.environ["LLAMPC_LPM"] = lpm
            try:
                with ModelBank(p, device=0) as b:
                    r = b.lookahead(x0, U, xref, np.zeros(2), Ts=TS, return_costs=True)
            finally:
                del os.environ["LLAMPC_LPM"]
            close(r["costs"].ravel(), cref, RTOL_ROLL)
    # linear tires (Dynamic(approx=True), dynamic.py:126-136): every lane takes the fallback
    x0 = cases[0]
    with ModelBank(p, device=0, approx=True) as b:
        r = b.lookahead(x0, U, xref, np.zeros(2), Ts=TS, return_costs=True)
    traj = O.rollout_rk4(shared(), tuple(p), x0, U, TS, approx=True)
    close(r["costs"].ravel(), O.mpc_cost(traj, U, xref, np.zeros(2), Q, R, P), RTOL_ROLL)


def test_plan_device_refused_while_async_outstanding(nat):
    """llampc_plan_device returns LLAMPC_E_STATE while an llampc_plan_async tick is
    outstanding on the bank (both would share its completion state and window), and runs
    once llampc_plan_wait has returned."""
    import ctypes
    import torch
    from llampc import _native
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    H = 20
    U = np.tile(u[:, 1], (H, 1))[None]
    xref = s[:2, 1:H + 2]
    sb = ShardedBank(generate_bank(500, seed=2), 0, 1, 0, W=3)
    try:
        staged = sb.stage(s[:, 0], u[:, 0], s[:, 1], U, xref, u[:, 0])
        pin = sb.make_plan_in(staged["pack"], 1, H, K=5)
        lib = _native.load()
        sb.bank.plan_async(s[:, 0], u[:, 0], s[:, 1], U, xref, u[:, 0], K=5)
        rc = lib.llampc_plan_device(sb.bank.handle, ctypes.byref(pin), sb.d_local.data_ptr(), None, None, None,
                                    sb.stream.cuda_stream)
        assert rc == _native.E_STATE, rc
        out = sb.bank.plan_wait()
        assert out.status == 0
        sb.launch(pin)
        torch.cuda.synchronize()
        assert sb.fetch().best_cand == 0
    finally:
        sb.close()


def test_plan_async_two_banks(nat):
    """llampc_plan_async / llampc_plan_wait: two banks (two tracks) in flight together give
    the same records as the blocking llampc_plan; a second async tick on a busy bank and a
    wait without a tick are refused (LLAMPC_E_STATE)."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    H, W = 20, 3
    banks = [ModelBank(generate_bank(700, seed=k), W=W, device=0) for k in (0, 1)]
    refs = [ModelBank(generate_bank(700, seed=k), W=W, device=0) for k in (0, 1)]
    try:
        for t in range(1, W + 3):
            U = u[:, t:t + H].T[None]
            xref = s[:2, t:t + H + 1] + 0.01 * np.arange(2)[:, None]
            args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
            for b in banks:
                b.plan_async(*args, K=5, current_model=2)
            with pytest.raises(RuntimeError):
                banks[0].plan_async(*args, K=5)
            outs = [b.plan_wait() for b in banks]
            for o, r in zip(outs, refs):
                want = r.plan_raw(*args, K=5, current_model=2)[0]
                a, w = _native.plan_out_to_dict(o), _native.plan_out_to_dict(want)
                for k in a:
                    if isinstance(a[k], np.ndarray):
                        np.testing.assert_array_equal(a[k], w[k])
                    else:
                        assert a[k] == w[k] or (a[k] != a[k] and w[k] != w[k]), k
        with pytest.raises(RuntimeError):
            banks[0].plan_wait()
    finally:
        for b in banks + refs:
            b.close()


def _mobil_states(T, u):
    """A physical ETHZMobil trajectory (no recorded one exists): the oracle's RK6 plant from
    the track's start pose at 1 m/s, driven by the recorded controls, friction dropping by
    x21/22 for 9 ticks after tick 2 (the sudden scenario of config 3, rt.py:132-141)."""
    from llampc.tracks import ETHZMobil
    tr = ETHZMobil('optimal', True)
    p = O.orca_params()
    v = O.Vehicle.from_params(p)
    xs = [np.array([tr.x_init, tr.y_init, tr.psi_init, 1.0, 0.0, 0.0])]
    for k in range(T):
        if 2 <= k < 11:
            v.Df -= v.Df / 22.
            v.Dr -= v.Dr / 22.
        xn, _ = O.sim_continuous(v, xs[-1], u[:, k].reshape(2, 1), [0, TS])
        xs.append(xn[:, -1])
    return np.array(xs).T


def test_config5_concurrent_tracks_vs_oracle(nat):
    """BASELINE config 5's workload on one GPU: an ETHZ bank (seed 0) and an ETHZMobil bank
    (seed 1) of 10^4 models each, H = 40, ticked CONCURRENTLY every control step through
    llampc_plan_async / llampc_plan_wait (two streams in flight), over W + 2 ticks, against
    the oracle (rt.py:347-366 look-back + H x _integrate_batch + nmpc.py cost per track):
    selection, top-K and the look-ahead argmin exact; every cost in the record (selected
    model's, top-K models', global best) within 1e-6; top-K Df/Dr bitwise."""
    from llampc import _native
    from llampc.mpc import ConstantSpeed, ModelBank, generate_bank
    from llampc.tracks import ETHZ, ETHZMobil
    d = golden("dyn_slice.npz")
    u = d["inputs"]
    N, H, W, K = 10000, 40, 10, 10
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    T = W + 2
    tracks = {"ETHZ": (ETHZ('optimal', True), d["states"], 0), "ETHZMobil": (ETHZMobil('optimal', True),
                                                                              _mobil_states(T + 1, u), 1)}
    banks, wins, params, proj = {}, {}, {}, {}
    try:
        for name, (tr, s, seed) in tracks.items():
            params[name] = generate_bank(N, seed=seed)
            banks[name] = ModelBank(params[name], W=W, device=0)
            wins[name] = O.LookbackWindow(N, W, K)
            proj[name] = 0
        for t in range(1, T + 1):
            args = {}
            for name, (tr, s, _) in tracks.items():
                xref, proj[name], _ = ConstantSpeed(s[:2, t], s[3, t], tr, H, TS, proj[name], scale=0.9)
                U = u[:, t:t + H].T[None].copy()
                args[name] = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
            for name, b in banks.items():                 # both in flight before either wait
                b.plan_async(*args[name], K=K, current_model=3)
            outs = {name: _native.plan_out_to_dict(b.plan_wait()) for name, b in banks.items()}
            for name, (tr, s, _) in tracks.items():
                p, win, o = params[name], wins[name], outs[name]
                x_prev, u_prev, x_now, U, xref, uprev = args[name]
                win.push(O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), x_prev, u_prev, TS), x_now))
                cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), x_now, U, TS), U, xref, uprev, Q, R, P)
                cinf = np.where(np.isnan(cref), np.inf, cref)
                assert o["status"] == 0
                assert o["window_full"] == (win.count >= W)
                sel = win.current if win.count >= W else 3
                assert o["sel_model"] == sel, (name, t)
                if np.isfinite(cref[sel]):
                    assert o["sel_cand"] == 0
                np.testing.assert_allclose(o["sel_cost"], cref[sel], rtol=RTOL_ROLL)
                j = int(np.argmin(cinf))
                assert (o["la_best_model"], o["la_best_cand"]) == (j, 0), (name, t)
                np.testing.assert_allclose(o["la_best_cost"], cref[j], rtol=RTOL_ROLL)
                if win.count >= W:
                    assert o["lb_best"] == win.current
                    np.testing.assert_array_equal(o["topk"][:K], win.best_k)
                    np.testing.assert_array_equal(o["topk_Df"][:K], p[2][win.best_k])
                    np.testing.assert_array_equal(o["topk_Dr"][:K], p[5][win.best_k])
                    np.testing.assert_allclose(o["topk_val"][:K], win.avg[win.best_k], rtol=RTOL_STEP)
                    np.testing.assert_allclose(o["topk_cost"][:K], cref[win.best_k], rtol=RTOL_ROLL)
                assert o["n_nonfinite"] == int(np.count_nonzero(~np.isfinite(cref)))
    finally:
        for b in banks.values():
            b.close()


def test_polled_completion_equals_ticket_completion(nat):
    """The polled in-launch completion (look-ahead blocks publish tagged records, the
    look-back winner polls them) gives records identical to the ticket + last-block path
    (LLAMPC_NO_POLL=1), tick after tick (tags advance per launch; stale words never pass),
    at C = 1 (LPM 4), C = 3 and C = 64, with the window filling and full; status stays 0."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    H, W = 20, 3
    rng = np.random.RandomState(9)
    for N, C in ((5000, 1), (1200, 3), (300, 64)):
        a_bank = ModelBank(generate_bank(N, seed=3), W=W, device=0)
        b_bank = ModelBank(generate_bank(N, seed=3), W=W, device=0)
        try:
            for t in range(1, W + 4):
                U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
                U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
                xref = s[:2, t:t + H + 1] + 0.01 * np.arange(2)[:, None]
                args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
                o = a_bank.plan_raw(*args, K=5, current_model=1)[0]
                os.environ["LLAMPC_NO_POLL"] = "1"
                try:
                    w = b_bank.plan_raw(*args, K=5, current_model=1)[0]
                finally:
                    del os.environ["LLAMPC_NO_POLL"]
                A, B = _native.plan_out_to_dict(o), _native.plan_out_to_dict(w)
                assert A["status"] == 0 and B["status"] == 0
                for k in A:
                    if isinstance(A[k], np.ndarray):
                        np.testing.assert_array_equal(A[k], B[k], err_msg=k)
                    else:
                        assert A[k] == B[k] or (A[k] != A[k] and B[k] != B[k]), (k, A[k], B[k])
        finally:
            a_bank.close()
            b_bank.close()


def test_bank_concurrency_lane_split_equals_default(nat):
    """llampc_bank_set_concurrency(2) (BASELINE config 5: two tracks share the chip) sizes the
    look-ahead for half the SIMDs — at N = 10^4, H = 40, C = 1 the lane pair (LPM 2) instead of
    the quad — with the same selections and top-K as the default bank and costs within 1e-9,
    tick after tick; 0 and 65 are rejected."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, H, W = 10000, 40, 3
    a_bank = ModelBank(generate_bank(N, seed=1), W=W, device=0)
    b_bank = ModelBank(generate_bank(N, seed=1), W=W, device=0)
    try:
        b_bank.set_concurrency(2)
        for bad in (0, 65):
            with pytest.raises(_native.NativeError):
                b_bank.set_concurrency(bad)
        for t in range(1, W + 3):
            U = u[:, t:t + H].T[None].copy()
            xref = s[:2, t:t + H + 1] + 0.01
            args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
            A = _native.plan_out_to_dict(a_bank.plan_raw(*args, K=10)[0])
            B = _native.plan_out_to_dict(b_bank.plan_raw(*args, K=10)[0])
            for k in ("window_full", "lb_best", "sel_model", "sel_cand", "la_best_model", "la_best_cand", "n_nonfinite",
                      "status"):
                assert A[k] == B[k], (t, k, A[k], B[k])
            np.testing.assert_array_equal(A["topk"], B["topk"])
            np.testing.assert_array_equal(A["topk_cand"], B["topk_cand"])
            np.testing.assert_allclose(B["sel_cost"], A["sel_cost"], rtol=1e-9)
            np.testing.assert_allclose(B["la_best_cost"], A["la_best_cost"], rtol=1e-9)
    finally:
        a_bank.close()
        b_bank.close()


def test_shared_queue_stream_equals_dedicated(nat, monkeypatch):
    """A bank on a plain stream (LLAMPC_SHARED_QUEUES=1, shared hardware queues) and one on its
    own full-CU-mask stream (the default) tick to identical records."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, H, W = 2000, 20, 3
    a_bank = ModelBank(generate_bank(N, seed=4), W=W, device=0)
    monkeypatch.setenv("LLAMPC_SHARED_QUEUES", "1")
    b_bank = ModelBank(generate_bank(N, seed=4), W=W, device=0)
    monkeypatch.delenv("LLAMPC_SHARED_QUEUES")
    try:
        for t in range(1, W + 3):
            U = np.repeat(u[:, t:t + H].T[None], 3, axis=0)
            U[1:, :, 1] += 0.01
            args = (s[:, t - 1], u[:, t - 1], s[:, t], U, s[:2, t:t + H + 1], u[:, t - 1])
            A = _native.plan_out_to_dict(a_bank.plan_raw(*args, K=5)[0])
            B = _native.plan_out_to_dict(b_bank.plan_raw(*args, K=5)[0])
            for k in A:
                if isinstance(A[k], np.ndarray):
                    np.testing.assert_array_equal(A[k], B[k], err_msg=k)
                else:
                    assert A[k] == B[k] or (A[k] != A[k] and B[k] != B[k]), (k, A[k], B[k])
    finally:
        a_bank.close()
        b_bank.close()


def test_work_queue_layout_equals_static_and_oracle(nat, monkeypatch):
    """The throughput layout (launch_plan's work queue: one look-ahead block per CU, waves
    taking units of models from the bank's counter) at N = 3000, C = 64 (750 static blocks >
    the CUs) and C = 40 (G = 64, ragged candidates), with 4-wave and (forced) 8-wave blocks:
    every record field equal to the static
    block-per-models layout (LLAMPC_NO_WQ=1) tick after tick — polled and ticket completion —
    costs equal to the oracle's at 1e-6, and the counter's base carried correctly across
    ticks, a reset and a second bank."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, H, W = 3000, 20, 3
    rng = np.random.RandomState(13)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    p = generate_bank(N, seed=4)
    for C, waves in ((64, None), (40, None), (64, "8"), (40, "8")):
        if waves:                       # the 8-wave layout (launch_plan picks 4 waves here)
            monkeypatch.setenv("LLAMPC_WQ_WAVES", waves)
        a_bank = ModelBank(p, W=W, device=0)
        b_bank = ModelBank(p, W=W, device=0)
        try:
            for t in range(1, W + 3):
                U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
                U[1:] += rng.uniform(-0.03, 0.03, U[1:].shape)
                U[:, :, 1] = np.clip(U[:, :, 1], -0.35, 0.35)
                xref = s[:2, t:t + H + 1] + 0.01
                args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
                if t == 3:
                    monkeypatch.setenv("LLAMPC_NO_POLL", "1")
                o, _, _, costs = a_bank.plan_raw(*args, K=5, current_model=7, return_costs=(t == 2))
                monkeypatch.setenv("LLAMPC_NO_WQ", "1")
                w = b_bank.plan_raw(*args, K=5, current_model=7)[0]
                monkeypatch.delenv("LLAMPC_NO_WQ")
                monkeypatch.delenv("LLAMPC_NO_POLL", raising=False)
                _same_records(o, w)
                if costs is not None:
                    cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), s[:, t], U, TS), U, xref, u[:, t - 1], Q, R, P)
                    close(costs.ravel(), cref, RTOL_ROLL)
                    assert (o.la_best_model, o.la_best_cand) == divmod(int(np.argmin(np.where(np.isnan(cref), np.inf, cref))), C)
            a_bank.reset()
            b_bank.reset()
            o = a_bank.plan_raw(*args, K=5, current_model=7)[0]
            monkeypatch.setenv("LLAMPC_NO_WQ", "1")
            w = b_bank.plan_raw(*args, K=5, current_model=7)[0]
            monkeypatch.delenv("LLAMPC_NO_WQ")
            _same_records(o, w)
        finally:
            a_bank.close()
            b_bank.close()


@pytest.mark.parametrize("N,C", [(6000, 20), (10000, 7)])
def test_work_queue_several_models_per_wave(nat, monkeypatch, N, C):
    """The work queue with units of several models per wave (G = 32: two models of 20
    candidates; G = 8: eight models of 7 — lanes of one wave then read different Pacejka rows
    and reduce over G-lane groups): records equal to the static layout, polled and ticket
    completion, costs and the look-ahead argmin equal to the oracle's."""
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    H, W = 20, 2
    rng = np.random.RandomState(17)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    p = generate_bank(N, seed=5)
    a_bank = ModelBank(p, W=W, device=0)
    b_bank = ModelBank(p, W=W, device=0)
    try:
        for t in range(1, W + 2):
            U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
            U[1:] += rng.uniform(-0.03, 0.03, U[1:].shape)
            U[:, :, 1] = np.clip(U[:, :, 1], -0.35, 0.35)
            xref = s[:2, t:t + H + 1] + 0.01
            args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
            if t == W + 1:
                monkeypatch.setenv("LLAMPC_NO_POLL", "1")
            o, _, _, costs = a_bank.plan_raw(*args, K=5, current_model=3, return_costs=(t == W))
            monkeypatch.setenv("LLAMPC_NO_WQ", "1")
            w = b_bank.plan_raw(*args, K=5, current_model=3)[0]
            monkeypatch.delenv("LLAMPC_NO_WQ")
            monkeypatch.delenv("LLAMPC_NO_POLL", raising=False)
            _same_records(o, w)
            if costs is not None:
                cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), s[:, t], U, TS), U, xref, u[:, t - 1], Q, R, P)
                close(costs.ravel(), cref, RTOL_ROLL)
                assert (o.la_best_model, o.la_best_cand) == divmod(int(np.argmin(np.where(np.isnan(cref), np.inf, cref))), C)
    finally:
        a_bank.close()
        b_bank.close()


def test_poll_bound_scales_with_launch_work(nat, monkeypatch):
    """The polled completion's wait bound grows with the launch's rollout steps
    (poll_bound_ticks: floor + 40 ns per step), so a valid long look-ahead is never reported
    as a timeout.  With the floor cut to 1 ms (LLAMPC_POLL_BOUND_S) a ~10 ms tick (N=1e5,
    C=64, H=40) still returns status 0 through the default per-step term; with the per-step
    term off as well it reports LLAMPC_STATUS_POLL_TIMEOUT — the bound is live — and the
    bank keeps working afterwards."""
    from llampc import _native
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, C, H = 100_000, 64, 40
    rng = np.random.RandomState(11)
    U = np.repeat(u[:, 1:1 + H].T[None], C, axis=0)
    U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
    xref = s[:2, 1:H + 2]
    args = (s[:, 0], u[:, 0], s[:, 1], U, xref, u[:, 0])
    with ModelBank(generate_bank(N, seed=12), W=3, device=0) as b:
        ref = b.plan_raw(*args, K=5, current_model=1)[0]
        monkeypatch.setenv("LLAMPC_POLL_BOUND_S", "0.001")
        b.reset()
        o = b.plan_raw(*args, K=5, current_model=1)[0]
        _same_records(o, ref)
        monkeypatch.setenv("LLAMPC_POLL_STEP_NS", "0")
        b.reset()
        with pytest.raises(_native.NativeError, match="status 1"):
            b.plan_raw(*args, K=5, current_model=1)
        monkeypatch.delenv("LLAMPC_POLL_BOUND_S")
        monkeypatch.delenv("LLAMPC_POLL_STEP_NS")
        b.reset()
        _same_records(b.plan_raw(*args, K=5, current_model=1)[0], ref)


def _same_records(o, w):
    from llampc import _native
    A, B = _native.plan_out_to_dict(o), _native.plan_out_to_dict(w)
    assert A["status"] == 0 and B["status"] == 0
    for k in A:
        if isinstance(A[k], np.ndarray):
            np.testing.assert_array_equal(A[k], B[k], err_msg=k)
        else:
            assert A[k] == B[k] or (A[k] != A[k] and B[k] != B[k]), (k, A[k], B[k])


def test_host_completion_equals_copy_completion(nat):
    """Host completion (the kernel writes the record into pinned host memory, then a tag the
    host spins on) and inputs passed as kernel arguments return the same records as the
    H2D/D2H copy + stream-synchronise path (LLAMPC_SYNC_COMPLETION=1): polled and ticket
    (LLAMPC_NO_POLL=1) completions, look-back-only and look-ahead-only ticks,
    llampc_plan_async / llampc_plan_wait, and the H2D input copy (LLAMPC_NO_INLINE=1)."""
    from llampc.mpc import ModelBank, generate_bank
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    H, W, C, N = 20, 3, 3, 3000
    rng = np.random.RandomState(11)
    banks = [ModelBank(generate_bank(N, seed=4), W=W, device=0) for _ in range(5)]
    # bank 0: host completion, polled, inputs as kernel arguments; 1: H2D + D2H copies and a
    # stream synchronise; 2: host completion, ticket path; 3: host completion through
    # plan_async / plan_wait; 4: host completion with the H2D input copy
    modes = [{}, {"LLAMPC_SYNC_COMPLETION": "1"}, {"LLAMPC_NO_POLL": "1"}, {}, {"LLAMPC_NO_INLINE": "1"}]
    try:
        for t in range(1, W + 4):
            U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
            U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
            xref = s[:2, t:t + H + 1]
            args = (s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
            kw = dict(K=4, current_model=2,
                      do_lookahead=(t != 2), do_lookback=(t != 3))   # one lb-only, one la-only tick
            outs = []
            for i, (b, env) in enumerate(zip(banks, modes)):
                os.environ.update(env)
                try:
                    if i == 3:
                        b.plan_async(*args, **kw)
                        outs.append(b.plan_wait())
                    else:
                        outs.append(b.plan_raw(*args, **kw)[0])
                finally:
                    for k in env:
                        del os.environ[k]
            for o in outs[:1] + outs[2:]:
                _same_records(o, outs[1])
    finally:
        for b in banks:
            b.close()


def test_setupnlp_solve_sampling(nat):
    """setupNLP.solve drop-in (sampling over the NLP transcription on the GPU): the returned
    (umpc, fval, xmpc) are consistent with the oracle's NLP restatement — xmpc is the Euler
    trajectory of umpc, fval its objective (nmpc.py:44-111) — umpc meets the bounds and the
    steering-rate limits, and fval is no worse than holding uprev.  IPOPT's own optimum is
    parity unpinned (casadi absent)."""
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.mpc.planner import ConstantSpeed
    from llampc.params import ORCA
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    p = ORCA(control="pwm")
    H, Ts = 20, TS
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    model = Dynamic(**p)
    nlp = setupNLP(H, Ts, Q, P, R, p, model, ETHZ('optimal', True))
    track = ETHZ('optimal', True)
    x0, uprev, projidx = s[:, 10].copy(), u[:, 9].copy(), 0
    bank6 = tuple(np.array([p[k]]) for k in O.BANK_ORDER)
    for tick in range(3):
        xref, projidx, _ = ConstantSpeed(x0[:2], x0[3], track, H, Ts, projidx, curr_mu=0.9, scale=0.9)
        umpc, fval, xmpc, viol = nlp.solve(x0=x0, xref=xref[:2, :], uprev=uprev)
        assert umpc.shape == (2, H) and xmpc.shape == (6, H + 1) and viol == 0.0
        assert np.all(umpc >= np.array(p["min_inputs"])[:, None] - 1e-15)
        assert np.all(umpc <= np.array(p["max_inputs"])[:, None] + 1e-15)
        dd = np.diff(np.concatenate([uprev[1:2], umpc[1]]))
        assert np.all(np.abs(dd) <= 5.0 * Ts * (1 + 1e-12))
        traj = O.rollout_euler_nlp(shared(), bank6, x0, umpc.T[None], Ts)
        close(xmpc, traj[:, 0, :].T, RTOL_STEP * 10)
        close(fval, O.mpc_cost(traj, umpc.T[None], xref, uprev, Q, R, P)[0], RTOL_ROLL)
        hold = np.tile(uprev, (H, 1))[None]
        jh = O.mpc_cost(O.rollout_euler_nlp(shared(), bank6, x0, hold, Ts), hold, xref, uprev, Q, R, P)[0]
        assert fval <= jh * (1 + 1e-12)
        xn, _ = O.sim_continuous(O.Vehicle.from_params(O.orca_params()), x0, umpc[:, :1], [0, Ts])
        x0, uprev = xn[:, -1], umpc[:, 0].copy()
    nlp.close()


def _nlp(H=20):
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.params import ORCA
    from llampc.tracks import ETHZ
    p = ORCA(control="pwm")
    return setupNLP(H, TS, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, Dynamic(**p), ETHZ('optimal', True)), p


def test_setupnlp_cem_equals_oracle(nat):
    """The device cross-entropy search (csrc/nlp.hip) against its NumPy restatement
    (oracle.nlp_cem) over three successive solves (warm start, the held uprev in the first
    round): the same sequence (the samples are bitwise the oracle's; the elite ranking follows
    costs equal to 1e-6) and fval at 1e-6."""
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    nlp, p = _nlp()
    p6 = [p[k] for k in O.BANK_ORDER]
    try:
        from llampc.mpc.planner import ConstantSpeed
        from llampc.tracks import ETHZ
        tr = ETHZ('optimal', True)
        last = None
        for call, t in enumerate((10, 11, 12)):
            x0, up = s[:, t].copy(), u[:, t - 1].copy()
            xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, 20, TS, 0)
            umpc, fval, xmpc, _ = nlp.solve(x0, xref, up)
            base = None if last is None else np.concatenate([last[1:], last[-1:]])
            uo, jo = O.nlp_cem(shared(), p6, x0, xref, up, base, last is not None, 20, TS, call=call)
            np.testing.assert_array_equal(umpc.T, uo)
            np.testing.assert_allclose(fval, jo, rtol=RTOL_ROLL)
            last = umpc.T.copy()
    finally:
        nlp.close()


def test_setupnlp_one_launch_equals_round_launches(nat, monkeypatch):
    """Every CEM round in one launch (the sample blocks wait for each round's mean / std on a
    tagged word, nlp.hpp nlp_persistent) against one launch per round
    (LLAMPC_NLP_ROUND_LAUNCHES=1 at create): the same umpc, fval and xmpc, bitwise, over four
    successive solves (the warm start and the best-so-far carried across rounds)."""
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    outs = []
    for per_round in ("0", "1"):
        monkeypatch.setenv("LLAMPC_NLP_ROUND_LAUNCHES", per_round)
        nlp, _ = _nlp()
        try:
            got = []
            for t in (10, 11, 12, 13):
                x0, up = s[:, t].copy(), u[:, t - 1].copy()
                xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, 20, TS, 0)
                umpc, fval, xmpc, _ = nlp.solve(x0, xref, up)
                got.append((np.array(umpc, copy=True), float(fval), np.array(xmpc, copy=True)))
        finally:
            nlp.close()
        outs.append(got)
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a[0], b[0])
        assert a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])


def test_setupnlp_kept_states_equal_rerun(nat, monkeypatch):
    """The result's trajectory copied from the last round's rollout states kept in LDS (nlp.hip
    NlpLaunch.ltraj, the best sample's own block) against the best sequence's rollout re-run
    by block 0 (LLAMPC_NLP_RERUN_TRAJ=1 at create): umpc and fval bitwise, xmpc to 1e-12 (the
    staged and the unstaged rollout of the same inputs), over six successive solves."""
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    outs = []
    for rerun in ("0", "1"):
        monkeypatch.setenv("LLAMPC_NLP_RERUN_TRAJ", rerun)
        nlp, _ = _nlp()
        try:
            got = []
            for t in range(20, 26):
                x0, up = s[:, t].copy(), u[:, t - 1].copy()
                xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, 20, TS, 0)
                umpc, fval, xmpc, _ = nlp.solve(x0, xref, up)
                got.append((np.array(umpc, copy=True), float(fval), np.array(xmpc, copy=True)))
        finally:
            nlp.close()
        outs.append(got)
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a[0], b[0])
        assert a[1] == b[1]
        np.testing.assert_allclose(a[2], b[2], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("samples,elite,iters,H", [(64, 5, 3, 20), (256, 17, 3, 20), (4096, 64, 2, 20), (1024, 1, 2, 20),
                                                   (512, 32, 3, 40)])
def test_setupnlp_cem_shapes_equal_oracle(nat, samples, elite, iters, H):
    """The CEM's selection (each sample block's in-wave sort, the merge tree of the blocks'
    lists) at other sizes: one block (64 samples), a non-power-of-two elite, the largest
    search (4,096 samples, 64 elite) and elite 1 — the same sequence and fval as oracle.nlp_cem."""
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.mpc.planner import ConstantSpeed
    from llampc.params import ORCA
    from llampc.tracks import ETHZ
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    p = ORCA(control="pwm")
    tr = ETHZ('optimal', True)
    nlp = setupNLP(H, TS, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, Dynamic(**p), tr,
                   samples=samples, elite=elite, iters=iters)
    p6 = [p[k] for k in O.BANK_ORDER]
    try:
        x0, up = s[:, 20].copy(), u[:, 19].copy()
        xref, _, _ = ConstantSpeed(x0[:2], x0[3], tr, H, TS, 0)
        umpc, fval, xmpc, _ = nlp.solve(x0, xref, up)
        uo, jo = O.nlp_cem(shared(), p6, x0, xref, up, None, False, H, TS, samples=samples, iters=iters, elite=elite)
        np.testing.assert_array_equal(umpc.T, uo)
        np.testing.assert_allclose(fval, jo, rtol=RTOL_ROLL)
        bank6 = tuple(np.array([p[k]]) for k in O.BANK_ORDER)
        traj = O.rollout_euler_nlp(shared(), bank6, x0, uo[None], TS)   # xmpc: the last round's quad
        np.testing.assert_allclose(xmpc, traj[:, 0, :].T, rtol=RTOL_STEP * 10, atol=1e-12)
    finally:
        nlp.close()


def test_setupnlp_within_1pct_of_local_optimum(nat):
    """Solution quality of the setupNLP drop-in: on three DYN-slice ticks its fval is within
    1 % of a local optimum of the same restated NLP found by scipy's SLSQP
    (tests/golden/nlp_optimum.npz, gen_nlp_optimum.py) — measured 1.0013, 1.0023, 1.0079 (the
    search is deterministic: bitwise the oracle's, test_setupnlp_cem_equals_oracle).
    IPOPT's own optimum stays unpinned."""
    g = golden("nlp_optimum.npz")
    for i in range(len(g["fstar"])):
        nlp, _ = _nlp()
        try:
            umpc, fval, _, _ = nlp.solve(g["x0"][i], g["xref"][i], g["uprev"][i])
        finally:
            nlp.close()
        assert fval <= 1.01 * g["fstar"][i], (int(g["tick"][i]), fval, g["fstar"][i])


@pytest.mark.parametrize("track_name,start", [("ETHZ", "projected"), ("ETHZ", "lap_end"), ("ETHZMobil", "projected")])
def test_lookahead_raceline_per_model_xref(nat, track_name, start):
    """xref_mode RACELINE: every model's look-ahead tracks its own
    ConstantSpeed reference with mu_n = (Df_n + Dr_n) / (9.81 m), evaluated on the device
    from the raceline splines — against the oracle's ConstantSpeed loop (planner.py:34-65,
    pinned by tests/golden/planner.npz) per model.  Wide bank: mu_n below, inside and above
    the profile range; 'lap_end' starts 3 cm before the lap length (the mod-L wrap)."""
    from llampc.mpc import ModelBank, generate_bank, plan
    from llampc.mpc.planner import raceline_start
    from llampc.tracks import ETHZ, ETHZMobil
    tr = ETHZ('optimal', True) if track_name == "ETHZ" else ETHZMobil('optimal', True)
    td = np.load(os.path.join(os.path.dirname(__file__), "..", "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td[f"{track_name}_x"], td[f"{track_name}_y"], td[f"{track_name}_speeds"], td[f"{track_name}_mus"])
    N, C, H, scale = 192, 2, 20, 0.9
    p = generate_bank(N, seed=21, sigma=0.45)
    d = golden("dyn_slice.npz")
    x0 = d["states"][:, 30].copy()
    if track_name == "ETHZMobil":
        x0[:3] = [tr.x_init, tr.y_init, tr.psi_init]
    rng = np.random.RandomState(4)
    U = np.stack([rng.uniform(0.2, 0.8, (C, H)), rng.uniform(-0.2, 0.2, (C, H))], axis=-1)
    uprev = U[0, 0]
    if start == "lap_end":
        s0 = float(tr.length) - 0.03
    else:
        s0, _ = raceline_start(x0, tr, 0)
    v0 = float(x0[3])
    mass = O.orca_params()["mass"]
    mu = (p[2] + p[5]) / (9.81 * mass)
    assert mu.min() < ref.mus[0] and mu.max() > ref.mus[-1]
    traj = O.rollout_rk4(shared(), tuple(p), x0, U, TS)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    cref = np.empty((N, C))
    for n in range(N):
        xr, _ = O.constant_speed_from(s0, x0[:2], v0, ref, H, TS, scale, mu[n])
        cref[n] = O.mpc_cost(traj[:, n * C:(n + 1) * C], U, xr, uprev, Q, R, P)
    with ModelBank(p, device=0) as b:
        b.set_raceline(tr)
        res = plan(b, x0, uprev, x0, None, U, uprev=uprev, Ts=TS, do_lookback=False,
                   return_costs=True, raceline_start=(s0, v0, scale))
    close(res.costs, cref, RTOL_ROLL)
    assert res.global_best[0] * C + res.global_best[1] == int(np.argmin(np.where(np.isnan(cref), np.inf, cref).ravel()))


@pytest.mark.parametrize("C,gap", [(64, 1e-9), (64, 1e-12), (8, 1e-7)])
def test_lookahead_argmin_near_ties(nat, C, gap):
    """The look-ahead's candidate choice when candidates nearly tie: C candidates
    that differ by `gap` (relative) in their steering, so many costs lie within the rollouts'
    error bound of each other.  The choice must be exact where the oracle's best and second
    best differ by more than twice RTOL_ROLL, and wherever they do not, the chosen candidate's
    ORACLE cost must lie within 2 RTOL_ROLL of the minimum (a flip among costs the fp64 cores
    cannot tell apart, never a worse control).  The flip count is reported."""
    from llampc.mpc import ModelBank, generate_bank
    N, H = 400, 20
    p = generate_bank(N, seed=77)
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    x0 = s[:, 40]
    base = u[:, 40:40 + H].T.copy()
    U = np.repeat(base[None], C, axis=0)
    U[:, :, 1] += (np.arange(C) * gap * 0.3)[:, None]
    xref = np.vstack([s[0, 40:41 + H] + 0.01, s[1, 40:41 + H] - 0.02])
    up = u[:, 39]
    with ModelBank(p, device=0) as b:
        r = b.lookahead(x0, U, xref, up, Ts=TS, return_costs=True, return_best_cand=True)
    cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), x0, U, TS), U, xref, up, np.eye(2), np.diag([5e-3, 1]),
                      np.zeros((2, 2))).reshape(N, C)
    close(r["costs"].ravel(), cref.ravel(), RTOL_ROLL)
    cm = np.where(np.isnan(cref), np.inf, cref)
    got = r["best_cand_per_model"]
    srt = np.sort(cm, axis=1)
    sep = (srt[:, 1] - srt[:, 0]) > 2 * RTOL_ROLL * np.abs(srt[:, 0])
    want = np.argmin(cm, axis=1)
    np.testing.assert_array_equal(got[sep], want[sep])
    chosen = cm[np.arange(N), got]
    assert np.all(chosen <= srt[:, 0] * (1 + 2 * RTOL_ROLL)), np.max(chosen / srt[:, 0])
    flips = int(np.sum(got != want))
    print(f"C={C} gap={gap}: {int(np.sum(~sep))} of {N} models near-tied, {flips} choices differ from the oracle's argmin")


def _decided_argmin(cost, bound):
    """The oracle's argmin over `cost` (NaN last, ties to the lower index; the kernel's order) and
    whether it is DECIDED: its relative gap to the runner-up exceeds the two entries' core-error
    bounds (no evaluation within those errors can rank them the other way)."""
    c = np.where(np.isnan(cost), np.inf, cost)
    order = np.argsort(c, kind="stable")
    b, r = int(order[0]), int(order[1]) if c.size > 1 else -1
    if not np.isfinite(c[b]):
        return b, False
    if r < 0 or not np.isfinite(c[r]):
        return b, False                      # no finite runner-up to measure the gap against
    gap = (c[r] - c[b]) / max(abs(c[b]), 1e-300)
    return b, bool(gap > bound[b] + bound[r])


@pytest.mark.parametrize("sigma", [1.5, 2.0])
def test_wide_sigma_lookahead_argmins(nat, sigma):
    """The reference's wide banks (sigma = 1.5: nrt.py:170-175; sigma = 2: plot_comp_time.py:186-191)
    hold models far from nominal whose rollouts amplify the look-ahead's core errors (the sigma = 2
    fixture's costs differ from the oracle by up to 1.2e-2).  Every cost is held to its
    core-error bound (conftest.core_error_bound), and the per-model argmin over the C candidates
    and the global argmin must equal the oracle's wherever the oracle's best-vs-second gap exceeds
    the two pairs' bounds; where it does not, the argmin may flip, and the test reports how often
    it did (profiles/r06: the flip rate per sigma)."""
    import json
    from llampc.mpc import ModelBank, generate_bank
    N, C, H = 1500, 8, 20
    p = generate_bank(N, seed=37, sigma=sigma)
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    x0, uprev = s[:, 60], u[:, 59]
    rng = np.random.RandomState(5)
    U = np.repeat(u[:, 60:60 + H].T[None], C, axis=0)
    U[1:] += rng.randn(C - 1, H, 2) * np.array([0.05, 0.02])
    U = np.clip(U, [-0.1, -0.35], [1.0, 0.35])
    xref = s[:2, 60:61 + H].copy()
    Q, R, P = np.eye(2), np.diag([5e-3, 1.0]), np.zeros((2, 2))
    with ModelBank(p, device=0) as b:
        res = b.lookahead(x0, U, xref, uprev, Ts=TS, return_costs=True, return_best_cand=True)
    with np.errstate(all="ignore"):
        cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), x0, U, TS), U, xref, uprev, Q, R, P)
    bound = core_error_bound(shared(), tuple(p), x0, U, xref, uprev, Q, R, P)
    got = res["costs"].ravel()
    # tracked pairs: the oracle's cost is finite and reproducible to 10 % under the cores' errors
    # — held to max(rtol, their bound); the rest diverge (NaN / inf, or a cost the cores' errors
    # move by more than 10 %: a one-ulp change of x0 moves it as much in NumPy) and are counted
    fin = np.isfinite(cref)
    tracked = fin & (bound <= 0.1)
    assert np.isfinite(got[tracked]).all()
    rel = np.abs(got[tracked] - cref[tracked]) / np.abs(cref[tracked])
    allowed = np.maximum(RTOL_ROLL, bound[tracked])
    assert (rel <= allowed).all(), (rel[rel > allowed][:5], allowed[rel > allowed][:5])
    conditioned = int((rel > RTOL_ROLL).sum())
    nonfinite_agree = int((np.isfinite(got[~fin]) == False).sum())   # noqa: E712
    cr, bd = cref.reshape(N, C), bound.reshape(N, C)
    decided = flips = undecided = 0
    for n in range(N):
        best, ok = _decided_argmin(cr[n], bd[n])
        if not np.isfinite(cr[n, best]):
            continue                                     # no finite candidate
        if ok:
            decided += 1
            assert res["best_cand_per_model"][n] == best, (n, res["best_cand_per_model"][n], best, cr[n])
        else:
            undecided += 1
            flips += int(res["best_cand_per_model"][n] != best)
    gbest, gok = _decided_argmin(cref, bound)
    g_got = res["best_model"] * C + res["best_cand"]
    if gok:
        assert g_got == gbest, (g_got, gbest)
    out = dict(sigma=sigma, N=N, C=C, H=H, tracked=int(tracked.sum()), held_by_bound=conditioned,
               diverged=int((~tracked).sum()), oracle_nonfinite=int((~fin).sum()), nonfinite_agree=nonfinite_agree,
               models_decided=decided, models_undecided=undecided, undecided_flips=flips,
               global_decided=gok, global_flip=bool(g_got != gbest))
    print("wide-sigma argmins:", json.dumps(out))
    assert decided > N // 2                              # the check covers most of the bank
