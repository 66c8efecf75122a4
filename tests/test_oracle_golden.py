"""Pin the CPU oracle (oracle/llampc_oracle.py) against vectors produced by running the
reference itself (tests/golden/gen_golden.py) and the reference's own stored known
answers (results/**/MUs.npy).  Bitwise wherever the reference ran the same NumPy ops."""
import numpy as np
import pytest

from conftest import golden
from oracle import llampc_oracle as O

TS = 0.02


def shared():
    p = O.orca_params()
    return {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}


def veh(params6, **kw):
    s = shared()
    Bf, Cf, Df, Br, Cr, Dr = params6
    return O.Vehicle(Bf=Bf, Cf=Cf, Df=Df, Br=Br, Cr=Cr, Dr=Dr, **s, **kw)


def test_bank_generation_matches_reference_loop():
    g = golden("bank_rt_seed0_n1000.npz")
    np.testing.assert_array_equal(O.make_bank(1000, 0), g["bank"])
    w = golden("bank_wide_seed7_n512.npz")
    np.testing.assert_array_equal(O.make_bank(512, 7, sigma=2.0), w["bank"])


def test_batched_forces_deriv_rk4_bitwise():
    g = golden("dynamics_batch.npz")
    v = veh(tuple(g["params"]))
    with np.errstate(all="ignore"):
        Ffy, Frx, Fry, af, ar = O.calc_forces_batch(v, g["x"], g["u"], return_slip=True)
        for a, b in ((Ffy, "Ffy"), (Frx, "Frx"), (Fry, "Fry"), (af, "alphaf"), (ar, "alphar")):
            np.testing.assert_array_equal(a, g[b])
        np.testing.assert_array_equal(O.diffequation_batch(v, g["x"], g["u"]), g["dxdt"])
        np.testing.assert_array_equal(O.integrate_batch(v, g["x"], g["u"], 0, TS), g["x_rk4"])
    p = O.orca_params()
    vn = veh(tuple(p[k] for k in O.BANK_ORDER))
    np.testing.assert_array_equal(O.diffequation_batch(vn, g["x"], g["u"]), g["dxdt_nominal"])
    np.testing.assert_array_equal(O.integrate_batch(vn, g["x"], g["u"], 0, TS), g["x_rk4_nominal"])


def test_approx_and_input_acc_variants():
    g = golden("dynamics_batch.npz")
    p = O.orca_params()
    va = O.Vehicle.from_params(p, Bf=None, Br=None, Df=None, Dr=None)
    assert va.approx
    np.testing.assert_array_equal(O.diffequation_batch(va, g["x_apx"], g["u"]), g["dxdt_approx"])
    vi = O.Vehicle.from_params(p, input_acc=True)
    np.testing.assert_array_equal(O.diffequation_batch(vi, g["x"], g["u"]), g["dxdt_input_acc"])


def test_lookback_window_argmin_topk():
    g = golden("lookback_n1000.npz")
    d = golden("dyn_slice.npz")
    bank = golden("bank_rt_seed0_n1000.npz")["bank"]
    s, u = d["states"], d["inputs"]
    win = O.LookbackWindow(bank.shape[1], int(g["W"]), int(g["K"]))
    full = 0
    for t in range(int(g["ticks"])):
        pred = O.evaluate_models_vectorized(shared(), tuple(bank), s[:, t], u[:, t], TS)
        if t < 3:
            np.testing.assert_array_equal(pred, g["pred"][t])
        e = O.lookback_errors(pred, s[:, t + 1])
        np.testing.assert_array_equal(e, g["errors"][t])
        if win.push(e):
            np.testing.assert_array_equal(win.avg, g["window_mean"][full])
            assert win.current == g["best"][full]
            np.testing.assert_array_equal(win.best_k, g["topk"][full])
            full += 1
    assert full == len(g["best"])


def test_window_mean_pairwise_order_matches_numpy():
    g = golden("lookback_n1000.npz")
    e = g["errors"]
    W = int(g["W"])
    # ring slot order oldest->newest for the first full window
    for n in range(0, e.shape[1], 97):
        col = [e[t, n] for t in range(W)]
        assert O.np_pairwise_sum(col) / W == g["window_mean"][0][n]


def test_rk4_rollout_matches_reference_composition():
    g = golden("rollout_rk4.npz")
    traj = O.rollout_rk4(shared(), tuple(g["params"]), g["x0"], g["U"], TS)
    np.testing.assert_array_equal(traj, g["traj"])


def test_wide_bank_nonfinite():
    g = golden("rollout_wide.npz")
    with np.errstate(all="ignore"):
        traj = O.rollout_rk4(shared(), tuple(g["params"]), g["x0"], g["U"], TS)
        pred = O.evaluate_models_vectorized(shared(), tuple(g["params"]), g["x0"], g["U"][0, 0], TS)
    np.testing.assert_array_equal(traj[-1], g["x_final"])
    np.testing.assert_array_equal(pred, g["lookback_pred"])


def test_rk6_plant():
    g = golden("plant_rk6.npz")
    p = O.orca_params()
    x = g["x"][0]
    for k in range(g["u"].shape[1]):
        v = O.Vehicle.from_params(p, Df=g["Df"][k], Dr=g["Dr"][k])
        xn, _ = O.sim_continuous(v, x, g["u"][:, k:k + 1], [0, TS])
        x = xn[:, -1]
        np.testing.assert_array_equal(x, g["x"][k + 1])
    xm, dm = O.sim_continuous(O.Vehicle.from_params(p), g["x"][0], g["u"][:, :10], np.arange(11) * TS)
    np.testing.assert_array_equal(xm, g["x_multi"])
    np.testing.assert_array_equal(dm, g["dxdt_multi"])


@pytest.mark.parametrize("name", ["ETHZ", "ETHZMobil"])
def test_planner_constant_speed(name):
    g = golden("planner.npz")
    tr = np.load(O.__file__.replace("oracle/llampc_oracle.py", "lla-mpc_amd/llampc/tracks/data/tracks.npz"))
    rl = O.RacelineRef(tr[f"{name}_x"], tr[f"{name}_y"], tr[f"{name}_speeds"], tr[f"{name}_mus"])
    np.testing.assert_array_equal(np.asarray(rl.spline.s), tr[f"{name}_s"])
    for case, xr in zip(g[f"{name}_cases"], g[f"{name}_xref"]):
        px, py, v0, pi, mu, scale, H, pidx, vr = case
        H = int(H)
        out, oidx, ovr = O.constant_speed(np.array([px, py]), v0, rl, H, TS, int(pi), scale=scale, curr_mu=mu)
        np.testing.assert_array_equal(out, xr[:, :H + 1])
        assert oidx == pidx and ovr == vr


def test_closed_loop_lookback_and_mu_estimator():
    g = golden("closed_loop.npz")
    bank = g["bank"]
    np.testing.assert_array_equal(bank, O.make_bank(bank.shape[1], int(g["seed"])))
    p = O.orca_params()
    x, u = g["x"], g["u"]
    win = O.LookbackWindow(bank.shape[1], 10, 10)
    mu = O.MuEstimator(mass=p["mass"], lf=p["lf"], lr=p["lr"])
    b6 = tuple(bank)
    for idt in range(u.shape[1]):
        if idt <= 10:
            mu.warmup()
        else:
            mu.update(bank[5][win.best_k], bank[2][win.best_k])
            assert mu.mu_pred == g["mu_pred"][idt]
        assert mu.mu_logged[-1] == g["mu_logged"][idt]
        if idt > 0:
            e = O.lookback_errors(O.evaluate_models_vectorized(shared(), b6, x[idt], u[:, idt], TS), x[idt + 1])
            if win.push(e):
                np.testing.assert_array_equal(win.best_k, g["topk"][idt])
        assert win.current == g["current"][idt]


@pytest.mark.parametrize("key,style,kw", [
    ("LLA_CASE2GRADAFTER", "const_decay", dict(start=14.3)),
    ("LLA_CASE4SUDDAFTER_22", "sudden", dict(window=(14.3, 14.5))),
    ("LLA_CASE5CONSTANT", "no_change", {}),
    ("LLAT2_CASE2GRADAFTER", "const_decay", dict(start=5)),
    ("LLA_CASE3SUDDBEG_22", "sudden", dict(window=(3.3, 3.5))),
])
def test_friction_schedule_known_answers(key, style, kw):
    """results/**/MUs.npy (the reference's stored runs) pin update_friction (rt.py:125-141)."""
    ans = golden("mus_known_answers.npz")[key]
    p = O.orca_params()
    Df, Dr = p["Df"], p["Dr"]
    out = []
    for i in range(len(ans)):
        Df, Dr = O.update_friction(Df, Dr, i * TS, style, **kw)
        out.append((Df + Dr) / (9.81 * p["mass"]))
    np.testing.assert_array_equal(np.array(out), ans)


def test_cost_and_feasibility_sanity():
    """The MPC cost restatement (nmpc.py:44-111, parity unpinned): hand-computed case."""
    H, C = 3, 2
    U = np.zeros((C, H, 2))
    U[1, :, 1] = [0.1, 0.2, 0.3]
    traj = np.zeros((H + 1, 2, 6))
    traj[:, :, 0] = 1.0                      # x error of 1 at every step
    xref = np.zeros((2, H + 1))
    Q, R, P = np.diag([1, 1]), np.diag([5e-3, 1]), np.diag([0, 0])
    c = O.mpc_cost(traj, U, xref, np.zeros(2), Q, R, P)
    np.testing.assert_allclose(c, [3.0, 3.0 + 3 * 0.01])
    ok = O.candidates_feasible(U, np.zeros(2), [-0.1, -0.35], [1.0, 0.35], 5.0, 0.02)
    assert list(ok) == [True, True]
    U[1, 1, 1] = 0.5
    assert list(O.candidates_feasible(U, np.zeros(2), [-0.1, -0.35], [1.0, 0.35], 5.0, 0.02)) == [True, False]


def test_config1_plan_cpu_matches_reference():
    """BASELINE config 1 exactly as SURVEY.md §8(d) states it (tests/golden/config1.npz, written
    by the reference: N = 100, DYN states[:, 490:501], U = inputs[:, 500:520], ConstantSpeed with
    mu = 0.9092, scale = 0.9): the oracle's bank, look-back window / argmin / top-K, H-step RK4
    rollout (bitwise) and its ConstantSpeed (1e-12: banded vs dense spline solve)."""
    g = golden("config1.npz")
    N, W, K, H = g["bank"].shape[1], int(g["W"]), int(g["K"]), int(g["H"])
    np.testing.assert_array_equal(O.make_bank(N, int(g["seed"])), g["bank"])
    s, u = g["states"], g["inputs"]
    win = O.LookbackWindow(N, W, K)
    for t in range(W):
        e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(g["bank"]), s[:, t], u[:, t], TS), s[:, t + 1])
        np.testing.assert_array_equal(e, g["errors"][t])
        full = win.push(e)
    assert full and win.current == int(g["best"])
    np.testing.assert_array_equal(win.avg, g["window_mean"])
    np.testing.assert_array_equal(win.best_k, g["topk"])
    traj = O.rollout_rk4(shared(), tuple(g["bank"]), g["x0"], g["U"], TS)
    np.testing.assert_array_equal(traj, g["traj"])
    import os
    from conftest import REPO
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td["ETHZ_x"], td["ETHZ_y"], td["ETHZ_speeds"], td["ETHZ_mus"])
    xref, pidx = O.constant_speed(g["x0"][:2], g["x0"][3], ref, H, TS, int(g["projidx_in"]), scale=float(g["scale"]),
                                  curr_mu=float(g["mu"]))[:2]
    assert pidx == int(g["projidx_out"])
    np.testing.assert_allclose(xref, g["xref"], rtol=1e-12, atol=1e-12)
