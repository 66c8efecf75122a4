"""BASELINE configs through the HIP path, each on its own inputs as SURVEY.md §8(d) states them:

  config 1  the reference-generated fixture tests/golden/config1.npz (N = 100, DYN states[:,
            490:501], U = inputs[:, 500:520], ConstantSpeed(mu = 0.9092, scale = 0.9)): the
            ten look-back ticks and the look-ahead of plan() against the reference's own errors,
            window mean, argmin, top-K and H x _integrate_batch trajectories
  config 2  ETHZ, N = 10^4, H = 20, the gradual-friction scenario states of the bench
            (llampc.mpc.scenarios, the RK6 plant) — every tick's errors, and on the ticks with a
            full window the selection and every model's cost, against the oracle
  config 3  ETHZMobil, N = 10^4, H = 40, the sudden-drop scenario's synthetic Mobil states
            (track start, seed 3), same checks
Tolerances: one integration step 1e-9 (the look-back); rollout costs RTOL_ROLL = 1e-7, or for
an ill-conditioned rollout its core-error bound: the lean cores' measured errors propagated
through the oracle's rollout (conftest.core_error_bound / assert_costs_close; DESIGN §4 has the
measured errors per shape); indices exact."""
import os

import numpy as np
import pytest

from conftest import REPO, assert_costs_close, core_error_bound, golden
from oracle import llampc_oracle as O

pytestmark = pytest.mark.gpu

TS = 0.02
RTOL_STEP = 1e-9
RTOL_ROLL = 1e-7
Q, R, P = np.eye(2), np.diag([5e-3, 1.0]), np.zeros((2, 2))


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


def close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
    fin = np.isfinite(b)
    sc = np.max(np.abs(b[fin])) if fin.any() else 1.0
    np.testing.assert_allclose(a[fin], b[fin], rtol=rtol, atol=rtol * 1e-3 * sc)


def test_config1_plan_vs_reference_fixture(nat):
    """Config 1 exactly: ten plan() ticks on the DYN transitions 490 -> 500 (the window fills on
    the last), look-ahead of the one candidate U = inputs[:, 500:520] from x0 = states[:, 500]
    with the reference's ConstantSpeed(mu = 0.9092, scale = 0.9) reference."""
    from llampc.mpc import DeviceController, ModelBank, plan
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    g = golden("config1.npz")
    bank, s, u = g["bank"], g["states"], g["inputs"]
    W, K, H = int(g["W"]), int(g["K"]), int(g["H"])
    tr = ETHZ('optimal', True)
    # the package's planner (host and device) on the config's exact call
    xr, pj, vr = ConstantSpeed(g["x0"][:2], g["x0"][3], tr, H, TS, int(g["projidx_in"]), scale=float(g["scale"]),
                               curr_mu=float(g["mu"]))
    np.testing.assert_allclose(xr, g["xref"], rtol=1e-10, atol=1e-12)
    assert pj == int(g["projidx_out"])
    np.testing.assert_allclose(vr, float(g["vr"]), rtol=1e-10)
    with ModelBank(bank, W=W, device=0) as b:
        ctl = DeviceController(b, tr, H=H, C=1, K=K)
        try:
            dxr, dpj, dvr = ctl.reference(g["x0"][:2], g["x0"][3], H, int(g["projidx_in"]), float(g["mu"]),
                                          float(g["scale"]))
        finally:
            ctl.close()
        np.testing.assert_allclose(dxr, g["xref"], rtol=1e-10, atol=1e-12)
        assert dpj == int(g["projidx_out"])
        for t in range(W):
            res = plan(b, s[:, t + 1], u[:, t], s[:, t], g["xref"], g["U"], uprev=u[:, t], Ts=TS, K=K,
                       return_errors=True, return_window_mean=True, return_costs=(t == W - 1))
            close(res.lookback_err, g["errors"][t], RTOL_STEP)
            assert res.window_full == (t == W - 1)
    close(res.window_mean, g["window_mean"], RTOL_STEP)
    assert res.best_model == int(g["best"])
    np.testing.assert_array_equal(res.topk, g["topk"])
    cref = O.mpc_cost(g["traj"], g["U"], g["xref"], g["uprev"], Q, R, P)
    close(res.costs.ravel(), cref, RTOL_ROLL)
    assert res.best_cand == 0
    np.testing.assert_allclose(res.cost, cref[int(g["best"])], rtol=RTOL_ROLL)
    assert res.global_best[0] == int(np.argmin(cref))


@pytest.mark.parametrize("track,H,seed", [("ETHZ", 20, 0), ("ETHZMobil", 40, 1)])
def test_config_scenario_ticks_vs_oracle(nat, track, H, seed):
    """Configs 2 and 3 at their size (N = 10^4, C = 1) on the bench's own scenario inputs
    (llampc.mpc.scenarios.scenario_ticks: RK6-plant states under the config's friction change,
    ConstantSpeed xref): W + 3 plan() ticks; every tick's look-back errors, then on each of the
    three ticks with a full window the window mean, argmin, top-K and all N costs vs the oracle."""
    from llampc.mpc import ModelBank, generate_bank, plan
    from llampc.mpc.scenarios import scenario_ticks, unpack
    N, C, W, K = 10000, 1, 10, 10
    ticks = scenario_ticks(track, H, C, W + 3, device=0)
    if track == "ETHZMobil":                       # Mobil states, not the ETHZ recording
        from llampc.tracks import ETHZMobil
        tr = ETHZMobil('optimal', True)
        assert np.hypot(ticks[0][0] - tr.x_init, ticks[0][1] - tr.y_init) < 0.2
    p = generate_bank(N, seed=seed)
    win = O.LookbackWindow(N, W, K)
    full_ticks = conditioned = 0
    with ModelBank(p, W=W, device=0) as b:
        for t, pk in enumerate(ticks):
            f = unpack(pk, H, C)
            last = t >= W - 1
            res = plan(b, f["x_now"], f["u_prev"], f["x_prev"], f["xref"], f["U"], uprev=f["uprev"], Ts=TS, K=K,
                       return_errors=True, return_window_mean=last, return_costs=last)
            e = O.lookback_errors(O.evaluate_models_vectorized(shared(), tuple(p), f["x_prev"], f["u_prev"], TS),
                                  f["x_now"])
            close(res.lookback_err, e, RTOL_STEP)
            assert win.push(e) == res.window_full
            if not res.window_full:
                continue
            full_ticks += 1
            close(res.window_mean, win.avg, RTOL_STEP)
            assert res.best_model == win.current
            np.testing.assert_array_equal(res.topk, win.best_k)
            cref = O.mpc_cost(O.rollout_rk4(shared(), tuple(p), f["x_now"], f["U"], TS), f["U"], f["xref"],
                              f["uprev"], Q, R, P)
            sens = lambda idx: core_error_bound(shared(), tuple(p[:, idx]), f["x_now"], f["U"], f["xref"],  # noqa: E731
                                                f["uprev"], Q, R, P)
            conditioned += assert_costs_close(res.costs.ravel(), cref, RTOL_ROLL, sens)
            assert_costs_close([res.cost], [cref[win.current]], RTOL_ROLL, lambda idx: sens(np.array([win.current])))
            assert res.global_best[0] == int(np.argmin(np.where(np.isnan(cref), np.inf, cref)))
    assert full_ticks == 4
    print(f"{track}: {conditioned} of {4 * N} costs held by their conditioning bound")
