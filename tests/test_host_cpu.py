"""CPU tests (no GPU): the C-ABI library loads and exports every symbol include/llampc.h
declares, the shared merge code (run on the host here), and the host-side logic of the
package (bank generation, sharding, planner, splines, candidates, mu-hat, friction)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, golden
from oracle import llampc_oracle as O

HEADER = os.path.join(REPO, "include", "llampc.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(llampc_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from llampc import _native
    lib = _native.load()
    names = header_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_native._SIGNATURES), set(names) ^ set(_native._SIGNATURES)
    assert lib.llampc_abi_version() == 1


def test_struct_layouts_match_header():
    from llampc import _native
    # llampc_plan_out: 4 int32 + lb(8+8) + sel(8+4+4+8) + la(8+4+4+8) + 6 arrays of KMAX
    expect = 16 + 16 + 24 + 24 + 32 * (8 + 8 + 8 + 8 + 4 + 8)
    assert _native.PLAN_OUT_BYTES == expect
    assert ctypes.sizeof(_native.Cost) == 8 * 18 + 8
    assert ctypes.sizeof(_native.Vehicle) == 8 * 8 + 8
    # llampc_ctl_cfg / llampc_ctl_out (static_asserts in capi.hip hold the same numbers)
    assert ctypes.sizeof(_native.CtlCfg) == 280
    assert ctypes.sizeof(_native.CtlOut) == _native.PLAN_OUT_BYTES + 56 + 16 * _native.HMAX


def test_no_device_fails_loudly():
    """Without a GPU the product raises instead of falling back to the CPU."""
    from llampc import _native
    if _native.device_count() > 0:
        pytest.skip("a HIP device is visible")
    from llampc.models import Dynamic
    from llampc.mpc import ModelBank
    with pytest.raises(_native.NoDeviceError):
        ModelBank(np.ones((6, 4)))
    with pytest.raises(_native.NoDeviceError):
        Dynamic(**O.orca_params())._diffequation_batch(None, np.zeros((2, 6)), np.zeros((2, 2)))


# ------------------------------------------------------------------ merge (host build)
def _record(nat, gidx, vals, Df, Dr, cand, ccost, K, count, W, lb=None, la=None, sel=None):
    o = nat.PlanOut()
    o.window_count, o.window_full, o.K = count, int(count >= W), K
    order = sorted(range(len(vals)), key=lambda i: (np.isnan(vals[i]), vals[i] if not np.isnan(vals[i]) else 0, gidx[i]))
    for k in range(nat.KMAX):
        if k < K and k < len(order):
            i = order[k]
            o.topk[k], o.topk_val[k], o.topk_Df[k], o.topk_Dr[k] = gidx[i], vals[i], Df[i], Dr[i]
            o.topk_cand[k], o.topk_cost[k] = cand[i], ccost[i]
        else:
            o.topk[k], o.topk_cand[k] = -1, -1
    o.lb_best, o.lb_best_val = lb if lb is not None else (-1, np.nan)
    o.sel_model, o.sel_owned, o.sel_cand, o.sel_cost = sel
    o.la_best_model, o.la_best_cand, o.la_best_cost = la
    o.n_nonfinite = 1
    return o


@pytest.mark.parametrize("seed", range(6))
def test_merge_matches_unsharded_numpy(seed):
    from llampc import _native as nat
    rng = np.random.RandomState(seed)
    N, G, K, C = 200, 4, 10, 3
    wm = rng.rand(N)
    wm[rng.randint(0, N, 3)] = wm[5]                    # exact ties
    if seed % 2:
        wm[rng.randint(0, N, 2)] = np.nan               # NaNs (argmin -> first NaN)
    cost = rng.rand(N, C)
    Df, Dr = rng.rand(N), rng.rand(N)
    bc = np.argmin(cost, axis=1)
    bcost = cost[np.arange(N), bc]
    parts = []
    bounds = np.linspace(0, N, G + 1).astype(int)
    for g in range(G):
        lo, hi = bounds[g], bounds[g + 1]
        idx = np.arange(lo, hi)
        loc_min = lo + int(np.argmin(wm[lo:hi]))
        la = divmod(lo * C + int(np.argmin(cost[lo:hi].ravel())), C)
        parts.append(_record(nat, idx, wm[lo:hi], Df[lo:hi], Dr[lo:hi], bc[lo:hi], bcost[lo:hi], K, 10, 10,
                             lb=(loc_min, wm[loc_min]), la=(la[0], la[1], cost[la]),
                             sel=(loc_min, 1, bc[loc_min], bcost[loc_min])))
    m = nat.plan_out_to_dict(nat.merge(parts))
    gbest = int(np.argmin(wm))
    assert m["lb_best"] == gbest and m["sel_model"] == gbest and m["sel_cand"] == bc[gbest]
    ref_top = sorted(range(N), key=lambda i: (np.isnan(wm[i]), 0 if np.isnan(wm[i]) else wm[i], i))[:K]
    np.testing.assert_array_equal(m["topk"], ref_top)
    np.testing.assert_array_equal(m["topk_Df"], Df[ref_top])
    np.testing.assert_array_equal(m["topk_cand"], bc[ref_top])
    assert (m["la_best_model"], m["la_best_cand"]) == divmod(int(np.argmin(cost.ravel())), C)
    assert m["n_nonfinite"] == G
    # NaN-ignore policy: nanargmin
    if seed % 2:
        parts2 = []
        for g, o in enumerate(parts):
            lo, hi = bounds[g], bounds[g + 1]
            j = lo + int(np.nanargmin(wm[lo:hi]))
            o.lb_best, o.lb_best_val = j, wm[j]
            parts2.append(o)
        m2 = nat.plan_out_to_dict(nat.merge(parts2, nat.NAN_IGNORE))
        assert m2["lb_best"] == int(np.nanargmin(wm))


def test_merge_window_filling_uses_owner_of_current_model():
    from llampc import _native as nat
    parts = []
    for g in range(3):
        o = nat.PlanOut()
        o.window_count, o.window_full, o.K = 4, 0, 10
        o.lb_best = -1
        for k in range(nat.KMAX):
            o.topk[k] = -1
        o.sel_model, o.sel_owned = 42, int(g == 1)
        o.sel_cand, o.sel_cost = (7, 1.5) if g == 1 else (-1, np.nan)
        o.la_best_model, o.la_best_cand, o.la_best_cost = 10 * g, g, float(3 - g)
        parts.append(o)
    m = nat.plan_out_to_dict(nat.merge(parts))
    assert m["sel_model"] == 42 and m["sel_owned"] and m["sel_cand"] == 7 and m["sel_cost"] == 1.5
    assert (m["la_best_model"], m["la_best_cand"], m["la_best_cost"]) == (20, 2, 1.0)
    assert list(m["topk"]) == [-1] * 10
    bad = nat.PlanOut()
    bad.K, bad.window_count = 10, 5
    with pytest.raises(nat.NativeError):
        nat.merge(parts + [bad])


# ------------------------------------------------------------------ host logic
def test_generate_bank_matches_reference_loop_and_shards():
    from llampc.mpc import generate_bank, shard_range
    np.testing.assert_array_equal(generate_bank(1000, 0), golden("bank_rt_seed0_n1000.npz")["bank"])
    np.testing.assert_array_equal(generate_bank(512, 7, sigma=2.0), golden("bank_wide_seed7_n512.npz")["bank"])
    for n, G in ((80000, 8), (10001, 8), (7, 2), (5, 4)):
        r = [shard_range(n, g, G) for g in range(G)]
        assert r[0][0] == 0 and r[-1][1] == n and all(r[i][1] == r[i + 1][0] for i in range(G - 1))


@pytest.mark.parametrize("name", ["ETHZ", "ETHZMobil"])
def test_product_planner_matches_reference_constant_speed(name):
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ, ETHZMobil
    tr = ETHZ('optimal', True) if name == "ETHZ" else ETHZMobil('optimal', True)
    g = golden("planner.npz")
    for case, xr in zip(g[f"{name}_cases"], g[f"{name}_xref"]):
        px, py, v0, pi, mu, scale, H, pidx, vr = case
        H = int(H)
        out, oidx, ovr = ConstantSpeed(np.array([px, py]), v0, tr, H, 0.02, int(pi), scale=scale, curr_mu=mu)
        np.testing.assert_allclose(out, xr[:, :H + 1], rtol=1e-10, atol=1e-12)
        assert oidx == pidx
        np.testing.assert_allclose(ovr, vr, rtol=1e-10)


@pytest.mark.parametrize("name", ["ETHZ", "ETHZMobil"])
def test_track_center_loader_matches_reference(name):
    """ETHZ/ETHZMobil(reference='center') — the reference's default — pinned to the
    reference's own objects (tracks_center.npz, gen_golden.py): the centre-line raceline and
    its spline knots, track length, theta_track, param_to_xy, xy_to_param and project on the
    closed centre line (closing segment = index -1), the init pose; ConstantSpeed on the
    centre line fails as the reference's does (no speed profiles: TypeError)."""
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ, ETHZMobil
    g = golden("tracks_center.npz")
    t = ETHZ() if name == "ETHZ" else ETHZMobil()
    assert t.reference == 'center' and t.mus is None
    np.testing.assert_array_equal(t.raceline, g[f"{name}_center_raceline"])
    np.testing.assert_allclose(t.spline.s, g[f"{name}_center_s"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose([t.x_init, t.y_init, t.psi_init, t.vx_init], g[f"{name}_center_init"], rtol=0)
    np.testing.assert_allclose(t.track_length, g[f"{name}_track_length"], rtol=1e-13)
    np.testing.assert_allclose(t.theta_track, g[f"{name}_theta_track"], rtol=1e-13, atol=1e-13)
    got = np.array([t.param_to_xy(th) for th in g[f"{name}_thetas"]])
    np.testing.assert_allclose(got, g[f"{name}_param_to_xy"], rtol=1e-12, atol=1e-13)
    for (px, py), th, pxy, pidx in zip(g[f"{name}_xy_points"], g[f"{name}_xy_to_param"],
                                       g[f"{name}_project_xy"], g[f"{name}_project_idx"]):
        xy, idx = t.project(px, py, t.center_line)
        assert idx == pidx
        np.testing.assert_allclose(xy, pxy, rtol=1e-12, atol=1e-13)
        np.testing.assert_allclose(t.xy_to_param(px, py), th, rtol=1e-12, atol=1e-12)
    assert str(g[f"{name}_center_constantspeed_error"]) == "TypeError"
    with pytest.raises(TypeError):
        ConstantSpeed(t.raceline[:, 5], 1.0, t, 5, 0.02, 0)


def test_track_txt_format_and_short_raceline():
    """The packaged lines equal what ETHZTrack.load_txt reads from a file in the reference's
    txt format (comma-separated x row / y row); ETHZ(reference='optimal', longer=False)
    loads the short raceline (6 friction profiles) and ConstantSpeed on it matches the
    reference; ETHZMobil has no short raceline (FileNotFoundError, as the reference)."""
    import tempfile
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ, ETHZMobil, ETHZTrack
    g = golden("tracks_center.npz")
    t = ETHZ()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        f.write("# x row, y row\n")
        for row in t.center:
            f.write(",".join(repr(float(v)) for v in row) + "\n")
    try:
        np.testing.assert_array_equal(ETHZTrack.load_txt(f.name), t.center)
    finally:
        os.unlink(f.name)
    assert t.inner.shape == t.outer.shape == t.center.shape and t.center.shape[0] == 2
    ts = ETHZ(reference='optimal', longer=False)
    np.testing.assert_allclose(ts.spline.s, g["ETHZ_short_s"], rtol=1e-13, atol=1e-13)
    np.testing.assert_array_equal(ts.mus, g["ETHZ_short_mus"])
    for case, xr in zip(g["ETHZ_short_cases"], g["ETHZ_short_xref"]):
        px, py, v0, pi, mu, scale, H, pidx, vr = case
        H = int(H)
        out, oidx, ovr = ConstantSpeed(np.array([px, py]), v0, ts, H, 0.02, int(pi), scale=scale, curr_mu=mu)
        np.testing.assert_allclose(out, xr[:, :H + 1], rtol=1e-10, atol=1e-12)
        assert oidx == pidx
        np.testing.assert_allclose(ovr, vr, rtol=1e-10)
    assert str(g["ETHZMobil_short_error"]) == "FileNotFoundError"
    with pytest.raises(FileNotFoundError):
        ETHZMobil(reference='optimal', longer=False)
    with pytest.raises(NotImplementedError):
        ETHZ(reference='inner')


def test_spline_coefficients_match_reference_dense_solve():
    from llampc.utils import Spline
    tr = np.load(os.path.join(REPO, "lla-mpc_amd/llampc/tracks/data/tracks.npz"))
    s = tr["ETHZ_s"]
    v = tr["ETHZ_speeds"][3]
    ref = O.Spline1D(list(s), v)
    mine = Spline(s, v)
    np.testing.assert_allclose(mine.c, ref.c, rtol=1e-9, atol=1e-12)
    for t in np.linspace(0, s[-1], 97)[:-1]:
        np.testing.assert_allclose(mine.calc(t), ref.calc(t), rtol=1e-12)
    np.testing.assert_allclose(mine.calc(s[-1]), v[-1], rtol=1e-9)
    assert mine.calc(-1.0) is None and mine.calc(s[-1] + 1) is None
    assert mine.coefficients().shape == (4, len(s) - 1)


def test_projection_matches_reference():
    from llampc.utils import Projection
    rng = np.random.RandomState(0)
    for _ in range(200):
        p, a, b = rng.randn(3, 2)
        if rng.rand() < 0.2:
            p = a + (b - a) * rng.choice([-0.5, 0.0, 0.5, 1.0, 1.5])
        r_ref, d_ref = O.project_point(p, a, b)
        r, d = Projection([p], [a, b])
        np.testing.assert_allclose(r, r_ref, atol=1e-12)
        np.testing.assert_allclose(d, d_ref, atol=1e-12)


def test_candidate_generator_bounds_and_rate():
    from llampc.mpc import CandidateGenerator
    gen = CandidateGenerator(64, 20, seed=3)
    U = gen(None, np.array([0.3, 0.1]))
    assert U.shape == (64, 20, 2)
    assert O.candidates_feasible(U, np.array([0.3, 0.1]), [-0.1, -0.35], [1.0, 0.35], 5.0, 0.02).all()
    np.testing.assert_array_equal(U[0], np.tile([0.3, 0.1], (20, 1)))
    U2 = gen(U[5], U[5, 0])
    np.testing.assert_array_equal(U2[0, :-1], U[5, 1:])


def test_mu_estimator_and_friction_known_answers():
    from llampc.mpc import MuEstimator, update_friction, FRICTION_CASES
    g = golden("closed_loop.npz")
    p = O.orca_params()
    bank = g["bank"]
    mu = MuEstimator(mass=p["mass"], lf=p["lf"], lr=p["lr"])
    for idt in range(g["u"].shape[1]):
        if idt <= 10:
            mu.warmup()
        else:
            tk = g["topk"][idt - 1]
            mu.update(bank[5][tk], bank[2][tk])
            assert mu.mu_pred == g["mu_pred"][idt]
        assert mu.mu_logged[-1] == g["mu_logged"][idt]
    ans = golden("mus_known_answers.npz")
    for key, case in (("LLA_CASE2GRADAFTER", "ETHZ_gradual"), ("LLA_CASE4SUDDAFTER_22", "ETHZ_sudden"),
                      ("LLA_CASE3SUDDBEG_22", "ETHZ_sudden_begin"), ("LLAT2_CASE2GRADAFTER", "ETHZMobil_gradual"),
                      ("LLA_CASE5CONSTANT", "nominal")):
        style, kw = FRICTION_CASES[case]
        Df, Dr, out = p["Df"], p["Dr"], []
        for i in range(len(ans[key])):
            Df, Dr = update_friction(Df, Dr, i * 0.02, style, **kw)
            out.append((Df + Dr) / (9.81 * p["mass"]))
        np.testing.assert_array_equal(np.array(out), ans[key])


def test_oracle_not_imported_by_product():
    """Product sources never reference the oracle (it is test infrastructure)."""
    root = os.path.join(REPO, "lla-mpc_amd")
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".h")):
                assert "oracle" not in open(os.path.join(dp, f)).read(), f


def test_div6_correctly_rounded():
    """fastmath.hpp div6: q = RN(v * RN(1/6)); r = v - 6q (exact by FMA); RN(q + r * RN(1/6))
    equals RN(v / 6) (Markstein's theorem).  Exact rational arithmetic on random values
    over the whole exponent range plus the neighbours of multiples of 6."""
    from fractions import Fraction as F
    y = F(1.0 / 6.0)
    rng = np.random.default_rng(7)
    vals = list(rng.standard_normal(20000) * 10.0 ** rng.integers(-300, 300, 20000))
    vals += [float(np.nextafter(6.0 * k, s)) for k in range(1, 500) for s in (0.0, np.inf)]
    vals += [1.0, -1.0, 6.0, 3.0, 2.0 ** -1000, 1e308]
    for v in vals:
        q = float(F(v) * y)
        r = F(v) - 6 * F(q)
        assert float(r) == r                       # the FMA residual is exact
        assert float(F(q) + r * y) == v / 6.0, v


def test_setupnlp_interface_cpu():
    """llampc.mpc.nmpc.setupNLP keeps nmpc.py:16's constructor; construction touches no
    device (one instance per bank model, rt.py:195-202); track_cons=True is refused."""
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.params import ORCA
    p = ORCA(control="pwm")
    m = Dynamic(**p)
    nlps = [setupNLP(20, 0.02, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, m, None) for _ in range(50)]
    assert all(n._bank is None for n in nlps)
    assert nlps[0].rate[0] == (None, None) and np.allclose(nlps[0].rate[1], (-0.1, 0.1))
    with pytest.raises(NotImplementedError):
        setupNLP(20, 0.02, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, m, None, track_cons=True)


def test_raceline_npz_reader_reference_format(tmp_path):
    """Raceline.from_raceline_npz reads the reference's raceline file layout
    (ethz.py:59-96 keys x, y, speed, time, speeds, mus) into the same splines and device
    tables as the packaged library; a file without ``speeds`` gets one profile."""
    from llampc.tracks import ETHZ, Raceline
    ref = ETHZ('optimal', True)
    n = ref.raceline.shape[1]
    f = tmp_path / "ethz_raceline_long_.npz"
    np.savez(f, x=ref.x_raceline, y=ref.y_raceline, speed=ref.v_raceline[0], time=np.arange(n) * 0.02,
             speeds=ref.v_raceline, mus=ref.mus)
    tr = Raceline.from_raceline_npz(f, name="ETHZ", track_width=0.37, psi_init=-np.pi / 4, lap_projidx=656)
    for a, b in zip(tr.device_table(), ref.device_table()):
        np.testing.assert_array_equal(a, b)
    assert tr.length == ref.length and tr.lap_projidx == 656
    f2 = tmp_path / "single.npz"
    np.savez(f2, x=ref.x_raceline, y=ref.y_raceline, speed=ref.v_raceline[3], time=np.arange(n) * 0.02)
    one = Raceline.from_raceline_npz(f2)
    assert one.v_raceline.shape == (1, n) and list(one.mus) == [1.0]


def test_exchange_probe_record_merge_and_mode(monkeypatch):
    """The peer transport's setup probe: the host merge of probe records is the global
    top-K by value; LLAMPC_EXCHANGE selects the transport (bad values refused)."""
    from llampc import _native as nat
    from llampc.mpc.sharded import exchange_mode, probe_record, records_equal
    parts = [probe_record(r, 4) for r in range(4)]
    m = nat.merge(parts)
    want = sorted((parts[r].topk_val[j], parts[r].topk[j]) for r in range(4) for j in range(10))[:10]
    assert [m.topk[j] for j in range(10)] == [i for _, i in want]
    assert m.n_nonfinite == 0 + 1 + 2 + 3 and m.status == 0
    assert records_equal(m, nat.merge(parts)) and not records_equal(m, parts[0])
    monkeypatch.delenv("LLAMPC_C10D_EXCHANGE", raising=False)
    monkeypatch.setenv("LLAMPC_EXCHANGE", "bogus")
    with pytest.raises(ValueError):
        exchange_mode()
    monkeypatch.setenv("LLAMPC_EXCHANGE", "rccl")
    assert exchange_mode() == "rccl"
    monkeypatch.setenv("LLAMPC_C10D_EXCHANGE", "1")
    assert exchange_mode() == "c10d"


def test_plan_in_builder_pointers_and_fields():
    """The host tick's PlanIn (ModelBank._plan_in, no device needed): every input pointer
    addresses its own values in the packed array, defaults come from the template, and each
    non-default argument lands in its field."""
    import ctypes as C
    from llampc import _native as nat
    from llampc.mpc.bank import ModelBank
    rng = np.random.RandomState(3)
    x_prev, u_prev, x_now, uprev = rng.randn(6), rng.randn(2), rng.randn(6), rng.randn(2)
    U, xref = rng.randn(3, 7, 2), rng.randn(2, 8)

    def read(addr, n):
        return np.ctypeslib.as_array((C.c_double * n).from_address(addr)).copy()

    pin, keep = ModelBank._plan_in(None, x_prev, u_prev, x_now, U, xref, uprev, 0.02, 10, "rk4",
                                   True, True, 0, nat.NAN_FIRST, None)
    for addr, want in ((pin.x_prev, x_prev), (pin.u_prev, u_prev), (pin.x_now, x_now),
                       (pin.uprev, uprev), (pin.xref, xref.ravel()), (pin.U, U.ravel())):
        np.testing.assert_array_equal(read(addr, want.size), want)
    assert (pin.C, pin.H, pin.K, pin.integrator, pin.do_lookback, pin.do_lookahead) == (3, 7, 10, nat.RK4, 1, 1)
    assert (pin.nan_policy, pin.current_model, pin.Ts, pin.xref_mode) == (nat.NAN_FIRST, 0, 0.02, nat.XREF_GIVEN)
    assert bytes(pin.cost) == bytes(nat.default_cost())
    cost = nat.cost_struct(enforce_bounds=True)
    pin, keep = ModelBank._plan_in(None, None, None, list(x_now), U[0], None, uprev, 0.01, 4, "euler_nlp",
                                   False, True, 17, nat.NAN_IGNORE, cost, (1.5, 2.0, 0.9))
    np.testing.assert_array_equal(read(pin.x_prev, 6), np.zeros(6))
    np.testing.assert_array_equal(read(pin.x_now, 6), x_now)
    np.testing.assert_array_equal(read(pin.xref, 4), [1.5, 2.0, 0.9, 0.0])
    np.testing.assert_array_equal(read(pin.U, 14), U[0].ravel())
    assert (pin.C, pin.H, pin.K, pin.integrator, pin.do_lookback) == (1, 7, 4, nat.EULER_NLP, 0)
    assert (pin.nan_policy, pin.current_model, pin.Ts, pin.xref_mode) == (nat.NAN_IGNORE, 17, 0.01, nat.XREF_RACELINE)
    assert bytes(pin.cost) == bytes(cost)


def test_bench_spawn_ranks_environment_and_failure():
    """bench.py's self-spawn of `--gpus N` (no launcher): every rank gets torchrun's
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1) and one shared FileStore
    path for the rendezvous (LLAMPC_INIT_FILE: no port to race for),
    the parent's status is 0 when all ranks succeed, and when one rank fails the others are
    stopped and its exit status is returned (CPU only: the ranks are stand-in scripts)."""
    import importlib.util
    import sys
    import tempfile
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    with tempfile.TemporaryDirectory() as tmp:
        ok = ("import os, sys; open(os.path.join(%r, os.environ['RANK']), 'w').write("
              "' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'LLAMPC_INIT_FILE')))") % tmp
        assert bench.spawn_ranks(3, [sys.executable, "-c", ok]) == 0
        got = [open(os.path.join(tmp, str(r))).read().split() for r in range(3)]
        assert [g[:4] for g in got] == [[str(r), str(r), "3", "127.0.0.1"] for r in range(3)]
        assert len({g[4] for g in got}) == 1
        fail = ("import os, sys, time\n"
                "if os.environ['RANK'] == '1': sys.exit(3)\n"
                "time.sleep(60)\n")
        import time
        t0 = time.time()
        assert bench.spawn_ranks(3, [sys.executable, "-c", fail]) == 3
        assert time.time() - t0 < 30            # the sleeping ranks were stopped, not waited for


def test_native_exchange_fallback_reported(monkeypatch):
    """The library's RCCL communicator (llampc_comm_*) cannot be made — here: no HIP device, so
    ncclGetUniqueId fails — ShardedBank keeps the c10d / host gather, reports the transport and
    says why in transport_fallback (the bench line carries both); with a communicator it takes
    'rccl'.  Every step is decided over the ranks (here a one-rank stand-in group)."""
    from llampc.mpc import sharded

    monkeypatch.setattr(sharded, "_all_gather_obj", lambda obj, group=None: [obj])

    def fresh(fallback=None):
        sb = sharded.ShardedBank.__new__(sharded.ShardedBank)
        sb._mailbox, sb._comm, sb.backend = None, None, "nccl"
        sb.rank, sb.world, sb.device, sb.group = 0, 1, 0, None
        sb.fallback_reason = fallback
        return sb

    sb = fresh("peer: IPC unavailable")
    sb._setup_native_exchange("cpu")           # the real library: RCCL loads, no device for its id
    assert sb._comm is None and sb._decide_transport() == "c10d"
    assert sb.fallback_reason.startswith("peer: IPC unavailable; rccl: llampc error")

    class Lib:                                 # a library whose RCCL works
        def llampc_comm_unique_id(self, buf):
            buf[0] = 7
            return 0

        def llampc_comm_create(self, uid, world, rank, dev, out):
            assert bytes(uid)[0] == 7 and (world, rank, dev) == (1, 0, 0)
            out._obj.value = 1234
            return 0

    monkeypatch.setattr(sharded.nat, "load", lambda: Lib())
    sb = fresh()
    sb._setup_native_exchange("cpu")
    assert sb._decide_transport() == "rccl" and sb.fallback_reason is None and sb.comm.value == 1234
    sb.backend = "gloo"
    sb._comm = None
    assert sb._decide_transport() == "host"


def test_controller_oracle_restatement():
    """The device controller's CPU restatement (oracle ControllerOracle, the checker of
    tests/test_ctl_gpu.py) against the reference's pieces it composes, in closed loop: its
    reference equals ConstantSpeed (planner.py:12-67) with the tick's mu / scale / projidx and
    the lap wrap of rt.py:287-296, its start arc length is the reference's own sum, its
    candidates respect the bounds and the rate bound, mu-hat follows rt.py:326-344."""
    from llampc.mpc import generate_bank
    from llampc.mpc.planner import ConstantSpeed
    from llampc.tracks import ETHZ
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td["ETHZ_x"], td["ETHZ_y"], td["ETHZ_speeds"], td["ETHZ_mus"])
    tr = ETHZ('optimal', True)
    p = O.orca_params()
    sh = {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
    bank = generate_bank(64, seed=21)
    W = 3
    orc = O.ControllerOracle(sh, bank, ref, tr.lap_projidx, H=12, C=6, K=4, W=W)
    np.testing.assert_array_equal(orc.prefix, tr.ctl_table()[1])
    x = golden("dyn_slice.npz")["states"][:, 0].copy()
    plant = O.Vehicle.from_params(p)
    projidx, mus = 0, O.MuEstimator(mass=sh["mass"], lf=sh["lf"], lr=sh["lr"])
    for t in range(9):
        o = orc.tick(x)
        assert (o["mu_used"], o["scale_used"]) == ((mus.mu_pred, 0.9) if t > W + 1 else (1.0, 1.0))
        host, hidx, _ = ConstantSpeed(x[:2], x[3], tr, 12, 0.02, projidx, scale=o["scale_used"], curr_mu=o["mu_used"])
        np.testing.assert_allclose(o["xref"], host, rtol=0, atol=1e-12)
        assert o["projidx"] == (0 if hidx > tr.lap_projidx else hidx)
        assert O.candidates_feasible(o["U"], np.zeros(2) if t == 0 else u, [-0.1, -0.35], [1.0, 0.35], 5.0, 0.02).all()
        if o["warm"]:
            mus.warmup()
        else:
            mus.update(bank[5][o["topk"]], bank[2][o["topk"]])
            assert o["mu_pred"] == mus.mu_pred
        projidx = o["projidx"]
        u = o["u_seq"][:, 0].copy()
        xn, _ = O.sim_continuous(plant, x, u.reshape(2, 1), [0, 0.02])
        x = xn[:, -1]


def test_controller_guard_marks_only_device_failures():
    """LLAMPC._guarded: a tick the library refused before launching anything (an
    argument or state error) leaves the host mirror and the controller usable; a tick that failed
    on the device (LLAMPC_E_DEVICE: a wait that expired or timed out; a record with a status)
    consumed its step — t advances and the controller refuses further ticks."""
    from llampc import _native as nat
    from llampc.mpc.controller import LLAMPC
    ctl = LLAMPC.__new__(LLAMPC)
    ctl.failed, ctl.t = None, 5

    def boom(code):
        def f():
            raise nat.NativeError("x", code)
        return f

    for code in (nat.E_ARG, nat.E_STATE):
        with pytest.raises(nat.NativeError):
            ctl._guarded(boom(code))
        assert (ctl.failed, ctl.t) == (None, 5)
    ctl._usable()
    with pytest.raises(nat.NativeError):
        ctl._guarded(boom(nat.E_DEVICE))
    assert (ctl.failed, ctl.t) == (5, 6)
    with pytest.raises(nat.NativeError, match="unusable"):
        ctl._usable()
