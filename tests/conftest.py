"""Shared pytest setup: markers, import paths, golden-fixture loader."""
import os
import sys

import numpy as np
import pytest

# device kernel arguments, as bench.py (set before anything initialises HIP; llampc itself
# leaves the process environment alone)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "lla-mpc_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests proper")


def golden(name):
    """Load a committed fixture written by tests/golden/gen_golden.py (data only)."""
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold():
    return golden


# ---- look-ahead cost parity on ill-conditioned rollouts (DESIGN §4 "Tolerances") -------------
# The look-ahead rollouts evaluate atan2, atan and the tire / yaw sines with LEAN cores (8-term
# polynomials, a division without its residual step: fastmath.hpp), whose per-call relative error
# is ~1e-13 instead of NumPy's ~1e-16.  On a well-conditioned rollout that stays far below the
# tests' rtol; on an ill-conditioned one (config 3's Mobil states, the sigma = 2 bank) the
# rollout amplifies it, and NO fp64 evaluation whose roundings differ from NumPy's can be held
# to rtol there.  Such a pair is held to a bound derived from the kernel's own error model instead
# of a fitted constant: core_error_bound propagates the cores' MEASURED worst relative errors
# (lean_core_errors: the device's own cores against NumPy) through the oracle's rollout — every
# atan2 / atan / sin / cos result perturbed by +-its core's error, all signs up, all down and
# random sign patterns — and the pair may differ from the oracle by at most CORE_MARGIN times the
# largest cost change that produced, and never by more than the north star's 1e-5.
CORE_MARGIN = 2.0
NORTH_STAR_RTOL = 1e-5
_CORE_ERR = {}


def lean_core_errors() -> dict:
    """The worst relative error of the look-ahead's lean cores on the device (llampc_math_batch
    fn 10 atan2, 11 atan, 12 sin_wide) against NumPy over 2^18 arguments each from the rollouts'
    ranges (slip-angle ratios, |C atan| <= 2): {'atan2', 'atan', 'sin'}.  Measured once per
    session (it needs the GPU)."""
    if not _CORE_ERR:
        from llampc import _native as nat
        lib = nat.load()
        rng = np.random.RandomState(12)
        n = 1 << 18

        def run(fn, a, b=None):
            a = np.ascontiguousarray(a, dtype=np.float64)
            bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
            out = np.empty_like(a)
            nat.check(lib.llampc_math_batch(fn, a.ctypes.data, None if bb is None else bb.ctypes.data, a.size,
                                            out.ctypes.data, 0))
            return out

        def rel(got, want):
            m = np.abs(want) > 1e-300
            return float(np.max(np.abs(got[m] - want[m]) / np.abs(want[m])))

        y, x = rng.uniform(-3, 3, n), rng.uniform(1e-3, 4, n)
        z = np.concatenate([rng.uniform(-2, 2, n // 2), rng.standard_cauchy(n // 2) * 10])
        a = rng.uniform(-2, 2, n)
        _CORE_ERR.update(atan2=rel(run(10, y, x), np.arctan2(y, x)), atan=rel(run(11, z), np.arctan(z)),
                         sin=rel(run(12, a), np.sin(a)))
    return dict(_CORE_ERR)


class _PerturbedNumpy:
    """numpy with atan2 / atan / sin / cos results perturbed by relative errors +-eps (sign: +1,
    -1, or None = a random sign per element); every other attribute is numpy's."""

    def __init__(self, eps, sign, rng):
        self._eps, self._sign, self._rng = eps, sign, rng

    def __getattr__(self, k):
        return getattr(np, k)

    def _p(self, r, e):
        r = np.asarray(r, dtype=np.float64)
        sg = self._sign if self._sign is not None else self._rng.choice([-1.0, 1.0], size=r.shape)
        return r * (1.0 + sg * e)

    def arctan2(self, y, x):
        return self._p(np.arctan2(y, x), self._eps["atan2"])

    def arctan(self, z):
        return self._p(np.arctan(z), self._eps["atan"])

    def sin(self, a):
        return self._p(np.sin(a), self._eps["sin"])

    def cos(self, a):
        return self._p(np.cos(a), self._eps["sin"])


def core_error_bound(shared, cols6, x0, U, xref, uprev, Q, R, P, Ts=0.02, draws=4, seed=0):
    """[n_models * C]: CORE_MARGIN times the largest relative cost change of the oracle's RK4
    rollout + cost when every transcendental result carries its lean core's measured worst
    relative error (lean_core_errors) — all signs +, all -, and `draws` random sign patterns."""
    from oracle import llampc_oracle as O
    eps = lean_core_errors()
    x0 = np.asarray(x0, dtype=np.float64)
    rng = np.random.RandomState(seed)
    real = O.np
    with np.errstate(all="ignore"):
        c0 = O.mpc_cost(O.rollout_rk4(shared, cols6, x0, U, Ts), U, xref, uprev, Q, R, P)
        dev = np.zeros_like(c0)
        try:
            for sign in [1.0, -1.0] + [None] * draws:
                O.np = _PerturbedNumpy(eps, sign, rng)
                cj = O.mpc_cost(O.rollout_rk4(shared, cols6, x0, U, Ts), U, xref, uprev, Q, R, P)
                O.np = real
                dev = np.maximum(dev, np.abs(cj - c0) / np.abs(c0))
        finally:
            O.np = real
    return CORE_MARGIN * dev


def cost_sensitivity(shared, cols6, x0, U, xref, uprev, Q, R, P, Ts=0.02):
    """[n_models * C]: the oracle's relative cost change for a one-ulp change of x0 (the largest
    over its six components) of every (model column, candidate) pair — the conditioning of the
    pair as a diagnostic (DESIGN §4 reports it beside core_error_bound)."""
    from oracle import llampc_oracle as O
    x0 = np.asarray(x0, dtype=np.float64)
    with np.errstate(all="ignore"):
        c0 = O.mpc_cost(O.rollout_rk4(shared, cols6, x0, U, Ts), U, xref, uprev, Q, R, P)
        s = np.zeros_like(c0)
        for j in range(6):
            xp = x0.copy()
            xp[j] = np.nextafter(xp[j], np.inf)
            cj = O.mpc_cost(O.rollout_rk4(shared, cols6, xp, U, Ts), U, xref, uprev, Q, R, P)
            s = np.maximum(s, np.abs(cj - c0) / np.abs(c0))
    return s


def assert_costs_close(got, want, rtol, bound_fn):
    """got vs the oracle's want: the same NaN / finite pattern, then every finite pair within
    rtol — or, beyond it, within its core-error bound (bound_fn(flat indices) -> those pairs'
    allowed relative errors, core_error_bound; computed only for the pairs that need it) and
    within the north star's 1e-5.  Returns the number of pairs that needed the bound."""
    got, want = np.asarray(got, dtype=np.float64).ravel(), np.asarray(want, dtype=np.float64).ravel()
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    np.testing.assert_array_equal(np.isfinite(got), np.isfinite(want))
    fin = np.isfinite(want)
    rel = np.zeros_like(want)
    rel[fin] = np.abs(got[fin] - want[fin]) / np.maximum(np.abs(want[fin]), 1e-300)
    over = np.flatnonzero(fin & (rel > rtol))
    if over.size:
        b = np.asarray(bound_fn(over), dtype=np.float64)
        bad = (rel[over] > b) | (rel[over] > NORTH_STAR_RTOL)
        assert not bad.any(), (f"{int(bad.sum())} costs beyond rtol {rtol:g} and their core-error bound: "
                               f"rel {rel[over][bad][:5]}, bound {b[bad][:5]}, index {over[bad][:5]}")
    return int(over.size)
