"""``setupNLP`` drop-in: the selected model's NMPC solved on the GPU by a cross-entropy search.

The reference (llampc/mpc/nmpc.py:14-203) transcribes the problem for CasADi/IPOPT:
states x[6, H+1] with x_{k+1} = x_k + Ts f_nlp(x_k, u_k) (dynamic.py:195-226 +
nmpc.py:58-60), objective (x_H - xref_H)' P (.) + sum_k [(x_{k+1} - xref_{k+1})' Q (.) +
du_k' R du_k], du_0 = u_0 - uprev (nmpc.py:44-111), bounds on u and on the steering rate
(nmpc.py:102-105).  CasADi and IPOPT are not available on this platform (and IPOPT's optimum
is not reproducible here: parity unpinned), so this ``solve()`` keeps the
interface and the problem and minimises it on the device (llampc_nlp_solve, csrc/nlp.hip):
``iters`` rounds of ``samples`` control sequences drawn around the current mean (the warm
start first: the previous solution shifted one step; the held uprev is a candidate of the
first round) with a per-(step, input) spread, clipped to the bounds and rate-clipped in order,
every one rolled out with the NLP's own Euler transcription and scored with its objective
(infeasible: +inf); the ``elite`` best set the next mean and spread (the cross-entropy
method).  All rounds run in ONE launch on the GPU (the sample blocks wait for each round's
mean and spread), the result comes back through pinned host memory.  Every returned
``umpc`` satisfies the NLP's bounds and rate constraints; ``fval`` is the objective of
``umpc`` and ``xmpc`` its Euler trajectory — the same triple IPOPT's feasible point would give.

``track_cons=True`` (rt.py:63 uses False everywhere) would add the track-boundary half-planes
of constraints.py; the boundary lines are packaged (llampc.tracks) but the constraint is not
implemented here (out of scope): it raises.
"""
from __future__ import annotations

import numpy as np

from llampc import _native as nat
from llampc.mpc.bank import ModelBank, SHARED_KEYS

_PACEJKA = ("Bf", "Cf", "Df", "Br", "Cr", "Dr")


def _attr(model, k, default=None):
    if isinstance(model, dict):
        return model.get(k, default)
    return getattr(model, k, default)


class setupNLP:
    """Same constructor and ``solve`` contract as nmpc.py:14-203 (see module doc)."""

    def __init__(self, horizon, Ts, Q, P, R, params, model, track, track_cons=False,
                 samples=1024, iters=8, elite=32, sigma=(0.3, 0.15), std_floor=1e-4, seed=0, device=0):
        if track_cons:
            raise NotImplementedError("track_cons=True (constraints.py boundary half-planes) is not "
                                      "implemented: the reference's LLA-MPC runs use TRACK_CONS=False (rt.py:63)")
        self.horizon, self.Ts = int(horizon), float(Ts)
        self.params, self.model, self.track, self.track_cons = params, model, track, track_cons
        self.samples, self.iters, self.elite = int(samples), int(iters), int(elite)
        self.sigma = np.asarray(sigma, dtype=np.float64)
        self.std_floor, self.seed, self.device = float(std_floor), int(seed), device
        self.umin = np.asarray(params["min_inputs"], dtype=np.float64)
        self.umax = np.asarray(params["max_inputs"], dtype=np.float64)
        # steering-rate bounds min_rates[1]*Ts <= d delta <= max_rates[1]*Ts (nmpc.py:104-105);
        # the pwm rate is unconstrained (None)
        rmin = [None if r is None else float(r) * self.Ts for r in params["min_rates"]]
        rmax = [None if r is None else float(r) * self.Ts for r in params["max_rates"]]
        self.rate = list(zip(rmin, rmax))
        # the kernel's feasibility test is symmetric |du| <= rate_max*Ts: use the tighter side
        rate_max = tuple(-1.0 if lo is None else min(-lo, hi) / self.Ts for lo, hi in self.rate)
        self.cost = nat.cost_struct(Q=Q, R=R, P=P, umin=self.umin, umax=self.umax,
                                    rate_max=rate_max, enforce_bounds=True)
        self._bank = None
        self._h = None
        self._dyn = None
        self._last = None            # previous umpc [H, 2] for the warm start

    # the device objects are created at the first solve(): rt.py builds one setupNLP per
    # bank model (rt.py:195-202) but solves with one of them per tick
    def _ensure(self):
        if self._h is not None:
            return
        m = self.model
        p6 = np.array([[float(_attr(m, k))] for k in _PACEJKA])
        shared = {k: float(_attr(m, k, 0.0) or 0.0) for k in SHARED_KEYS}
        approx = any(_attr(m, k) is None for k in ("Bf", "Br", "Df", "Dr")) or bool(_attr(m, "approx", False))
        if approx:
            p6 = np.nan_to_num(p6)
        self._bank = ModelBank(p6, shared=shared, W=1, device=self.device,
                               input_acc=bool(_attr(m, "input_acc", False)), approx=approx)
        cfg = nat.NlpCfg()
        cfg.H, cfg.samples, cfg.iters, cfg.elite = self.horizon, self.samples, self.iters, self.elite
        cfg.Ts, cfg.std_floor, cfg.seed = self.Ts, self.std_floor, self.seed
        cfg.sigma0[0], cfg.sigma0[1] = float(self.sigma[0]), float(self.sigma[1])
        cfg.cost = self.cost
        for j, (lo, hi) in enumerate(self.rate):
            cfg.rate_lo[j], cfg.rate_hi[j] = (1.0, -1.0) if lo is None else (lo, hi)
        h = nat.C.c_void_p()
        nat.check(nat.load().llampc_nlp_create(self._bank.handle, nat.C.byref(cfg), nat.C.byref(h)))
        self._h = h
        self.cfg = cfg
        H = self.horizon
        self._io = {"x0": np.zeros(6), "xref": np.zeros((2, H + 1)), "up": np.zeros(2), "base": np.zeros((H, 2)),
                    "umpc": np.zeros((H, 2)), "fval": np.zeros(1), "xmpc": np.zeros((H + 1, 6))}
        self._addr = {k: v.ctypes.data for k, v in self._io.items()}

    def solve(self, x0, xref, uprev):
        """-> (umpc [2, H], fval, xmpc [6, H+1], violation in {0, 0.02}) as nmpc.py:161-203."""
        self._ensure()
        b = self._io
        H = self.horizon
        # the inputs into the persistent buffers (their addresses cached at the first solve: the
        # per-call ctypes pointer objects cost more host time than the copies)
        b["x0"][:] = np.asarray(x0, dtype=np.float64).ravel()
        b["xref"][:] = np.asarray(xref, dtype=np.float64)[:2, :H + 1]
        b["up"][:] = np.asarray(uprev, dtype=np.float64).ravel()
        hold = self._last is not None
        if hold:                         # the warm start: the last solution shifted one step
            b["base"][:-1] = self._last[1:]
            b["base"][-1] = self._last[-1]
        a = self._addr
        nat.check(nat.load().llampc_nlp_solve(self._h, a["x0"], a["xref"], a["up"], a["base"] if hold else None,
                                               int(hold), a["umpc"], a["fval"], a["xmpc"]))
        umpc = b["umpc"].copy()
        self._last = umpc
        return umpc.T.copy(), float(b["fval"][0]), b["xmpc"].T.copy(), 0.0

    def close(self):
        if self._h is not None:
            nat.load().llampc_nlp_destroy(self._h)
            self._h = None
        if self._bank is not None:
            self._bank.close()
            self._bank = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
