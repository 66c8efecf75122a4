"""``setupNLP`` drop-in: the selected model's NMPC solved by sampling on the GPU.

The reference (llampc/mpc/nmpc.py:14-203) transcribes the problem for CasADi/IPOPT:
states x[6, H+1] with x_{k+1} = x_k + Ts f_nlp(x_k, u_k) (dynamic.py:195-226 +
nmpc.py:58-60), objective (x_H - xref_H)' P (.) + sum_k [(x_{k+1} - xref_{k+1})' Q (.) +
du_k' R du_k], du_0 = u_0 - uprev (nmpc.py:44-111), bounds on u and on the steering rate
(nmpc.py:102-105).  CasADi and IPOPT are not available on this platform (and IPOPT's
optimum is not reproducible here: parity unpinned), so this ``solve()``
keeps the interface and the problem but searches it by sampling: ``samples`` control
sequences per round around the best so far (the warm start first: the previous solution
shifted one step), every one rolled out with the NLP's own Euler transcription and scored
with the NLP's objective by the look-ahead kernel (``ModelBank.lookahead``,
integrator ``euler_nlp``, infeasible sequences cost +inf), ``iters`` rounds with the
spread shrinking.  Every returned ``umpc`` satisfies the NLP's bounds and rate
constraints; ``fval`` is the objective of ``umpc`` and ``xmpc`` its Euler trajectory —
the same triple IPOPT's feasible point would give.

``track_cons=True`` (rt.py:63 uses False) needs the track-boundary half-planes
(constraints.py Boundary on the centre line), which are not packaged: it raises.
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
                 samples=1024, iters=4, sigma=(0.08, 0.04), shrink=0.5, seed=0, device=0):
        if track_cons:
            raise NotImplementedError("track_cons=True needs the track boundary data "
                                      "(constraints.py Boundary), which is not packaged")
        self.horizon, self.Ts = int(horizon), float(Ts)
        self.params, self.model, self.track, self.track_cons = params, model, track, track_cons
        self.samples, self.iters, self.shrink = int(samples), int(iters), float(shrink)
        self.sigma = np.asarray(sigma, dtype=np.float64)
        self.rng = np.random.RandomState(seed)
        self.device = device
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
        self._dyn = None
        self._last = None            # previous umpc [H, 2] for the warm start

    # the device objects are created at the first solve(): rt.py builds one setupNLP per
    # bank model (rt.py:195-202) but solves with one of them per tick
    def _ensure(self):
        if self._bank is not None:
            return
        m = self.model
        p6 = np.array([[float(_attr(m, k))] for k in _PACEJKA])
        shared = {k: float(_attr(m, k, 0.0) or 0.0) for k in SHARED_KEYS}
        approx = any(_attr(m, k) is None for k in ("Bf", "Br", "Df", "Dr")) or bool(_attr(m, "approx", False))
        if approx:
            p6 = np.nan_to_num(p6)
        self._bank = ModelBank(p6, shared=shared, W=1, device=self.device,
                               input_acc=bool(_attr(m, "input_acc", False)), approx=approx)
        from llampc.models import Dynamic
        kw = dict(shared)
        kw.update({k: (None if approx and k in ("Bf", "Br", "Df", "Dr") else float(p6[i, 0]))
                   for i, k in enumerate(_PACEJKA)})
        self._dyn = Dynamic(**kw, input_acc=bool(_attr(m, "input_acc", False)), device=self.device)

    def _sample(self, base, uprev, sigma, extra):
        """``samples`` sequences [C, H, 2] around ``base`` [H, 2] (row 0 = base itself, then
        ``extra`` rows), clipped to the input bounds, then to the rate bounds in order."""
        C, H = self.samples, self.horizon
        U = np.repeat(base[None], C, axis=0)
        k = 1 + len(extra)
        for j, e in enumerate(extra):
            U[1 + j] = e
        if C > k:
            U[k:] += self.rng.randn(C - k, H, 2) * sigma
        U = np.clip(U, self.umin, self.umax)
        for j, (lo, hi) in enumerate(self.rate):
            if lo is None:
                continue
            prev = np.full(C, float(uprev[j]))
            for h in range(H):
                U[:, h, j] = np.clip(U[:, h, j], prev + lo, prev + hi)
                prev = U[:, h, j]
        return np.ascontiguousarray(U)

    def solve(self, x0, xref, uprev):
        """-> (umpc [2, H], fval, xmpc [6, H+1], violation in {0, 0.02}) as nmpc.py:161-203."""
        self._ensure()
        H = self.horizon
        x0 = np.asarray(x0, dtype=np.float64).ravel()
        xref = np.ascontiguousarray(np.asarray(xref, dtype=np.float64)[:2, :H + 1])
        uprev = np.asarray(uprev, dtype=np.float64).ravel()
        hold = np.tile(uprev, (H, 1))
        base = hold if self._last is None else np.concatenate([self._last[1:], self._last[-1:]])
        best_U, best_J = None, np.inf
        sigma = self.sigma.copy()
        for it in range(self.iters):
            extra = [hold] if it == 0 and self._last is not None else []
            U = self._sample(base, uprev, sigma, extra)
            r = self._bank.lookahead(x0, U, xref, uprev, Ts=self.Ts, cost=self.cost, integrator="euler_nlp")
            c, J = r["best_cand"], r["best_cost"]
            if best_U is None or J < best_J:
                best_U, best_J = U[c].copy(), J
            base = best_U
            sigma = sigma * self.shrink
        traj = self._dyn._native_integrate(x0[None], best_U[None], np.full(H, self.Ts), nat.EULER_NLP,
                                           final_only=False)
        self._last = best_U
        return best_U.T.copy(), float(best_J), traj[:, 0, :].T.copy(), 0.0

    def close(self):
        if self._bank is not None:
            self._bank.close()
            self._bank = None
