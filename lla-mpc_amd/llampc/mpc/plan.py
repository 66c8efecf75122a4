"""``plan()`` — one LLA-MPC tick on the GPU (new API).

Encodes the order of the reference tick (run_nmpc_orca_llampc_rt.py:300-366):
  1. look-back: score every model on the newest transition (x_{t-1}, u_{t-1}) -> x_t
     (evaluate_models_vectorized.py:4-24), update the W-window, and when it is full
     select argmin + top-K (rt.py:347-366);
  2. look-ahead: roll every (model, candidate control sequence) out over H steps from x_t
     and evaluate the NLP objective (model.py:32-40 composed H times; nmpc.py:44-111);
  3. the chosen control sequence is the best candidate of the selected model.
The reference scores the transition at the end of tick t-1; doing it at the start of tick
t is the same computation on the same data.

All three run as one fused launch sequence in libllampc_hip (llampc_plan).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from llampc import _native as nat
from llampc.mpc.bank import ModelBank


@dataclass
class PlanResult:
    best_model: int                 # selected model (global index)
    window_full: bool
    window_count: int
    topk: np.ndarray | None         # argsort(window mean)[:K] (rt.py:360), None until full
    topk_err: np.ndarray | None
    topk_Df: np.ndarray | None
    topk_Dr: np.ndarray | None
    best_cand: int                  # argmin_c cost[best_model, c]
    u_seq: np.ndarray | None        # [2, H] chosen control sequence (U[best_cand].T)
    cost: float
    global_best: tuple              # (model, cand, cost) over all pairs
    n_nonfinite: int
    mu_hat: float | None = None
    lookback_err: np.ndarray | None = None
    window_mean: np.ndarray | None = None
    costs: np.ndarray | None = None
    raw: object = None              # the llampc_plan_out record
    nominal: bool = False           # LLAMPC warm-up tick: planned with the nominal model


def result_from_out(o: nat.PlanOut, U=None, **extra) -> PlanResult:
    d = nat.plan_out_to_dict(o)
    if d.get("status", 0):
        raise nat.NativeError(f"tick record status {d['status']}: the in-launch completion timed out")
    full = d["window_full"] and d["lb_best"] >= 0
    # the record pads top-K with -1 when the bank holds fewer than K models; argsort()[:K]
    # (rt.py:360) returns only those n entries
    kk = int(np.count_nonzero(d["topk"] >= 0)) if full else 0
    u_seq = None
    if U is not None and d["sel_cand"] >= 0:
        u_seq = np.ascontiguousarray(np.asarray(U)[d["sel_cand"]].T)
    return PlanResult(
        best_model=int(d["sel_model"]), window_full=full, window_count=d["window_count"],
        topk=d["topk"][:kk] if full else None, topk_err=d["topk_val"][:kk] if full else None,
        topk_Df=d["topk_Df"][:kk] if full else None, topk_Dr=d["topk_Dr"][:kk] if full else None,
        best_cand=int(d["sel_cand"]), u_seq=u_seq, cost=float(d["sel_cost"]),
        global_best=(int(d["la_best_model"]), int(d["la_best_cand"]), float(d["la_best_cost"])),
        n_nonfinite=int(d["n_nonfinite"]), raw=o, **extra)


def plan(bank: ModelBank, x_t, u_prev, x_prev, xref, U_cand, uprev=None, Ts=0.02, K=10,
         current_model=0, integrator="rk4", cost=None, nan_policy=nat.NAN_FIRST,
         do_lookback=True, return_errors=False, return_window_mean=False,
         return_costs=False, raceline_start=None) -> PlanResult:
    """One tick.  x_t [6]; (x_prev [6], u_prev [2]) the previous transition (pass
    do_lookback=False on the first tick, rt.py:347); xref [2, H+1]; U_cand [C, H, 2];
    uprev [2] is the input applied last (defaults to u_prev), used for du_0
    (nmpc.py:65-66); current_model is used while the window fills (rt.py:264).
    raceline_start = (s0, v0, scale) (planner.raceline_start, the bank's set_raceline track):
    per-model references from the device raceline lookup instead of the shared xref."""
    U = np.asarray(U_cand, dtype=np.float64)
    if U.ndim == 2:
        U = U[None]
    uprev = u_prev if uprev is None else uprev
    o, err, wm, costs = bank.plan_raw(
        x_prev if do_lookback else np.zeros(6), u_prev if do_lookback else np.zeros(2), x_t, U, xref,
        uprev, Ts=Ts, K=K, integrator=integrator, do_lookback=do_lookback, do_lookahead=True,
        current_model=current_model, nan_policy=nan_policy, cost=cost, return_errors=return_errors,
        return_window_mean=return_window_mean, return_costs=return_costs,
        raceline_start=raceline_start)
    return result_from_out(o, U, lookback_err=err,
                           window_mean=wm if (wm is not None and o.window_full) else None,
                           costs=costs)
