"""Closed-loop LLA-MPC controller around the GPU bank: the caller side of ``plan()``.

Host logic restated from the reference driver (llampc/mpc/run_nmpc_orca_llampc_rt.py):
  * ``update_friction``      friction schedules (rt.py:125-141; windows per track/case)
  * ``ExponentialSmoother``  rt.py:103-113
  * ``MuEstimator``          mu-hat from the top-K models (rt.py:326-344)
  * ``CandidateGenerator``   sampled control sequences for the look-ahead (new; replaces
                             the per-tick IPOPT solve of nmpc.py:161-203 by candidate search)
  * ``LLAMPC.tick``          one tick in rt.py order: look-back on the newest transition,
                             mu-hat, ConstantSpeed reference with mu-hat (rt.py:278-282),
                             look-ahead, chosen control.  While the window fills (tick <= W)
                             the look-ahead plans with the NOMINAL model, as the reference's
                             nlp_initial (rt.py:207, 300-301); afterwards with the bank's
                             selected model (nlp_bank[current_model_idx], rt.py:303).
    mode="device" (default): the whole tick is ONE kernel launch (``DeviceController``,
                             llampc_ctl_tick): the reference trajectory (projection + the
                             prefix arc-length table + ConstantSpeed with mu-hat), the
                             candidates (Philox sampling), look-back + selection, the
                             look-ahead of the selected model and the top-K, mu-hat and the
                             controller state all on the GPU; the host passes x_t and reads
                             the record.  prelaunch=True (default): each tick's launch is
                             enqueued during the previous tick and waits for x_t on a
                             doorbell, having done the look-back's RK4 step (it needs only the
                             state) — the tick rings it (llampc_ctl_set_prelaunch).
    mode="host":             the round-3 loop: host ConstantSpeed + host CandidateGenerator
                             around the fused plan launch, every (model, candidate) rolled out.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from llampc import _native as nat
from llampc.mpc.bank import BANK_ORDER, ModelBank
from llampc.mpc.plan import PlanResult, result_from_out
from llampc.mpc.planner import ConstantSpeed

FRICTION_CASES = {
    # (style, params) reproducing results/**/MUs.npy of the reference runs
    "ETHZ_gradual": ("const_decay", dict(start=14.3)),
    "ETHZ_sudden": ("sudden", dict(window=(14.3, 14.5))),
    "ETHZ_sudden_begin": ("sudden", dict(window=(3.3, 3.5))),
    "ETHZMobil_gradual": ("const_decay", dict(start=5.0)),
    "ETHZMobil_sudden": ("sudden", dict(window=(5.0, 5.2))),
    "nominal": ("no_change", {}),
}


def update_friction(Df, Dr, curr_time, style="sudden", start=14.3, window=(14.3, 14.5)):
    """rt.py:125-141: 'const_decay' D -= D/2600 per tick after ``start``; 'sudden'
    D -= D/22 per tick strictly inside ``window``; 'no_change'."""
    if style == "const_decay":
        if curr_time > start:
            Df -= Df / 2600.
            Dr -= Dr / 2600.
    elif style == "sudden":
        if window[0] < curr_time < window[1]:
            Df -= Df / 22.
            Dr -= Dr / 22.
    return Df, Dr


class ExponentialSmoother:
    def __init__(self, alpha=0.3):
        self.alpha = alpha
        self.smooth_value = None

    def update(self, new_value):
        if self.smooth_value is None:
            self.smooth_value = new_value
        else:
            self.smooth_value = self.alpha * new_value + (1 - self.alpha) * self.smooth_value
        return self.smooth_value


@dataclass
class MuEstimator:
    """rt.py:326-344.  While the window fills (tick <= W) the Dr/Df histories take the
    nominal mu_init split (with g = 9.8, rt.py:327-328); afterwards the top-K mean."""
    mass: float
    lf: float
    lr: float
    mu_init: float = 1.0
    S: int = 20                      # smoothing_mu (rt.py:68)
    alpha: float = 0.08              # mu_alpha (rt.py:72)
    dr_hist: list = field(default_factory=list)
    df_hist: list = field(default_factory=list)
    mu_pred: float | None = None
    mu_logged: list = field(default_factory=list)

    def __post_init__(self):
        self.smoother = ExponentialSmoother(self.alpha)

    def warmup(self):
        self.dr_hist.append(self.mu_init * self.mass * 9.8 * self.lr / (self.lf + self.lr))
        self.df_hist.append(self.mu_init * self.mass * 9.8 * self.lf / (self.lf + self.lr))
        self.mu_logged.append(self.mu_init)

    def record(self, dr_mean, df_mean, mu_pred, warm):
        """The device controller's update of this tick (it computed the same values on the
        GPU, ctl.hip ctl_complete): the histories, mu-hat and the logged smoothed value."""
        self.dr_hist.append(dr_mean)
        self.df_hist.append(df_mean)
        if warm:
            self.mu_logged.append(self.mu_init)
        else:
            self.mu_pred = mu_pred
            self.mu_logged.append(self.smoother.update(mu_pred) * .95)

    def update(self, topk_Dr, topk_Df) -> float:
        self.dr_hist.append(np.mean(topk_Dr))
        self.df_hist.append(np.mean(topk_Df))
        dr = np.mean(np.array(self.dr_hist)[-self.S:])
        df = np.mean(np.array(self.df_hist)[-self.S:])
        self.mu_pred = (dr + df) / (9.81 * self.mass)
        self.mu_logged.append(self.smoother.update(self.mu_pred) * .95)
        return self.mu_pred


class CandidateGenerator:
    """C control sequences [C, H, 2] for the look-ahead: candidate 0 is the previous
    choice shifted one step (warm start); the rest add N(0, diag(sig^2)) noise, clipped to
    the input bounds and to the steering-rate bound |d delta| <= rate*Ts (orca.py:29-35,
    nmpc.py:102-105).  Seeded."""

    def __init__(self, C, H, Ts=0.02, sigma=(0.05, 0.02), umin=(-0.1, -0.35), umax=(1.0, 0.35),
                 rate_max=(None, 5.0), seed=2):
        self.C, self.H, self.Ts = C, H, Ts
        self.sigma = np.asarray(sigma, dtype=np.float64)
        self.umin, self.umax = np.asarray(umin, dtype=np.float64), np.asarray(umax, dtype=np.float64)
        self.rate = [None if r is None else r * Ts for r in rate_max]
        self.rng = np.random.RandomState(seed)

    def __call__(self, prev_seq, uprev):
        """prev_seq [H, 2] (or None), uprev [2] -> U [C, H, 2]."""
        H = self.H
        if prev_seq is None:
            base = np.tile(np.asarray(uprev, dtype=np.float64), (H, 1))
        else:
            prev_seq = np.asarray(prev_seq, dtype=np.float64)
            base = np.concatenate([prev_seq[1:], prev_seq[-1:]], axis=0)
        U = np.repeat(base[None], self.C, axis=0)
        if self.C > 1:
            U[1:] += self.rng.randn(self.C - 1, H, 2) * self.sigma
        U = np.clip(U, self.umin, self.umax)
        for j, r in enumerate(self.rate):
            if r is None:
                continue
            prev = np.full(self.C, float(uprev[j]))
            for k in range(H):
                U[:, k, j] = np.clip(U[:, k, j], prev - r, prev + r)
                prev = U[:, k, j]
        return np.ascontiguousarray(U)


class DeviceController:
    """Handle of llampc_ctl (include/llampc.h): the control step of rt.py:278-366 as ONE launch
    on the bank's device, the controller state (x_{t-1}, u_{t-1}, the chosen sequence,
    projidx, mu-hat histories, current model) resident there between ticks.  The bank must
    not be ticked by anything else while the controller drives it."""

    def __init__(self, bank: ModelBank, track, H=20, C=64, K=10, Ts=0.02, v_factor=0.9, mu_init=1.0, S=20,
                 sigma=(0.05, 0.02), seed=2, nominal6=None, cost=None, nan_policy=nat.NAN_FIRST,
                 debug_inputs=False, lap_projidx=None, prelaunch=False):
        if getattr(bank, "raceline", None) is not track:
            bank.set_raceline(track)
        self.bank, self.track, self.H, self.C = bank, track, int(H), int(C)
        cfg = nat.CtlCfg()
        cfg.C, cfg.H, cfg.K, cfg.nan_policy = int(C), int(H), int(K), int(nan_policy)
        cfg.Ts, cfg.v_factor, cfg.mu_init, cfg.S = float(Ts), float(v_factor), float(mu_init), int(S)
        cfg.lap_projidx = int(track.lap_projidx if lap_projidx is None else lap_projidx)
        cfg.sigma[0], cfg.sigma[1] = float(sigma[0]), float(sigma[1])
        cfg.seed = int(seed)
        if nominal6 is None:
            from llampc.params import ORCA
            nominal6 = [ORCA(control='pwm')[k] for k in BANK_ORDER]
        for j, v in enumerate(nominal6):
            cfg.nominal[j] = float(v)
        cfg.cost = cost if cost is not None else nat.cost_struct(enforce_bounds=True)
        cfg.debug_inputs = int(bool(debug_inputs))
        pts, prefix = track.ctl_table()
        h = nat.C.c_void_p()
        nat.check(nat.load().llampc_ctl_create(bank.handle, nat.C.byref(cfg), nat.dptr(pts), pts.shape[1],
                                               nat.dptr(prefix), nat.C.byref(h)))
        self._h = h
        self.cfg = cfg
        self._x = np.zeros(6)
        lib = nat.load()
        self._xp = self._x.ctypes.data
        self._f_async, self._f_wait = lib.llampc_ctl_tick_async, lib.llampc_ctl_wait
        self._carrier = None                 # a ShardedBank whose process group carries the exchange
        self.transport = None                # the sharded exchange's transport (set_exchange)
        self.prelaunch = False
        if prelaunch:
            self.set_prelaunch(True)

    def set_prelaunch(self, on=True):
        """Arm every next tick (llampc_ctl_set_prelaunch): its launch is enqueued behind the
        current one and waits for x_t on a doorbell, so the next ``tick`` only rings it — the
        launch call and the dispatch leave the step's latency.  Any other call on the bank or
        this controller cancels the armed launch first (the tick after it launches normally)."""
        nat.check(nat.load().llampc_ctl_set_prelaunch(self._h, int(bool(on))))
        self.prelaunch = bool(on)

    def device_us(self) -> float:
        """The last completed tick's device time (llampc_ctl_device_us): x_t on the device (the
        doorbell seen, or the launch started) to the record's stores issued, in microseconds by
        the GPU's 100 MHz clock; NaN before the first tick."""
        v = ctypes.c_double()
        nat.check(nat.load().llampc_ctl_device_us(self._h, ctypes.byref(v)))
        return v.value

    def tick(self, x_t, out=None) -> "nat.CtlOut":
        """One blocking step; ``out`` (a CtlOut) is filled and returned (a new one if None)."""
        out = nat.CtlOut() if out is None else out
        x = self._x
        x[:] = x_t
        if self._carrier is not None:        # the host carries the exchange between the launches
            self.tick_async(x_t)
            return self.wait(out)
        nat.check(nat.load().llampc_ctl_tick(self._h, x.ctypes.data, nat.C.addressof(out)))
        return out

    def tick_async(self, x_t):
        self._x[:] = x_t
        rc = self._f_async(self._h, self._xp)
        if rc:
            nat.check(rc)

    def wait(self, out=None) -> "nat.CtlOut":
        out = nat.CtlOut() if out is None else out
        if self._carrier is not None:
            self._carry()
        rc = self._f_wait(self._h, nat.C.addressof(out))
        if rc:
            nat.check(rc)
        return out

    def _carry(self):
        """The host-carried exchange of a gathered tick (llampc_ctl_shard_record / _resume): this
        rank's record after the first launch, the group's all-gather, the second launch."""
        lib = nat.load()
        nw = nat.C.c_int32()
        nat.check(lib.llampc_ctl_shard_record(self._h, self._words.ctypes.data, nat.C.byref(nw)))
        if nw.value == 0:                    # no exchange on this tick (the window is not full)
            return
        allw = np.ascontiguousarray(self._carrier.gather_words(self._words[:nw.value]))
        nat.check(lib.llampc_ctl_resume(self._h, allw.ctypes.data))

    def set_exchange(self, sharded):
        """Tick this controller as one rank of a SHARDED bank: ``sharded`` is this rank's
        ShardedBank (its shard is the bank this controller drives).  Every rank then holds the
        unsharded controller's selection, record and state.  Call on every rank before the first
        tick.  The transport is the ShardedBank's: its peer mailboxes (llampc_ctl_set_exchange: the
        exchange inside the tick's one launch), its RCCL communicator (llampc_ctl_set_gather: two
        launches with ncclAllGather between them on the bank's stream), or the process group on
        the host (c10d / host: llampc_ctl_set_gather without a communicator, the records carried
        by ``wait``)."""
        if sharded.bank is not self.bank:
            raise ValueError("the controller must drive the ShardedBank's own shard")
        pg = sharded.params_global
        lib = nat.load()
        if sharded.mailbox is not None:
            nat.check(lib.llampc_ctl_set_exchange(self._h, sharded.mailbox, nat.dptr(pg), int(pg.shape[1])))
            self.transport = "peer"
        else:
            comm = sharded.comm
            nat.check(lib.llampc_ctl_set_gather(self._h, int(sharded.world), int(sharded.rank), comm, nat.dptr(pg),
                                                int(pg.shape[1])))
            if comm is None:
                self._carrier = sharded
                self._words = np.zeros(int(lib.llampc_ctl_record_words(int(self.cfg.K))), dtype=np.uint64)
            self.transport = "rccl" if comm is not None else sharded.transport
        self._gparams = pg

    def inputs(self):
        """The last tick's reference xref [2, H+1] and candidates U [C, H, 2] (debug_inputs)."""
        xref = np.empty((2, self.H + 1))
        U = np.empty((self.C, self.H, 2))
        nat.check(nat.load().llampc_ctl_inputs(self._h, nat.dptr(xref), nat.dptr(U)))
        return xref, U

    def reference(self, x0, v0, H, projidx, curr_mu=1., scale=1.):
        """ConstantSpeed(x0, v0, track, H, Ts, projidx, scale, curr_mu) (planner.py:12-67)
        evaluated by the device code the controller ticks with -> (xref [2, H+1], projidx, vr)."""
        xref = np.empty((2, int(H) + 1))
        pj, vr = nat.C.c_int32(), nat.C.c_double()
        nat.check(nat.load().llampc_ctl_reference(self._h, nat.dptr(nat.f64(np.asarray(x0)[:2])), float(v0), int(H),
                                                  int(projidx), float(curr_mu), float(scale), nat.dptr(xref),
                                                  nat.C.byref(pj), nat.C.byref(vr)))
        return xref, pj.value, vr.value

    def close(self):
        if getattr(self, "_h", None) is not None:
            nat.load().llampc_ctl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_PLAN_DT = np.dtype(nat.PlanOut)


class CtlResult:
    """A controller tick's result: PlanResult's fields over the llampc_ctl_out record, the
    arrays (top-K, u_seq) views of the record built on first use — a 1 kHz loop that reads
    only the first control does not pay for NumPy arrays it never touches."""
    __slots__ = ("raw", "H", "best_model", "window_full", "window_count", "best_cand", "cost",
                 "n_nonfinite", "nominal", "mu_hat", "_kk", "_rec", "_u")
    lookback_err = window_mean = costs = None

    def __init__(self, o: "nat.CtlOut", H: int):
        p = o.plan
        if p.status:
            raise nat.NativeError(f"tick record status {p.status}: the in-launch completion timed out")
        self.raw, self.H = o, int(H)
        self.best_model, self.best_cand, self.cost = p.sel_model, p.sel_cand, p.sel_cost
        self.window_full = bool(p.window_full) and p.lb_best >= 0
        self.window_count, self.n_nonfinite = p.window_count, p.n_nonfinite
        self.nominal = bool(o.warm)
        mu = o.mu_pred
        self.mu_hat = None if mu != mu else mu
        self._kk = -1
        self._rec = self._u = None

    def _field(self, name):
        if self._rec is None:
            self._rec = np.frombuffer(self.raw, np.uint8, count=_PLAN_DT.itemsize).view(_PLAN_DT)[0]
            # the record pads top-K with -1 when the bank holds fewer than K models
            # (argsort()[:K], rt.py:360, returns only those entries)
            self._kk = int(np.count_nonzero(self._rec["topk"][:self.raw.plan.K] >= 0))
        return self._rec[name][:self._kk]

    topk = property(lambda self: self._field("topk") if self.window_full else None)
    topk_err = property(lambda self: self._field("topk_val") if self.window_full else None)
    topk_Df = property(lambda self: self._field("topk_Df") if self.window_full else None)
    topk_Dr = property(lambda self: self._field("topk_Dr") if self.window_full else None)

    @property
    def u_seq(self):
        """[2, H] the chosen control sequence (a view of the record)."""
        if self._u is None:
            self._u = np.frombuffer(self.raw.u_seq, np.float64, count=2 * self.H).reshape(self.H, 2).T
        return self._u

    @property
    def u0(self):
        """The control applied this tick, (u_seq[0, 0], u_seq[1, 0])."""
        r = self.raw.u_seq[0]
        return (r[0], r[1])

    @property
    def global_best(self):
        p = self.raw.plan
        return (p.la_best_model, p.la_best_cand, p.la_best_cost)


def result_from_ctl(o: "nat.CtlOut", H: int) -> CtlResult:
    """The result of a controller tick: the record plus the chosen sequence [2, H]."""
    return CtlResult(o, H)


class LLAMPC:
    """Stateful LLA-MPC tick loop over a ``ModelBank`` (rt.py:269-366 without IPOPT).

    ``nominal``: the Pacejka parameters the warm-up ticks plan with (default ORCA(),
    the reference's true_model / params at setup, rt.py:78-79, 207).  ``prelaunch``: device
    mode's armed ticks (module docstring); results are those of launched ticks."""

    def __init__(self, bank: ModelBank, track, H=20, Ts=0.02, K=10, C=64, v_factor=0.9,
                 mu_init=1.0, S=20, alpha=0.08, cost=None, integrator="rk4", seed=2,
                 nan_policy=nat.NAN_FIRST, nominal: dict | None = None, mode="device",
                 sigma=(0.05, 0.02), debug_inputs=False, prelaunch=True):
        from llampc.params import ORCA
        if mode not in ("device", "host"):
            raise ValueError(f"mode={mode!r}: 'device' or 'host'")
        self.mode = mode
        # a ShardedBank: this rank's controller over its shard, exchanging the selection with the
        # other ranks every tick (device mode; BASELINE config 5 across GPUs)
        sharded = bank if hasattr(bank, "params_global") and hasattr(bank, "bank") else None
        if sharded is not None:
            if mode != "device":
                raise ValueError("a sharded bank needs mode='device' (the exchange runs inside the tick's launch)")
            bank = sharded.bank
        self.sharded = sharded
        self.bank, self.track = bank, track
        nominal = ORCA(control='pwm') if nominal is None else nominal
        col = np.array([[float(nominal[k])] for k in BANK_ORDER])
        self.nominal_bank = None
        self._ctl = None
        if mode == "device":
            if integrator != "rk4":
                raise ValueError("the device controller rolls out with RK4 (use mode='host' for other integrators)")
            self._ctl = DeviceController(bank, track, H=H, C=C, K=K, Ts=Ts, v_factor=v_factor, mu_init=mu_init,
                                         S=S, sigma=sigma, seed=seed, nominal6=col[:, 0],
                                         cost=cost if cost is not None else nat.cost_struct(enforce_bounds=True),
                                         nan_policy=nan_policy, debug_inputs=debug_inputs)
            if sharded is not None and sharded.exchange:
                self._ctl.set_exchange(sharded)
                if prelaunch and self._ctl.transport == "peer":
                    # an armed launch needs the bank's own (dedicated-queue) stream, not the
                    # ShardedBank's torch stream of plan() ticks (the shard is the controller's alone)
                    bank.set_stream(None)
                    self._ctl.set_prelaunch(True)
            elif prelaunch:
                self._ctl.set_prelaunch(True)
        else:
            # a one-model bank: the warm-up look-ahead runs the same kernel on the nominal model
            self.nominal_bank = ModelBank(col, shared=bank.shared, W=1, device=bank.device)
        self.H, self.Ts, self.K, self.W = H, Ts, K, bank.W
        self.v_factor = v_factor
        sh = bank.shared
        self.mu = MuEstimator(mass=sh["mass"], lf=sh["lf"], lr=sh["lr"], mu_init=mu_init, S=S, alpha=alpha)
        self.cost = cost if cost is not None else nat.cost_struct(enforce_bounds=True)
        self.integrator = integrator
        self.gen = CandidateGenerator(C, H, Ts, seed=seed)
        self.nan_policy = nan_policy
        self._last = self._last_full = None
        self._u_seq_host = self._u_prev_host = self._topk_host = None
        self.current_model = 0          # rt.py:264
        self.projidx = 0
        self.t = 0
        self.failed = None              # the tick that failed on the device (device mode), if any
        self.x_prev = None
        self.u_prev = None
        self.u_seq = None
        self.last_topk = None

    def set_prelaunch(self, on=True):
        """Device mode: arm every next tick (the default; DeviceController.set_prelaunch) or not.
        A sharded controller arms over the peer transport only (the gather transports run two
        launches per tick)."""
        if self._ctl is None:
            return
        if self.sharded is not None and self.sharded.exchange:
            if self._ctl.transport != "peer":
                return
            if on and not self._ctl.prelaunch:
                self.bank.set_stream(None)
        self._ctl.set_prelaunch(on)

    def device_us(self) -> float:
        """Device mode: the last tick's device time (DeviceController.device_us); else NaN."""
        return self._ctl.device_us() if self._ctl is not None else float("nan")

    def tick(self, x_t) -> PlanResult:
        """One control tick.  After the warm-up (t > W) it is ONE fused launch on the bank:
        look-back on the newest transition (rt.py:347-349), window + argmin + top-K
        (rt.py:352-366), and the look-ahead of every (model, candidate), the selected
        model's best candidate being the chosen control (rt.py:300-305).  While the window
        fills (t <= W) the look-ahead plans with the nominal model (rt.py:300-301), so the
        tick is the bank's look-back plus a one-model look-ahead (two launches).
        Raises NativeError if the selected model is not on this bank (a shard of a larger
        bank: use ShardedBank, whose merged record carries the owner's choice)."""
        x_t = np.asarray(x_t, dtype=np.float64)
        if self.mode == "device":
            return self._tick_device(x_t)
        t = self.t
        warm = t <= self.W
        # 1. reference (rt.py:278-282); it uses the mu-hat of the previous tick because
        #    the reference updates mu-hat after its solve (rt.py:326-344)
        if t > self.W + 1:
            xref, self.projidx, _ = ConstantSpeed(x_t[:2], x_t[3], self.track, self.H, self.Ts,
                                                  self.projidx, curr_mu=self.mu.mu_pred,
                                                  scale=self.v_factor)
        else:
            xref, self.projidx, _ = ConstantSpeed(x_t[:2], x_t[3], self.track, self.H, self.Ts,
                                                  self.projidx)
        if self.projidx > self.track.lap_projidx:              # lap wrap (rt.py:287-296)
            self.projidx = 0
        uprev = np.zeros(2) if self.u_prev is None else self.u_prev
        U = self.gen(self.u_seq, uprev)
        if warm:
            # 2w. look-back on the bank (the reference scores transition idt -> idt+1 for
            #     idt >= 1, so tick t >= 2 here; rt.py:347), look-ahead with the nominal model
            lb = None
            if t >= 2:
                lb = self.bank.lookback(self.x_prev, self.u_prev, x_t, Ts=self.Ts, K=self.K,
                                        nan_policy=self.nan_policy)
            o, _, _, _ = self.nominal_bank.plan_raw(np.zeros(6), np.zeros(2), x_t, U, xref, uprev,
                                                    Ts=self.Ts, K=self.K, integrator=self.integrator,
                                                    do_lookback=False, do_lookahead=True, current_model=0,
                                                    cost=self.cost)
            res = result_from_out(o, U)
            res.best_model = self.current_model
            res.window_count = lb["window_count"] if lb is not None else self.bank.window_count
            self.mu.warmup()                                   # rt.py:326-330
        else:
            # 2. ONE launch: look-back + selection + look-ahead of every (model, candidate);
            #    the record carries the selected model's best candidate (rt.py:303-305)
            o, _, _, _ = self.bank.plan_raw(self.x_prev, self.u_prev, x_t, U, xref, uprev, Ts=self.Ts,
                                            K=self.K, integrator=self.integrator, do_lookback=True,
                                            do_lookahead=True, current_model=self.current_model,
                                            nan_policy=self.nan_policy, cost=self.cost)
            res = result_from_out(o, U)
            if not res.window_full:
                raise nat.NativeError(f"tick {t}: the look-back window is not full after the warm-up "
                                      "(was the bank reset?)")
            if res.u_seq is None:
                raise nat.NativeError(
                    f"tick {t}: the selected model {res.best_model} is not on this bank "
                    f"(models [{self.bank.global_offset}, {self.bank.global_offset + self.bank.n})); "
                    "a shard's controller needs the merged record (ShardedBank)")
            self.current_model = res.best_model
            if res.window_full:
                self.last_topk = res.topk
                # 3. mu-hat from this look-back's top-K Df/Dr (rt.py:331-344); the record
                #    carries them, -1 padding (a bank of fewer than K models) already cut
                self.mu.update(res.topk_Dr, res.topk_Df)
        res.nominal = warm
        res.mu_hat = self.mu.mu_pred
        self.u_seq = res.u_seq.T
        self.x_prev = x_t
        self.u_prev = res.u_seq[:, 0].copy()
        self.t += 1
        return res

    def tick_begin(self, x_t):
        """Device mode: enqueue the tick (llampc_ctl_tick_async) and return at once, so the
        controllers of several banks (e.g. two tracks) run concurrently; tick_end() completes it."""
        if self.mode != "device":
            raise nat.NativeError("tick_begin/tick_end need mode='device'")
        self._usable()
        self._pending_x = x = np.array(x_t, dtype=np.float64)
        self._ctl.tick_async(x)

    def tick_end(self) -> PlanResult:
        return self._guarded(lambda: self._finish_device(self._ctl.wait(), self._pending_x))

    def _tick_device(self, x_t) -> PlanResult:
        """ONE launch (llampc_ctl_tick): the device computes the reference, the candidates, the
        look-back, the look-ahead of the selected and top-K models, mu-hat and its state."""
        self._usable()
        return self._guarded(lambda: self._finish_device(self._ctl.tick(x_t), x_t))

    def _usable(self):
        if self.failed is not None:
            raise nat.NativeError(f"controller unusable after the failed tick {self.failed}: a failed tick still "
                                  "consumed its step on the device (window slot, tick number); rebuild the "
                                  "bank and the controller")

    def _guarded(self, fn):
        """A device tick that failed on the device (a wait that timed out or expired: LLAMPC_E_DEVICE;
        a HIP error; a record with status != 0) has still advanced the device controller's tick and
        window: the host mirror records the step (t advances) and the controller refuses further
        ticks.  A call the library refused before launching anything (an argument or
        state error: LLAMPC_E_ARG / E_STATE) consumed no step and is re-raised as it is."""
        try:
            return fn()
        except nat.NativeError as e:
            if e.code in (nat.E_ARG, nat.E_STATE, nat.E_OOM, nat.E_NODEV):
                raise
            self.failed = self.t
            self.t += 1
            raise
        except Exception:
            self.failed = self.t
            self.t += 1
            raise

    def _finish_device(self, o, x_t) -> CtlResult:
        res = CtlResult(o, self.H)
        self.mu.record(o.dr_mean, o.df_mean, o.mu_pred, res.nominal)
        res.mu_hat = self.mu.mu_pred
        if res.window_full:
            self._last_full = res
        self.current_model = res.best_model
        self.projidx = o.projidx
        self._last = res
        self.x_prev = x_t
        self.t += 1
        return res

    # device mode keeps the last result; these read it on demand
    last_topk = property(lambda self: self._last_full.topk if self._last_full is not None else self._topk_host,
                         lambda self, v: setattr(self, "_topk_host", v))
    u_seq = property(lambda self: self._last.u_seq.T if self._last is not None else self._u_seq_host,
                     lambda self, v: setattr(self, "_u_seq_host", v))
    u_prev = property(lambda self: self._last.u_seq[:, 0].copy() if self._last is not None else self._u_prev_host,
                      lambda self, v: setattr(self, "_u_prev_host", v))

    def inputs(self):
        """Device mode with debug_inputs=True: the last tick's xref [2, H+1] and U [C, H, 2]."""
        return self._ctl.inputs()

    def close(self):
        if self._ctl is not None:
            self._ctl.close()
        if self.nominal_bank is not None:
            self.nominal_bank.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
