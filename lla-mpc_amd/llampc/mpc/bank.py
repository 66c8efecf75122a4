"""Device-resident model bank (one shard) — the handle behind the look-back/look-ahead.

Replaces the reference's MODEL_BANK list of N ``Dynamic`` objects, its ``params_pass``
tuple (run_nmpc_orca_llampc_rt.py:161-179) and the ``error_windows`` array
(rt.py:83-84).  Parameters live on the GPU as SoA [6][N] (Bf, Cf, Df, Br, Cr, Dr);
the W-window is a slot-major ring [W][N] updated in place each tick.
"""
from __future__ import annotations

import numpy as np

from llampc import _native as nat
from llampc.params import ORCA

BANK_ORDER = ("Bf", "Cf", "Df", "Br", "Cr", "Dr")       # rt.py:179 params_pass order
VARIATION_ORDER = ("Br", "Cr", "Dr", "Bf", "Cf", "Df")  # rt.py:153-158 draw order
RT_SIGMA = {"Br": 0.2, "Cr": 0.1, "Dr": 0.5, "Bf": 0.2, "Cf": 0.1, "Df": 0.5}
SHARED_KEYS = ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")


def generate_bank(n: int, seed: int, sigma=None, nominal: dict | None = None) -> np.ndarray:
    """Seeded bank [6, n] with the reference's multiplicative Gaussian variation
    p <- p * (1 + sigma_p z) (rt.py:161-170).  z is drawn model-major in rt.py's
    parameter order, so ``np.random.seed(seed)`` + the reference loop gives the same bank;
    the whole global bank is drawn on every rank, so shards are partition-invariant."""
    if sigma is None:
        sigma = RT_SIGMA
    elif not isinstance(sigma, dict):
        sigma = {k: float(sigma) for k in VARIATION_ORDER}
    nominal = ORCA(control='pwm') if nominal is None else nominal
    z = np.random.RandomState(seed).randn(n, len(VARIATION_ORDER))
    bank = np.empty((6, n))
    for j, name in enumerate(VARIATION_ORDER):
        bank[BANK_ORDER.index(name)] = nominal[name] * (1 + sigma[name] * z[:, j])
    return bank


def shard_range(n_global: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of rank ``rank``; the remainder goes to the last rank."""
    per = n_global // world
    lo = rank * per
    hi = n_global if rank == world - 1 else lo + per
    return lo, hi


_Z6, _Z2 = np.zeros(6), np.zeros(2)


def _pin_template() -> "nat.PlanIn":
    """The PlanIn fields _plan_in leaves at their defaults unless asked (rk4, look-back and
    look-ahead, NAN_FIRST, current model 0, Ts 0.02, the rt.py cost, shared xref)."""
    pin = nat.PlanIn()
    pin.integrator = nat.RK4
    pin.do_lookback = pin.do_lookahead = 1
    pin.nan_policy = nat.NAN_FIRST
    pin.current_model = 0
    pin.Ts = 0.02
    pin.cost = nat.default_cost()
    pin.xref_mode = nat.XREF_GIVEN
    return pin


_PIN_TEMPLATE = _pin_template()


class ModelBank:
    """A shard of the model bank resident on one HIP device."""

    def __init__(self, params6, shared: dict | None = None, W: int = 10, device: int = 0,
                 global_offset: int = 0, input_acc: bool = False, approx: bool = False):
        params6 = np.ascontiguousarray(np.asarray(params6, dtype=np.float64).reshape(6, -1))
        self.params = params6
        self.n = params6.shape[1]
        self.W = int(W)
        self.device = int(device)
        self.global_offset = int(global_offset)
        shared = ORCA(control='pwm') if shared is None else shared
        self.shared = {k: float(shared[k]) for k in SHARED_KEYS}
        self._veh = nat.vehicle(*(self.shared[k] for k in SHARED_KEYS), input_acc=input_acc, approx=approx)
        lib = nat.load()
        h = nat.C.c_void_p()
        nat.check(lib.llampc_bank_create(nat.dptr(params6), self.n, self.global_offset,
                                         nat.C.byref(self._veh), self.W, self.device, nat.C.byref(h)))
        self._h = h

    # -------------------------------------------------------------- constructors
    @classmethod
    def from_models(cls, models, W=10, device=0, global_offset=0):
        """From a list of ``Dynamic`` objects (the reference's MODEL_BANK); shared
        constants come from models[0] as in evaluate_models_vectorized.py:15-21."""
        p = np.array([[getattr(m, k) for m in models] for k in BANK_ORDER], dtype=np.float64)
        m0 = models[0]
        return cls(p, {k: getattr(m0, k) for k in SHARED_KEYS}, W=W, device=device,
                   global_offset=global_offset, input_acc=m0.input_acc,
                   approx=bool(getattr(m0, "approx", False)))

    @classmethod
    def generate(cls, n, seed=0, sigma=None, W=10, device=0, rank=0, world=1):
        full = generate_bank(n, seed, sigma)
        lo, hi = shard_range(n, rank, world)
        return cls(full[:, lo:hi], W=W, device=device, global_offset=lo)

    # -------------------------------------------------------------- lifecycle
    @property
    def handle(self):
        if self._h is None:
            raise nat.NativeError("bank is closed")
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None:
            nat.load().llampc_bank_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, stream_ptr: int | None):
        nat.check(nat.load().llampc_bank_set_stream(self.handle, stream_ptr))

    def stream_handle(self) -> int:
        """The hipStream_t the bank launches on now.  Its own stream is a plain one until
        set_concurrency(> 1) or an armed controller (LLAMPC prelaunch) gives it a hardware queue
        of its own — which REPLACES the stream: a handle read before either call is destroyed
        (read it again; llampc_bank_stream)."""
        h = nat.C.c_void_p()
        nat.check(nat.load().llampc_bank_stream(self.handle, nat.C.byref(h)))
        return int(h.value or 0)

    def set_concurrency(self, banks: int):
        """The number of banks ticked concurrently on this device (default 1; two tracks
        ticked together: 2): each look-ahead launch is sized for 1/banks of the chip, so the
        concurrent launches are resident together (llampc_bank_set_concurrency)."""
        nat.check(nat.load().llampc_bank_set_concurrency(self.handle, int(banks)))

    @property
    def window_count(self) -> int:
        c = nat.C.c_int32()
        nat.check(nat.load().llampc_bank_info(self.handle, None, None, None, nat.C.byref(c), None))
        return c.value

    @property
    def launches(self) -> int:
        """Plan-kernel launches enqueued on this bank so far (one per tick entry point)."""
        c = nat.C.c_int64()
        nat.check(nat.load().llampc_bank_launches(self.handle, nat.C.byref(c)))
        return c.value

    def reset(self):
        nat.check(nat.load().llampc_bank_reset(self.handle))

    def window(self) -> np.ndarray:
        """The error window as rt.py keeps it: [N, W], newest in the last column."""
        ring = np.empty((self.n, self.W))
        nat.check(nat.load().llampc_bank_window(self.handle, nat.dptr(ring), None))
        return ring

    # -------------------------------------------------------------- hot path
    def lookback(self, x_prev, u_prev, x_now, Ts=0.02, K=10, nan_policy=nat.NAN_FIRST,
                 return_errors=False, return_window_mean=False) -> dict:
        """One look-back tick (evaluate_models_vectorized.py:4-24 + rt.py:347-366)."""
        err = np.empty(self.n) if return_errors else None
        wm = np.empty(self.n) if return_window_mean else None
        best = nat.C.c_int64()
        topk = np.full(K, -1, dtype=np.int64)
        topv = np.empty(K)
        cnt = nat.C.c_int32()
        nat.check(nat.load().llampc_lookback(
            self.handle, nat.dptr(nat.f64(x_prev)), nat.dptr(nat.f64(u_prev)), nat.dptr(nat.f64(x_now)),
            float(Ts), int(K), int(nan_policy), nat.dptr(err), nat.dptr(wm), nat.C.byref(best),
            topk.ctypes.data_as(nat.C.POINTER(nat.C.c_int64)), nat.dptr(topv), nat.C.byref(cnt)))
        full = cnt.value >= self.W
        return dict(best=best.value if full else None, topk=topk if full else None,
                    topk_val=topv if full else None, window_count=cnt.value, full=full,
                    errors=err, window_mean=wm if full else None)

    def lookahead(self, x0, U, xref, uprev, Ts=0.02, cost=None, integrator="rk4",
                  return_costs=False, return_best_cand=False) -> dict:
        """Roll every (model, candidate) over H steps and evaluate the NLP objective
        (model.py:32-40 x H + nmpc.py:44-111).  U [C, H, 2]; xref [2, H+1]."""
        U = nat.f64(U)
        if U.ndim == 2:
            U = U.reshape(1, *U.shape)
        C_, H = U.shape[0], U.shape[1]
        xref = nat.f64(xref)
        if xref.shape != (2, H + 1):
            raise ValueError(f"xref must be [2, {H + 1}], got {xref.shape}")
        cost = cost if cost is not None else nat.cost_struct()
        costs = np.empty((self.n, C_)) if return_costs else None
        bc = np.empty(self.n, dtype=np.int32) if return_best_cand else None
        bm, bcand, bcost = nat.C.c_int64(), nat.C.c_int32(), nat.C.c_double()
        nat.check(nat.load().llampc_lookahead(
            self.handle, nat.dptr(nat.f64(x0)), nat.dptr(U), C_, H, nat.dptr(xref),
            nat.dptr(nat.f64(uprev)), nat.C.byref(cost), float(Ts), nat.INTEGRATORS[integrator],
            nat.dptr(costs), None if bc is None else bc.ctypes.data_as(nat.C.POINTER(nat.C.c_int32)),
            nat.C.byref(bm), nat.C.byref(bcand), nat.C.byref(bcost)))
        return dict(best_model=bm.value, best_cand=bcand.value, best_cost=bcost.value, costs=costs,
                    best_cand_per_model=bc)

    def set_raceline(self, track):
        """Attach ``track``'s raceline library (llampc_bank_set_raceline) for
        xref_mode='raceline' ticks: every model then tracks its own ConstantSpeed reference
        with mu_n = (Df_n + Dr_n) / (9.81 m)."""
        knots, xy, speed, mus = track.device_table()
        nat.check(nat.load().llampc_bank_set_raceline(self.handle, nat.dptr(knots), len(knots), nat.dptr(xy),
                                                      nat.dptr(speed), nat.dptr(mus), len(mus)))
        self.raceline = track

    def _plan_in(self, x_prev, u_prev, x_now, U, xref, uprev, Ts, K, integrator, do_lookback,
                 do_lookahead, current_model, nan_policy, cost, raceline_start=None):
        """raceline_start = (s0, v0, scale): xref_mode RACELINE (xref is then unused)."""
        if raceline_start is not None:
            xref = np.array([*map(float, raceline_start), 0.0])
        U = nat.f64(U)
        if U.ndim == 2:
            U = U.reshape(1, *U.shape)
        # one packed array, one address lookup (~1 us each in NumPy): pointers = base + offsets;
        # the constant fields come from a per-bank template (a struct copy, not ~15 setattrs)
        flat = (np.ravel(_Z6 if x_prev is None else x_prev), np.ravel(_Z2 if u_prev is None else u_prev),
                np.ravel(x_now), np.ravel(uprev), np.ravel(xref), U.reshape(-1))
        pack = np.concatenate(flat)
        if pack.dtype != np.float64:
            pack = pack.astype(np.float64)
        keep = [pack]
        base = pack.ctypes.data
        o1 = flat[0].size
        o2 = o1 + flat[1].size
        o3 = o2 + flat[2].size
        o4 = o3 + flat[3].size
        o5 = o4 + flat[4].size
        pin = nat.PlanIn.from_buffer_copy(_PIN_TEMPLATE)
        pin.x_prev, pin.u_prev, pin.x_now = base, base + 8 * o1, base + 8 * o2
        pin.uprev, pin.xref, pin.U = base + 8 * o3, base + 8 * o4, base + 8 * o5
        pin.C, pin.H, pin.K = U.shape[0], U.shape[1], int(K)
        if integrator != "rk4":
            pin.integrator = nat.INTEGRATORS[integrator]
        if not (do_lookback and do_lookahead):
            pin.do_lookback, pin.do_lookahead = int(bool(do_lookback)), int(bool(do_lookahead))
        if nan_policy:
            pin.nan_policy = int(nan_policy)
        if current_model:
            pin.current_model = int(current_model)
        if Ts != 0.02:
            pin.Ts = float(Ts)
        if cost is not None:
            pin.cost = cost
        if raceline_start is not None:
            pin.xref_mode = nat.XREF_RACELINE
        return pin, keep

    def plan_raw(self, x_prev, u_prev, x_now, U, xref, uprev, Ts=0.02, K=10, integrator="rk4",
                 do_lookback=True, do_lookahead=True, current_model=0, nan_policy=nat.NAN_FIRST,
                 cost=None, return_errors=False, return_window_mean=False, return_costs=False,
                 raceline_start=None):
        """The fused tick (llampc_plan): returns (PlanOut, errors, window_mean, costs)."""
        pin, keep = self._plan_in(x_prev, u_prev, x_now, U, xref, uprev, Ts, K, integrator,
                                  do_lookback, do_lookahead, current_model, nan_policy, cost,
                                  raceline_start)
        C_ = pin.C
        err = np.empty(self.n) if return_errors else None
        wm = np.empty(self.n) if return_window_mean else None
        costs = np.empty((self.n, C_)) if return_costs else None
        out = nat.PlanOut()
        nat.check(nat.load().llampc_plan(self.handle, nat.C.byref(pin), nat.C.byref(out), nat.dptr(err),
                                         nat.dptr(wm), nat.dptr(costs)))
        return out, err, wm, costs

    def plan_async(self, x_prev, u_prev, x_now, U, xref, uprev, Ts=0.02, K=10, integrator="rk4",
                   do_lookback=True, do_lookahead=True, current_model=0, nan_policy=nat.NAN_FIRST,
                   cost=None, raceline_start=None):
        """Enqueue one tick (llampc_plan_async): inputs are staged before return, the tick
        runs on the bank's stream; ``plan_wait()`` returns its PlanOut.  Independent banks
        (e.g. one per track) overlap on the device."""
        pin, keep = self._plan_in(x_prev, u_prev, x_now, U, xref, uprev, Ts, K, integrator,
                                  do_lookback, do_lookahead, current_model, nan_policy, cost,
                                  raceline_start)
        nat.check(nat.load().llampc_plan_async(self.handle, nat.C.byref(pin)))

    def plan_wait(self):
        out = nat.PlanOut()
        nat.check(nat.load().llampc_plan_wait(self.handle, nat.C.byref(out)))
        return out
