"""ctypes binding of libllampc_hip.so (include/llampc.h).

The product path has no CPU fallback: if the HIP library is missing or no HIP device is
visible, every compute call raises ``NativeError`` / ``NoDeviceError``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libllampc_hip.so")

KMAX = 32
WMAX = 128
RK4, EULER_NLP, RK6 = 0, 1, 2
INTEGRATORS = {"rk4": RK4, "euler_nlp": EULER_NLP, "rk6": RK6}
NAN_FIRST, NAN_IGNORE = 0, 1
XREF_GIVEN, XREF_RACELINE = 0, 1
OP_FORCES, OP_DERIV = 0, 1
E_ARG, E_HIP, E_NODEV, E_STATE, E_OOM, E_DEVICE = -1, -2, -3, -4, -5, -6


class NativeError(RuntimeError):
    """A libllampc_hip call failed (message = llampc_last_error(); ``code`` = its LLAMPC_E_* return
    code, None when raised by the Python layer)."""

    def __init__(self, msg="", code=None):
        super().__init__(msg)
        self.code = code


class NoDeviceError(NativeError):
    """No HIP device is visible; there is deliberately no CPU fallback."""


class Vehicle(C.Structure):
    _fields_ = [("lf", C.c_double), ("lr", C.c_double), ("mass", C.c_double), ("Iz", C.c_double),
                ("Cm1", C.c_double), ("Cm2", C.c_double), ("Cr0", C.c_double), ("Cr2", C.c_double),
                ("input_acc", C.c_int32), ("approx", C.c_int32)]


class Cost(C.Structure):
    _fields_ = [("Q", C.c_double * 4), ("R", C.c_double * 4), ("P", C.c_double * 4),
                ("umin", C.c_double * 2), ("umax", C.c_double * 2), ("rate_max", C.c_double * 2),
                ("enforce_bounds", C.c_int32), ("reserved", C.c_int32)]


_dp = C.POINTER(C.c_double)


class PlanIn(C.Structure):
    # the pointer members are declared void* (same C layout as llampc_plan_in's const
    # double*): the host assigns raw addresses, which is ~10x cheaper than ctypes casts
    _fields_ = [("x_prev", C.c_void_p), ("u_prev", C.c_void_p), ("x_now", C.c_void_p),
                ("U", C.c_void_p), ("xref", C.c_void_p), ("uprev", C.c_void_p),
                ("C", C.c_int32), ("H", C.c_int32), ("K", C.c_int32),
                ("integrator", C.c_int32), ("do_lookback", C.c_int32), ("do_lookahead", C.c_int32),
                ("nan_policy", C.c_int32), ("xref_mode", C.c_int32), ("current_model", C.c_int64),
                ("Ts", C.c_double), ("cost", Cost)]


class PlanOut(C.Structure):
    _fields_ = [("window_count", C.c_int32), ("window_full", C.c_int32), ("K", C.c_int32),
                ("sel_owned", C.c_int32), ("lb_best", C.c_int64), ("lb_best_val", C.c_double),
                ("sel_model", C.c_int64), ("sel_cand", C.c_int32), ("n_nonfinite", C.c_int32),
                ("sel_cost", C.c_double), ("la_best_model", C.c_int64), ("la_best_cand", C.c_int32),
                ("status", C.c_int32), ("la_best_cost", C.c_double),
                ("topk", C.c_int64 * KMAX), ("topk_val", C.c_double * KMAX),
                ("topk_Df", C.c_double * KMAX), ("topk_Dr", C.c_double * KMAX),
                ("topk_cand", C.c_int32 * KMAX), ("topk_cost", C.c_double * KMAX)]


PLAN_OUT_BYTES = C.sizeof(PlanOut)
HMAX = 64


class CtlCfg(C.Structure):
    """llampc_ctl_cfg (include/llampc.h): the controller tick's configuration."""
    _fields_ = [("C", C.c_int32), ("H", C.c_int32), ("K", C.c_int32), ("nan_policy", C.c_int32),
                ("Ts", C.c_double), ("v_factor", C.c_double), ("mu_init", C.c_double),
                ("S", C.c_int32), ("lap_projidx", C.c_int32), ("sigma", C.c_double * 2), ("seed", C.c_uint64),
                ("nominal", C.c_double * 6), ("cost", Cost), ("debug_inputs", C.c_int32), ("reserved", C.c_int32)]


class NlpCfg(C.Structure):
    """llampc_nlp_cfg: the setupNLP.solve drop-in's cross-entropy search."""
    _fields_ = [("H", C.c_int32), ("samples", C.c_int32), ("iters", C.c_int32), ("elite", C.c_int32),
                ("Ts", C.c_double), ("sigma0", C.c_double * 2), ("std_floor", C.c_double), ("seed", C.c_uint64),
                ("cost", Cost), ("rate_lo", C.c_double * 2), ("rate_hi", C.c_double * 2)]


class CtlOut(C.Structure):
    """llampc_ctl_out: the tick record plus the controller's own fields."""
    _fields_ = [("plan", PlanOut), ("tick", C.c_int64), ("projidx", C.c_int32), ("warm", C.c_int32),
                ("mu_used", C.c_double), ("scale_used", C.c_double), ("mu_pred", C.c_double),
                ("dr_mean", C.c_double), ("df_mean", C.c_double), ("u_seq", (C.c_double * 2) * HMAX)]

# name -> (restype, argtypes); exactly the symbols include/llampc.h declares.
_SIGNATURES = {
    "llampc_abi_version": (C.c_int32, []),
    "llampc_last_error": (C.c_char_p, []),
    "llampc_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "llampc_bank_create": (C.c_int, [_dp, C.c_int64, C.c_int64, C.POINTER(Vehicle), C.c_int32,
                                     C.c_int32, C.POINTER(C.c_void_p)]),
    "llampc_bank_destroy": (C.c_int, [C.c_void_p]),
    "llampc_bank_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "llampc_bank_reset": (C.c_int, [C.c_void_p]),
    "llampc_bank_launches": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
    "llampc_bank_window": (C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_int32)]),
    "llampc_bank_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_bank_set_concurrency": (C.c_int, [C.c_void_p, C.c_int32]),
    "llampc_bank_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "llampc_bank_set_raceline": (C.c_int, [C.c_void_p, _dp, C.c_int32, _dp, _dp, _dp, C.c_int32]),
    "llampc_plan_async": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_plan_wait": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_bank_timing": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "llampc_bank_timing_read": (C.c_int, [C.c_void_p, _dp, C.POINTER(C.c_int64)]),
    "llampc_lookback": (C.c_int, [C.c_void_p, _dp, _dp, _dp, C.c_double, C.c_int32, C.c_int32, _dp,
                                  _dp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _dp,
                                  C.POINTER(C.c_int32)]),
    "llampc_lookahead": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int32, C.c_int32, _dp, _dp,
                                   C.POINTER(Cost), C.c_double, C.c_int32, _dp,
                                   C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int32), _dp]),
    "llampc_plan": (C.c_int, [C.c_void_p, C.POINTER(PlanIn), C.POINTER(PlanOut), _dp, _dp, _dp]),
    "llampc_plan_device": (C.c_int, [C.c_void_p, C.POINTER(PlanIn), C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p]),
    "llampc_merge": (C.c_int, [C.POINTER(PlanOut), C.c_int32, C.c_int32, C.POINTER(PlanOut)]),
    "llampc_merge_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                      C.c_void_p]),
    "llampc_comm_unique_id": (C.c_int, [C.c_void_p]),
    "llampc_comm_create": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "llampc_comm_destroy": (C.c_int, [C.c_void_p]),
    "llampc_exchange_rccl": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "llampc_mailbox_create": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "llampc_mailbox_ipc_handle": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_mailbox_open_peer": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    "llampc_mailbox_link": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p]),
    "llampc_mailbox_set_bound": (C.c_int, [C.c_void_p, C.c_double]),
    "llampc_exchange_peer": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]),
    "llampc_plan_exchange": (C.c_int, [C.c_void_p, C.POINTER(PlanIn), C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    "llampc_mailbox_destroy": (C.c_int, [C.c_void_p]),
    "llampc_ctl_create": (C.c_int, [C.c_void_p, C.POINTER(CtlCfg), _dp, C.c_int32, _dp, C.POINTER(C.c_void_p)]),
    "llampc_ctl_tick": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "llampc_ctl_tick_async": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_ctl_wait": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_ctl_inputs": (C.c_int, [C.c_void_p, _dp, _dp]),
    "llampc_ctl_reference": (C.c_int, [C.c_void_p, _dp, C.c_double, C.c_int32, C.c_int32, C.c_double, C.c_double,
                                       _dp, C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
    "llampc_ctl_destroy": (C.c_int, [C.c_void_p]),
    "llampc_ctl_set_exchange": (C.c_int, [C.c_void_p, C.c_void_p, _dp, C.c_int64]),
    "llampc_ctl_set_gather": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, _dp, C.c_int64]),
    "llampc_ctl_record_words": (C.c_int32, [C.c_int32]),
    "llampc_ctl_shard_record": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)]),
    "llampc_ctl_resume": (C.c_int, [C.c_void_p, C.c_void_p]),
    "llampc_ctl_set_prelaunch": (C.c_int, [C.c_void_p, C.c_int32]),
    "llampc_ctl_device_us": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "llampc_ctl_merge": (C.c_int, [_dp, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, _dp,
                                   C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    "llampc_nlp_create": (C.c_int, [C.c_void_p, C.POINTER(NlpCfg), C.POINTER(C.c_void_p)]),
    # pointers as c_void_p: setupNLP.solve passes its persistent buffers' cached addresses
    "llampc_nlp_solve": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                   C.c_void_p, C.c_void_p, C.c_void_p]),
    "llampc_nlp_destroy": (C.c_int, [C.c_void_p]),
    "llampc_dynamics_batch": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                        C.POINTER(Vehicle), C.c_int64, C.c_void_p, C.c_int32,
                                        C.c_int32, C.c_void_p]),
    "llampc_math_batch": (C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32]),
    "llampc_integrate_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32,
                                         C.c_void_p, C.c_int64, C.POINTER(Vehicle), C.c_int64,
                                         C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_void_p]),
}

_lib = None
_lock = threading.Lock()


def lib_path() -> str:
    return os.environ.get("LLAMPC_HIP_LIB", _LIB_PATH)


def load():
    """Load libllampc_hip.so (raises NativeError if it is missing: no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = lib_path()
        # torch bundles its own libamdhip64.so.7: load it first so this library binds to
        # the same HIP runtime (one runtime per process; torch streams/pointers stay valid).
        if not os.environ.get("LLAMPC_NO_TORCH"):
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(path):
            raise NativeError(f"libllampc_hip.so not found at {path}: build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'` or "
                              "`make -C lla-mpc_amd/csrc` (there is no CPU fallback)")
        lib = C.CDLL(path)
        for name, (res, args) in _SIGNATURES.items():
            # an A/B build named by LLAMPC_HIP_LIB may predate newer entry points
            if path != _LIB_PATH and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.llampc_abi_version() != 1:
            raise NativeError("libllampc_hip ABI version mismatch")
        _lib = lib
        return lib


def check(rc: int):
    if rc != 0:
        msg = load().llampc_last_error().decode(errors="replace")
        raise (NoDeviceError if rc == E_NODEV else NativeError)(f"llampc error {rc}: {msg}", rc)


def device_count() -> int:
    n = C.c_int32(0)
    rc = load().llampc_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def dptr(a: np.ndarray | None):
    """Pointer to a C-contiguous float64 array (None -> NULL)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"], "need C-contiguous float64"
    return a.ctypes.data_as(_dp)


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def vehicle(lf, lr, mass, Iz, Cm1, Cm2, Cr0, Cr2, input_acc=False, approx=False) -> Vehicle:
    nz = lambda v: 0.0 if v is None else float(v)
    return Vehicle(float(lf), float(lr), float(mass), float(Iz), nz(Cm1), nz(Cm2), nz(Cr0), nz(Cr2),
                   int(bool(input_acc)), int(bool(approx)))


_DEFAULT_COST = None


def default_cost() -> Cost:
    """cost_struct() with its defaults, built once (a fresh copy per call)."""
    global _DEFAULT_COST
    if _DEFAULT_COST is None:
        _DEFAULT_COST = cost_struct()
    return Cost.from_buffer_copy(_DEFAULT_COST)


def cost_struct(Q=None, R=None, P=None, umin=(-0.1, -0.35), umax=(1.0, 0.35),
                rate_max=(-1.0, 5.0), enforce_bounds=False) -> Cost:
    """Objective of nmpc.py:44-111 with rt.py:60-62 defaults; bounds from orca.py:29-35."""
    Q = np.diag([1.0, 1.0]) if Q is None else np.asarray(Q, dtype=np.float64)
    R = np.diag([5 / 1000, 1.0]) if R is None else np.asarray(R, dtype=np.float64)
    P = np.diag([0.0, 0.0]) if P is None else np.asarray(P, dtype=np.float64)
    c = Cost()
    for dst, m in ((c.Q, Q), (c.R, R), (c.P, P)):
        for i, v in enumerate(np.asarray(m, dtype=np.float64).reshape(4)):
            dst[i] = float(v)
    for i in range(2):
        c.umin[i] = float(umin[i])
        c.umax[i] = float(umax[i])
        c.rate_max[i] = -1.0 if rate_max[i] is None else float(rate_max[i])
    c.enforce_bounds = int(bool(enforce_bounds))
    return c


def plan_out_to_dict(o: PlanOut) -> dict:
    K = o.K
    return dict(
        window_count=o.window_count, window_full=bool(o.window_full), K=K,
        lb_best=o.lb_best, lb_best_val=o.lb_best_val,
        sel_model=o.sel_model, sel_owned=bool(o.sel_owned), sel_cand=o.sel_cand, sel_cost=o.sel_cost,
        la_best_model=o.la_best_model, la_best_cand=o.la_best_cand, la_best_cost=o.la_best_cost,
        n_nonfinite=o.n_nonfinite, status=o.status,
        topk=np.array(o.topk[:K], dtype=np.int64), topk_val=np.array(o.topk_val[:K]),
        topk_Df=np.array(o.topk_Df[:K]), topk_Dr=np.array(o.topk_Dr[:K]),
        topk_cand=np.array(o.topk_cand[:K], dtype=np.int32), topk_cost=np.array(o.topk_cost[:K]),
    )


def merge(parts, nan_policy: int = NAN_FIRST) -> PlanOut:
    """Host run of the shared merge code (csrc/merge.hpp); same code as llampc_merge_device."""
    arr = (PlanOut * len(parts))(*parts)
    out = PlanOut()
    check(load().llampc_merge(arr, len(parts), nan_policy, C.byref(out)))
    return out
