"""Dynamic bicycle model with Pacejka tires, evaluated on the MI355X.

Drop-in for the reference class (llampc/models/dynamic.py:22-57): same constructor,
attributes and batched methods.  Pacejka parameters may be scalars (one model,
broadcast over the batch) or arrays [N] (one model per row — the batched bank that
evaluate_models_vectorized builds, evaluate_models_vectorized.py:13-22).  Every
evaluation runs in libllampc_hip (csrc/dyn.hpp); none falls back to NumPy.

The CasADi symbolic form (dynamic.py:195-275) is not part of this path: its
numerics are available as the ``euler_nlp`` integrator of the look-ahead.
"""
import numpy as np

from llampc import _native as nat
from llampc.models.model import Model

_TIRE = ("Bf", "Cf", "Df", "Br", "Cr", "Dr")


class Dynamic(Model):

    def __init__(self, lf, lr, mass, Iz, Cf, Cr, Bf=None, Br=None, Df=None, Dr=None,
                 Cm1=None, Cm2=None, Cr0=None, Cr2=None, input_acc=False, carla=False,
                 device=-1, **kwargs):
        self.lf, self.lr = lf, lr
        self.dr = lr / (lf + lr)
        self.mass, self.Iz = mass, Iz
        self.Cf, self.Cr = Cf, Cr
        self.Bf, self.Br, self.Df, self.Dr = Bf, Br, Df, Dr
        self.Cm1, self.Cm2, self.Cr0, self.Cr2 = Cm1, Cm2, Cr0, Cr2
        # dynamic.py:49-51: linear tires when any Pacejka B/D is missing
        self.approx = Bf is None or Br is None or Df is None or Dr is None
        self.input_acc = input_acc
        self.carla = carla
        self.n_states = 6
        self.n_inputs = 2
        self.device = device
        Model.__init__(self)

    # ---------------------------------------------------------------- native plumbing
    def _vehicle(self):
        return nat.vehicle(self.lf, self.lr, self.mass, self.Iz, self.Cm1, self.Cm2, self.Cr0,
                           self.Cr2, self.input_acc, self.approx)

    def _params6(self, n):
        """[6, P] SoA (Bf, Cf, Df, Br, Cr, Dr) with P in {1, n}."""
        vals = [0.0 if getattr(self, k) is None else getattr(self, k) for k in _TIRE]
        arrs = [np.asarray(v, dtype=np.float64).reshape(-1) for v in vals]
        if all(a.size == 1 for a in arrs):
            return np.ascontiguousarray(np.stack(arrs)), 1
        for a in arrs:
            if a.size not in (1, n):
                raise ValueError(f"parameter array of length {a.size} does not match batch {n}")
        return np.ascontiguousarray(np.stack([np.broadcast_to(a, (n,)) for a in arrs])), n

    def _native_integrate(self, x, u, h, integrator, final_only=True):
        """x [n,6], u [n,S,2] (per lane), h [S] -> final [n,6] or trajectory [S+1,n,6]."""
        n, S = x.shape[0], h.shape[0]
        u = nat.f64(np.broadcast_to(u, (n, S, 2)))
        p, P = self._params6(n)
        out = np.empty((n, 6) if final_only else (S + 1, n, 6))
        veh = self._vehicle()
        nat.check(nat.load().llampc_integrate_batch(
            x.ctypes.data, u.ctypes.data, 2 * S, h.ctypes.data, S, p.ctypes.data, P,
            nat.C.byref(veh), n, integrator, out.ctypes.data, int(final_only), self.device, 0, None))
        return out

    def _native_dyn(self, op, x_batch, u_batch):
        x = nat.f64(x_batch).reshape(-1, 6)
        n = x.shape[0]
        u = nat.f64(np.broadcast_to(np.asarray(u_batch, dtype=np.float64).reshape(-1, 2), (n, 2)))
        p, P = self._params6(n)
        out = np.empty((5, n) if op == nat.OP_FORCES else (n, 6))
        veh = self._vehicle()
        nat.check(nat.load().llampc_dynamics_batch(op, x.ctypes.data, u.ctypes.data, p.ctypes.data, P,
                                                   nat.C.byref(veh), n, out.ctypes.data, self.device,
                                                   0, None))
        return out

    # ---------------------------------------------------------------- batched API
    def calc_forces_batch(self, x_batch, u_batch, return_slip=False):
        """dynamic.py:117-154 -> (Ffy, Frx, Fry[, alphaf, alphar]) each [N]."""
        f = self._native_dyn(nat.OP_FORCES, x_batch, u_batch)
        return (f[0], f[1], f[2], f[3], f[4]) if return_slip else (f[0], f[1], f[2])

    def _diffequation_batch(self, t, x_batch, u_batch):
        """dynamic.py:98-115 -> dx/dt [N, 6]."""
        return self._native_dyn(nat.OP_DERIV, x_batch, u_batch)

    # ---------------------------------------------------------------- single-state API
    def calc_forces(self, x, u, return_slip=False):
        """dynamic.py:156-193 (one state; a batch of one on the device)."""
        f = self._native_dyn(nat.OP_FORCES, np.asarray(x).reshape(1, 6), np.asarray(u).reshape(1, 2))
        out = tuple(float(v[0]) for v in f)
        return out if return_slip else out[:3]

    def _diffequation(self, t, x, u):
        """dynamic.py:76-96."""
        return self._native_dyn(nat.OP_DERIV, np.asarray(x).reshape(1, 6), np.asarray(u).reshape(1, 2))[0]

    def sim_continuous(self, x0, u, t):
        """dynamic.py:59-74: plant simulation with one RK6 step per interval of ``t``.
        Returns (x [6, n+1], dxdt [6, n+1])."""
        u = nat.f64(u).reshape(2, -1)
        n = u.shape[1]
        t = np.asarray(t, dtype=np.float64)
        h = nat.f64(np.diff(t)[:n])
        x0 = nat.f64(x0).reshape(1, 6)
        traj = self._native_integrate(x0, u.T.reshape(1, n, 2), h, nat.RK6, final_only=False)[:, 0, :]
        x = np.ascontiguousarray(traj.T)
        uu = np.concatenate([np.zeros((1, 2)), u.T], axis=0)       # dxdt[:,0] uses u=[0,0]
        dxdt = self._native_dyn(nat.OP_DERIV, traj, uu).T
        return x, np.ascontiguousarray(dxdt)
