"""Base model (reference: llampc/models/model.py:13-40).

``_integrate`` (RK6, the plant) and ``_integrate_batch`` (RK4, the bank) run on the
MI355X through libllampc_hip; subclasses provide ``_native_args``.
"""
import numpy as np

from llampc import _native as nat


class Model:

    def __init__(self):
        pass

    def _integrate(self, x_t, u_t, t_start, t_end):
        """One RK6 step of a single state (model.py:18-30 / rk6.py:13-28)."""
        x = nat.f64(x_t).reshape(1, 6)
        u = nat.f64(u_t).reshape(1, 1, 2)
        return self._native_integrate(x, u, np.array([t_end - t_start], dtype=np.float64),
                                      nat.RK6, final_only=True)[0]

    def _integrate_batch(self, x_t_batch, u_t_batch, t_start, t_end):
        """One RK4 step per row (model.py:32-40 / rk6.py:50-68) -> [N, 6]."""
        x = nat.f64(x_t_batch).reshape(-1, 6)
        u = nat.f64(u_t_batch).reshape(-1, 1, 2)
        return self._native_integrate(x, u, np.array([t_end - t_start], dtype=np.float64),
                                      nat.RK4, final_only=True)
