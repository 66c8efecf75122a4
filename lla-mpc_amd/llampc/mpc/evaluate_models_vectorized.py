"""Look-back scoring of the whole bank on one transition, on the MI355X.

Same signature and result as the reference function
(llampc/mpc/evaluate_models_vectorized.py:4-24): tile the current state/input to every
model, take one RK4 step (model.py:32-40) with the per-model Pacejka arrays and return the
predicted [X, Y, psi, vx] rows, shape [N, 4].  ``n_models`` is ignored as in the reference
(len(models) is used); mass/geometry/motor constants come from ``models[0]``.

For repeated ticks prefer ``llampc.mpc.ModelBank`` (bank resident on the device, fused
error/window/argmin) — this entry point re-uploads the parameters on every call.
"""
import numpy as np

from llampc.models import Dynamic


def evaluate_models_vectorized(models, n_models, current_state, input_val, Ts, params):
    n_models = len(models)
    Bfs, Cfs, Dfs, Brs, Crs, Drs = params
    m0 = models[0]
    batch_model = Dynamic(Bf=Bfs, Cf=Cfs, Df=Dfs, Br=Brs, Cr=Crs, Dr=Drs, mass=m0.mass, lf=m0.lf,
                          lr=m0.lr, Iz=m0.Iz, Cm1=m0.Cm1, Cm2=m0.Cm2, Cr0=m0.Cr0, Cr2=m0.Cr2,
                          input_acc=m0.input_acc, device=getattr(m0, "device", -1))
    x0 = np.tile(np.asarray(current_state, dtype=np.float64), (n_models, 1))
    u0 = np.tile(np.asarray(input_val, dtype=np.float64), (n_models, 1))
    return batch_model._integrate_batch(x0, u0, 0, Ts)[:, 0:4]
