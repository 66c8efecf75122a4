"""Diagnostic: worst-ulp arguments of the fast atan2/atan cores (math fn 4/5) vs NumPy."""
import sys, os, numpy as np
sys.path[:0] = [".", "lla-mpc_amd"]
from llampc import _native as nat
nat.load()
def _math(nat, fn, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.float64)
    out = np.empty_like(a)
    nat.check(nat.load().llampc_math_batch(fn, a.ctypes.data, None if bb is None else bb.ctypes.data, a.size, out.ctypes.data, 0))
    return out
rng = np.random.RandomState(1)
n = 1 << 20
y = np.concatenate([rng.uniform(-3, 3, n), rng.standard_cauchy(n), [0.0, -0.0, 1.0, -1.0, 1e-300, 5.0]])
x = np.concatenate([rng.uniform(0, 4, n), np.abs(rng.standard_cauchy(n)), [1.0, 1.0, 0.0, 0.0, 0.0, 3.0]])
ok = (np.abs(y) + x >= 2.0 ** -1000) & (np.abs(y) + x <= 2.0 ** 1000)
g = _math(nat, 4, y[ok], x[ok]); w = np.arctan2(y[ok], x[ok])
u = np.abs(g - w) / np.spacing(np.abs(w))
i = np.argsort(u)[-5:]
print(os.environ.get("LLAMPC_HIP_LIB","")[-25:], "atan2 max ulp", u.max(), "at y,x,ratio", list(zip(y[ok][i], x[ok][i], (y[ok]/x[ok])[i], u[i])))
z = np.concatenate([rng.uniform(-2, 2, n), rng.standard_cauchy(n) * 10])
g = _math(nat, 5, z); w = np.arctan(z); u = np.abs(g - w) / np.spacing(np.abs(w)); print("atan max ulp", u.max(), z[np.argmax(u)])
