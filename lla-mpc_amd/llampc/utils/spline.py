"""Natural cubic splines for the raceline lookup (host side).

Same model and evaluation rule as the reference (llampc/utils/pycubicspline.py:17-182):
natural boundary (c_0 = c_{n-1} = 0), segment found by bisect-right on the knots,
y = a + b dx + c dx^2 + d dx^3, ``None`` outside [x_0, x_{n-1}].  The tridiagonal system is
solved banded (O(n)) instead of the reference's dense np.linalg.solve (O(n^3)); results
agree to ~1e-15.  ``coefficients()`` exports the [4, n-1] table a device lookup stages.
"""
import bisect

import numpy as np
from scipy.linalg import solve_banded


class Spline:

    def __init__(self, x, y):
        self.x = list(np.asarray(x, dtype=np.float64))
        self.y = np.asarray(y, dtype=np.float64)
        xs = np.asarray(self.x)
        n = self.nx = len(xs)
        h = np.diff(xs)
        a = self.y
        # banded form of pycubicspline.py:105-132 (rows: super, main, sub)
        ab = np.zeros((3, n))
        ab[1, 0] = ab[1, n - 1] = 1.0
        ab[1, 1:n - 1] = 2.0 * (h[:-1] + h[1:])
        ab[0, 2:n] = h[1:]          # A[i, i+1] = h[i] for i >= 1 (A[0,1] = 0)
        ab[2, 0:n - 2] = h[:-1]     # A[i+1, i] = h[i] for i <= n-3 (A[n-1,n-2] = 0)
        rhs = np.zeros(n)
        rhs[1:n - 1] = 3.0 * (a[2:] - a[1:-1]) / h[1:] - 3.0 * (a[1:-1] - a[:-2]) / h[:-1]
        c = solve_banded((1, 1), ab, rhs)
        self.a = list(a)
        self.c = c
        self.d = list((c[1:] - c[:-1]) / (3.0 * h))
        self.b = list((a[1:] - a[:-1]) / h - h * (c[1:] + 2.0 * c[:-1]) / 3.0)

    def _seg(self, t):
        # bisect-right as the reference; t == x[-1] maps to the last segment (the
        # reference would index past its coefficient lists there)
        return min(bisect.bisect(self.x, t) - 1, self.nx - 2)

    def calc(self, t):
        if t < self.x[0] or t > self.x[-1]:
            return None
        i = self._seg(t)
        dx = t - self.x[i]
        return self.a[i] + self.b[i] * dx + self.c[i] * dx ** 2.0 + self.d[i] * dx ** 3.0

    def calcd(self, t):
        if t < self.x[0] or t > self.x[-1]:
            return None
        i = self._seg(t)
        dx = t - self.x[i]
        return self.b[i] + 2.0 * self.c[i] * dx + 3.0 * self.d[i] * dx ** 2.0

    def calcdd(self, t):
        if t < self.x[0] or t > self.x[-1]:
            return None
        i = self._seg(t)
        dx = t - self.x[i]
        return 2.0 * self.c[i] + 6.0 * self.d[i] * dx

    def coefficients(self) -> np.ndarray:
        """[4, n-1] (a, b, c, d) per segment, for device staging."""
        m = self.nx - 1
        return np.stack([np.asarray(self.a[:m]), np.asarray(self.b), np.asarray(self.c[:m]),
                         np.asarray(self.d)])


class Spline2D:

    def __init__(self, x, y):
        dx, dy = np.diff(x), np.diff(y)
        self.ds = list(np.sqrt(dx ** 2 + dy ** 2))
        self.s = [0.0] + list(np.cumsum(self.ds))
        self.sx = Spline(self.s, x)
        self.sy = Spline(self.s, y)

    def calc_position(self, s):
        return self.sx.calc(s), self.sy.calc(s)

    def calc_curvature(self, s):
        dx, ddx = self.sx.calcd(s), self.sx.calcdd(s)
        dy, ddy = self.sy.calcd(s), self.sy.calcdd(s)
        return (ddy * dx - ddx * dy) / (dx ** 2 + dy ** 2)

    def calc_yaw(self, s):
        return float(np.arctan2(self.sy.calcd(s), self.sx.calcd(s)))
