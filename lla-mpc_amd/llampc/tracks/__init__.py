"""ETH Zurich race tracks with the optimal raceline library (host data).

Reference: llampc/tracks/ethz.py:15-139 and track.py:52-83,147-160.  The raceline
coordinates and the per-friction speed profiles (``speeds`` [M, n], ``mus`` [M]) are read
from ``tracks/data/tracks.npz`` (repacked from the reference's ethz*_raceline_long_.npz by
tests/golden/gen_golden.py).
"""
import os

import numpy as np

from llampc.utils import Spline, Spline2D, project_segments

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "tracks.npz")


class Raceline:
    """Raceline spline + speed-profile splines indexed by friction mu."""

    def __init__(self, name, path=None):
        d = np.load(path or _DATA, allow_pickle=False)
        self.name = name
        x, y = d[f"{name}_x"], d[f"{name}_y"]
        self.raceline = np.array([x, y])
        self.x_raceline, self.y_raceline = self.raceline
        self.spline = Spline2D(x, y)
        self.mus = np.asarray(d[f"{name}_mus"])
        self.v_raceline = np.asarray(d[f"{name}_speeds"])
        self.spline_v = [Spline(self.spline.s, v) for v in self.v_raceline]
        self.x_init, self.y_init, self.psi_init, self.vx_init = (float(v) for v in d[f"{name}_init"])
        self.track_width = float(d[f"{name}_track_width"])
        self.length = self.spline.s[-1]
        # projidx beyond which the driver counts a lap and restarts the projection window
        # (rt.py:287 uses 656 for ETHZ; 440 for ETHZMobil, rt.py:288 / nrt_avg_runs.py:354)
        self.lap_projidx = {"ETHZ": 656, "ETHZMobil": 440}.get(name, self.raceline.shape[1] - 44)

    def device_table(self):
        """(knots [n], xy [2, 4, n-1], speed [M, 4, n-1], mus [M]) for
        llampc_bank_set_raceline: the raceline and speed-profile spline coefficients."""
        knots = np.asarray(self.spline.s, dtype=np.float64)
        xy = np.stack([self.spline.sx.coefficients(), self.spline.sy.coefficients()])
        speed = np.stack([sp.coefficients() for sp in self.spline_v])
        return knots, np.ascontiguousarray(xy), np.ascontiguousarray(speed), np.asarray(self.mus, dtype=np.float64)

    def project_fast(self, x, y, raceline):
        """track.py:147-160: nearest segment of the polyline ``raceline`` [2, m]."""
        proj, dist = project_segments(np.array([x, y], dtype=np.float64), raceline[:, :-1], raceline[:, 1:])
        i = int(np.argmin(dist))
        return proj[:, i], i


class ETHZ(Raceline):
    def __init__(self, reference='optimal', longer=True, path=None):
        if reference != 'optimal' or not longer:
            raise NotImplementedError("only the optimal 'long' raceline library is packaged")
        super().__init__("ETHZ", path)


class ETHZMobil(Raceline):
    def __init__(self, reference='optimal', longer=True, path=None):
        if reference != 'optimal' or not longer:
            raise NotImplementedError("only the optimal 'long' raceline library is packaged")
        super().__init__("ETHZMobil", path)
