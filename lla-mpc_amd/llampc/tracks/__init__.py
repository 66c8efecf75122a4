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
        self._build(name, d[f"{name}_x"], d[f"{name}_y"], d[f"{name}_speeds"], d[f"{name}_mus"],
                    *(float(v) for v in d[f"{name}_init"]), float(d[f"{name}_track_width"]))

    def _build(self, name, x, y, speeds, mus, x_init, y_init, psi_init, vx_init, track_width):
        self.name = name
        self.raceline = np.array([x, y], dtype=np.float64)
        self.x_raceline, self.y_raceline = self.raceline
        self.spline = Spline2D(self.x_raceline, self.y_raceline)
        self.mus = np.asarray(mus, dtype=np.float64)
        self.v_raceline = np.atleast_2d(np.asarray(speeds, dtype=np.float64))
        self.spline_v = [Spline(self.spline.s, v) for v in self.v_raceline]
        self.x_init, self.y_init, self.psi_init, self.vx_init = x_init, y_init, psi_init, vx_init
        self.track_width = track_width
        self.length = self.spline.s[-1]
        # projidx beyond which the driver counts a lap and restarts the projection window
        # (rt.py:287 uses 656 for ETHZ; 440 for ETHZMobil, rt.py:288 / nrt_avg_runs.py:354)
        self.lap_projidx = {"ETHZ": 656, "ETHZMobil": 440}.get(name, self.raceline.shape[1] - 44)

    @classmethod
    def from_raceline_npz(cls, path, name="custom", track_width=0.37, psi_init=0.0, vx_init=0.1,
                          lap_projidx=None):
        """A raceline file in the reference's format (ethz.py:59-96: keys ``x``, ``y``,
        ``speed``, ``time`` and optionally ``speeds`` [M, n] + ``mus`` [M]); without
        ``speeds`` the single ``speed`` profile serves every friction (mus = [1.0]).
        Loaded with allow_pickle=False."""
        d = np.load(path, allow_pickle=False)
        x, y = d["x"], d["y"]
        if "speeds" in d.files:
            speeds, mus = d["speeds"], d["mus"]
        else:
            speeds, mus = np.asarray(d["speed"])[None], np.array([1.0])
        obj = cls.__new__(cls)
        obj._build(name, x, y, speeds, mus, float(x[0]), float(y[0]), psi_init, vx_init, track_width)
        obj.lap_projidx = lap_projidx if lap_projidx is not None else obj.raceline.shape[1] - 44
        return obj

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
