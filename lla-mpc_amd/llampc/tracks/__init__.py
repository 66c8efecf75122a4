"""ETH Zurich race tracks: boundary/centre lines and the raceline library (host data).

Reference: llampc/tracks/track.py:12-160 (``Track``) and llampc/tracks/ethz.py:15-139
(``ETHZTrack``, ``ETHZ``, ``ETHZMobil``).  The data the reference reads from
``llampc/tracks/src`` — the centre/inner/outer lines (``ethz{,Mobil}_{center,inner,outer}.txt``,
ethz.py:20-42) and the optimal racelines with their per-friction speed profiles
(``ethz_raceline_long_.npz``, ``ethz_raceline_.npz``, ``ethzMobil_raceline_long_.npz``,
ethz.py:73-95) — is repacked, as data only, into ``tracks/data/tracks.npz`` by
the test tree's golden generator (gen_golden.py); ``ETHZTrack.load_txt`` reads the reference's txt format directly.

Constructor semantics follow ethz.py:106-138: ``reference='center'`` (the reference's
default) fits the raceline spline to the centre line and carries no speed profiles
(``mus`` is None, so ``ConstantSpeed`` fails on it exactly as in the reference);
``reference='optimal'`` loads the optimal raceline (``longer`` picks the ``_long`` file; the
ETHZMobil short file does not exist in the reference either: FileNotFoundError).
"""
import os

import numpy as np

from llampc.utils import Spline, Spline2D, project_segments

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "tracks.npz")
_DYN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "dyn_slice.npz")


def dyn_slice() -> dict:
    """The recorded ETHZ closed-loop slice (the reference's
    llampc/data/DYN-GPMPC-NOCONS-with_var_speedsETHZ.npz, states[:6, 470:621] and
    inputs[:, 470:620], repacked as data by the test tree's gen_golden.py): ``states`` [6, 151],
    ``inputs`` [2, 150], ``first_index``.  The config-2 scenario's controls and start state."""
    with np.load(_DYN) as d:
        return {k: d[k] for k in d.files}


class Track:
    """track.py:12-160: centre line geometry and projections shared by all tracks."""

    def _init_geometry(self):
        # track.py:20-26: centre line 2 x n
        self.center_line = np.concatenate([self.x_center.reshape(1, -1), self.y_center.reshape(1, -1)])
        # track.py:28-35: closed length (last point joined to the first)
        self.track_length = self._calc_raceline_length(self.center_line)
        # track.py:45-50: arc length at every centre point, from 0
        seg = np.linalg.norm(np.diff(self.center_line), 2, axis=0)
        self.theta_track = np.concatenate([np.array([0.0]), np.cumsum(seg)])

    @staticmethod
    def _calc_raceline_length(raceline):
        """track.py:37-43: length of the closed polyline ``raceline`` [2, n]."""
        closed = np.concatenate([raceline, raceline[:, 0].reshape(-1, 1)], axis=1)
        return np.sum(np.linalg.norm(np.diff(closed), 2, axis=0))

    def _param2xy(self, theta):
        """track.py:101-111: point on the centre line at arc length ``theta`` (linear
        interpolation between the bracketing centre points, the reference's scan)."""
        tt = self.theta_track
        # first idt with tt[idt] > theta, capped at n-1 (the while loop of track.py:106-107)
        idt = int(np.searchsorted(tt, theta, side="right"))
        idt = min(idt, tt.shape[0] - 1)
        d = (theta - tt[idt - 1]) / (tt[idt] - tt[idt - 1])
        x = self.x_center[idt - 1] + d * (self.x_center[idt] - self.x_center[idt - 1])
        y = self.y_center[idt - 1] + d * (self.y_center[idt] - self.y_center[idt - 1])
        return x, y

    def project(self, x, y, raceline):
        """track.py:130-145: projection onto the CLOSED polyline ``raceline`` [2, n]; the
        closing segment (n-1 -> 0) is reported as index -1."""
        n = raceline.shape[1]
        A = np.concatenate([raceline[:, :-1], raceline[:, -1:]], axis=1)       # segment j: j -> j+1
        B = np.concatenate([raceline[:, 1:], raceline[:, :1]], axis=1)         # last: n-1 -> 0
        proj, dist = project_segments(np.array([x, y], dtype=np.float64), A, B)
        optidx = int(np.argmin(dist))
        if optidx == n - 1:
            optidx = -1
        return proj[:, optidx], optidx

    def project_fast(self, x, y, raceline):
        """track.py:147-160: nearest segment of the open polyline ``raceline`` [2, m]."""
        proj, dist = project_segments(np.array([x, y], dtype=np.float64), raceline[:, :-1], raceline[:, 1:])
        i = int(np.argmin(dist))
        return proj[:, i], i

    def _xy2param(self, x, y):
        """track.py:113-128: arc length along the centre line of the projection of (x, y)."""
        cl, tt = self.center_line, self.theta_track
        optxy, optidx = self.project(x, y, cl)
        distxy = np.linalg.norm(optxy - cl[:, optidx], 2)
        dist = np.linalg.norm(cl[:, optidx + 1] - cl[:, optidx], 2)
        deltaxy = distxy / dist
        if optidx == -1:
            theta = tt[optidx] + deltaxy * (self.track_length - tt[optidx])
        else:
            theta = tt[optidx] + deltaxy * (tt[optidx + 1] - tt[optidx])
        return theta % self.track_length

    def param_to_xy(self, theta):
        """ethz.py:48-51."""
        return self._param2xy(theta)

    def xy_to_param(self, x, y):
        """ethz.py:53-57."""
        return self._xy2param(x, y)


class Raceline(Track):
    """Raceline spline + speed-profile splines indexed by friction mu (track.py:52-83)."""

    def __init__(self, name, path=None):
        d = np.load(path or _DATA, allow_pickle=False)
        self._build(name, d[f"{name}_x"], d[f"{name}_y"], d[f"{name}_speeds"], d[f"{name}_mus"],
                    *(float(v) for v in d[f"{name}_init"]), float(d[f"{name}_track_width"]))

    def _build(self, name, x, y, speeds, mus, x_init, y_init, psi_init, vx_init, track_width):
        self.name = name
        self._load_raceline(x, y, speeds, mus)
        self.x_init, self.y_init, self.psi_init, self.vx_init = x_init, y_init, psi_init, vx_init
        self.track_width = track_width
        # projidx beyond which the driver counts a lap and restarts the projection window
        # (rt.py:287 uses 656 for ETHZ; 440 for ETHZMobil, rt.py:288 / nrt_avg_runs.py:354)
        self.lap_projidx = {"ETHZ": 656, "ETHZMobil": 440}.get(name, self.raceline.shape[1] - 44)

    def _load_raceline(self, x, y, speeds=None, mus=None):
        """track.py:52-83: the raceline spline; speed splines when profiles are given."""
        self.raceline = np.array([x, y], dtype=np.float64)
        self.x_raceline, self.y_raceline = self.raceline
        self.spline = Spline2D(self.x_raceline, self.y_raceline)
        self.length = self.spline.s[-1]
        if speeds is None:                      # reference='center': no speed profiles
            self.mus, self.v_raceline, self.spline_v = None, None, None
            return
        self.mus = np.asarray(mus, dtype=np.float64)
        self.v_raceline = np.atleast_2d(np.asarray(speeds, dtype=np.float64))
        self.spline_v = [Spline(self.spline.s, v) for v in self.v_raceline]

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
        if self.spline_v is None:
            raise ValueError(f"{self.name}: no speed profiles (reference='center'); the device "
                             "raceline lookup needs reference='optimal'")
        knots = np.asarray(self.spline.s, dtype=np.float64)
        xy = np.stack([self.spline.sx.coefficients(), self.spline.sy.coefficients()])
        speed = np.stack([sp.coefficients() for sp in self.spline_v])
        return knots, np.ascontiguousarray(xy), np.ascontiguousarray(speed), np.asarray(self.mus, dtype=np.float64)


    def ctl_table(self):
        """(points [2, np], prefix [np-1]) for llampc_ctl_create: the polyline project_fast
        projects on (track.py:147-160) and, per projection index p, the start arc length of
        ConstantSpeed (planner.py:29-36) evaluated with the reference's own expression — so the
        device controller's lookup equals the host planner's sum bitwise, in O(1) per tick."""
        cached = getattr(self, "_ctl_table", None)
        if cached is None:
            rl = np.ascontiguousarray(self.raceline, dtype=np.float64)
            prefix = np.array([np.sum(np.linalg.norm(np.diff(rl[:, :p + 2]), 2, axis=0))
                               for p in range(rl.shape[1] - 1)])
            cached = self._ctl_table = (rl, prefix)
        return cached


class ETHZTrack(Raceline):
    """ethz.py:15-97: boundary lines from the reference's txt files (packaged) plus the
    raceline chosen by ``reference`` / ``longer``."""

    _ID, _WIDTH, _PSI = "", 0.37, 0.0

    def __init__(self, reference='center', longer=False, path=None):
        d = np.load(path or _DATA, allow_pickle=False)
        name = type(self).__name__ if type(self).__name__ in ("ETHZ", "ETHZMobil") else "ETHZ"
        self.name = name
        self.inner, self.center, self.outer = (np.asarray(d[f"{name}_{k}"], dtype=np.float64)
                                              for k in ("inner", "center", "outer"))
        self.x_inner, self.y_inner = self.inner[0, :], self.inner[1, :]
        self.x_center, self.y_center = self.center[0, :], self.center[1, :]
        self.x_outer, self.y_outer = self.outer[0, :], self.outer[1, :]
        self.track_width = self._WIDTH
        self.mus = None
        self._init_geometry()
        self.reference, self.longer = reference, longer
        if reference == 'center':                                           # ethz.py:66-72
            self._load_raceline(self.x_center, self.y_center)
        elif reference == 'optimal':                                        # ethz.py:73-95
            key = name if longer else f"{name}_short"
            if f"{key}_x" not in d.files:
                raise FileNotFoundError(f"ethz{self._ID}_raceline{'_long' if longer else ''}_.npz: "
                                        "no such raceline in the reference's track data")
            self._load_raceline(d[f"{key}_x"], d[f"{key}_y"], d[f"{key}_speeds"], d[f"{key}_mus"])
        else:
            raise NotImplementedError(f"reference={reference!r}")
        self.psi_init = self._PSI                                           # ethz.py:118-121
        self.x_init, self.y_init = float(self.x_raceline[0]), float(self.y_raceline[0])
        self.vx_init = 0.1
        if reference == 'optimal' and longer:
            self.lap_projidx = {"ETHZ": 656, "ETHZMobil": 440}[name]
        else:
            self.lap_projidx = self.raceline.shape[1] - 44

    @staticmethod
    def load_txt(path):
        """One of the reference's line files (ethz.py:22-39: comma-separated, '#' comments,
        two rows x / y) -> [2, n] float64."""
        return np.loadtxt(path, comments='#', delimiter=',', unpack=False)


class ETHZ(ETHZTrack):
    """ethz.py:106-121 (track width 0.37, psi_init = -pi/4)."""
    _ID, _WIDTH, _PSI = "", 0.37, -np.pi / 4


class ETHZMobil(ETHZTrack):
    """ethz.py:124-138 (track width 0.46, psi_init = 0)."""
    _ID, _WIDTH, _PSI = "Mobil", 0.46, 0.0
