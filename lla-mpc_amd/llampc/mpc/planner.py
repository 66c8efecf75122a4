"""Look-ahead reference from the raceline library (host side).

``ConstantSpeed`` keeps the reference signature and result (llampc/mpc/planner.py:12-67):
project x0 onto the next 10 raceline points, start two points ahead, then advance H
times by scale*v*Ts along the arc length (mod the lap length), sampling the raceline
spline and the speed profile linearly interpolated between the two friction profiles
that bracket curr_mu.
"""
import numpy as np


def speed_at(track, dist, curr_mu):
    """Speed profile at arc length ``dist`` for friction ``curr_mu`` (planner.py:48-62)."""
    mus = track.mus
    if curr_mu < mus[0]:
        return track.spline_v[0].calc(dist)
    if curr_mu > mus[-1]:
        return track.spline_v[-1].calc(dist)
    ge = np.flatnonzero(mus >= curr_mu)      # first profile with mu_i >= curr_mu; none
    i = int(ge[0]) if ge.size else len(mus) - 1   # (NaN mu): the loop ends at the last
    lo, hi = mus[i - 1], mus[i]              # i == 0 wraps to the last profile, as the reference
    vb = track.spline_v[i - 1].calc(dist)
    va = track.spline_v[i].calc(dist)
    return vb * (hi - curr_mu) / (hi - lo) + va * (curr_mu - lo) / (hi - lo)


def raceline_start(x0, track, projidx):
    """The shared start of ConstantSpeed (planner.py:25-33): project x0 onto the next 10
    raceline points and return (arc length two points ahead, new projidx).  With
    xref_mode='raceline' the device continues from here per model (csrc/raceline.hpp)."""
    rl = track.raceline
    _, idx = track.project_fast(x0[0], x0[1], rl[:, projidx:projidx + 10])
    projidx = idx + projidx
    table = getattr(track, "ctl_table", None)
    if table is not None:                   # the cached prefix table: the same sum, O(1) per call
        prefix = table()[1]
        return float(prefix[min(projidx, prefix.shape[0] - 1)]), projidx
    seg = rl[:, :projidx + 2]
    return float(np.sum(np.linalg.norm(np.diff(seg), 2, axis=0))), projidx


def ConstantSpeed(x0, v0, track, N, Ts, projidx, scale=1., curr_mu=1.):
    """-> (xref [2, N+1], projidx, vr)."""
    dist, projidx = raceline_start(x0, track, projidx)
    xref = np.zeros([2, N + 1])
    xref[:2, 0] = x0
    L = track.spline.s[-1]
    v = max(v0, .01)
    vr = 0.
    for h in range(1, N + 1):
        dist = (dist + scale * v * Ts) % L
        xref[:2, h] = track.spline.calc_position(dist)
        v = speed_at(track, dist, curr_mu)
        if h == 1:
            vr = v * scale
    return xref, projidx, vr
