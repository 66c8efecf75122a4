// raceline.hpp — per-model reference trajectories from the raceline library on the device
// (SURVEY.md §8f #1): ConstantSpeed (llampc/mpc/planner.py:12-67) evaluated in every
// look-ahead lane with the lane's own friction mu_n = (Df_n + Dr_n) / (9.81 m) instead of
// one shared mu-hat.
//
//   start (host, shared):  projection of x0 on the raceline -> arc length s0, v0 (planner.py:
//                          19-33; llampc.mpc.planner.raceline_start)
//   per step (device):     s <- (s + scale v Ts) mod L                          (:41-42)
//                          xref = (x(s), y(s)) cubic splines                  (:43)
//                          v = speed profiles bracketing mu_n, linear in mu   (:48-62)
// Splines (pycubicspline.py:17-182): knots = arc length s_i, y = a + b dx + c dx^2 + d dx^3
// on the segment found by bisect-right; here each lane keeps its segment and walks it
// forward as s advances (a wrap restarts at 0) — the same segment as the bisection.
// Table layout (llampc_bank_set_raceline): knots [n]; xy [2][4][n-1] (x then y; a,b,c,d
// rows); speed [M][4][n-1]; mus [M] ascending.  Knots, xy and mus are staged in LDS per
// block, and of the speed profiles the window every walk of the launch reads (SpeedWin).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace llampc {

struct RacelineK {
  const double* knots;   // [n]
  const double* xy;      // [2][4][n-1]
  const double* speed;   // [M][4][n-1]
  const double* mus;     // [M]
  int32_t n, M;
  int32_t wcap;          // speed-window capacity in segments (LDS left by the launch)
  double hmin, vmax;     // shortest segment; bound of |v| on every profile (window_adv)
};

// The walkers' window of the speed profiles in LDS: segments seg0 .. seg0 + W - 1 (mod
// n - 1) of every profile, rows [M][4][W].  All models of a launch start at the same s0 and
// advance by at most scale Ts (v0 + (H - 1) vmax) (planner.py:41), so a window of that
// length holds every coefficient their walks read; a read outside it (a negative scale)
// goes to global memory.  Without the window, each walker step waited on two dependent
// global reads: ~20 us of the raceline tick at H = 20.
struct SpeedWin {
  const double* w;       // null: no window
  int seg0, W;
};

// |v| bound over a profile table: per segment |a| + |b| h + |c| h^2 + |d| h^3 (host, at
// llampc_bank_set_raceline).
__host__ __forceinline__ double speed_bound(const double* knots, const double* speed, int n, int M) {
  const int m = n - 1;
  double vmax = 0.0;
  for (int p = 0; p < M; ++p)
    for (int i = 0; i < m; ++i) {
      const double h = knots[i + 1] - knots[i];
      const double* c = speed + (size_t)p * 4 * m;
      const double b = fabs(c[i]) + fabs(c[m + i]) * h + fabs(c[2 * m + i]) * h * h + fabs(c[3 * m + i]) * h * h * h;
      vmax = b > vmax ? b : vmax;
    }
  return vmax;
}

// The largest arc length H walker steps advance (planner.py:41: scale Ts v per step, v0
// first, then profile speeds <= vmax); NaN / inf -> inf (no window).  The window spans the
// knots from s0 to s0 + this advance (kernels.hip lookahead_block).
__device__ __host__ __forceinline__ double window_adv(double v0, double scale, double Ts, int H,
                                                      double vmax) {
  const double adv = fabs(scale) * Ts * (fmax(v0, 0.01) + (H - 1) * vmax);
  return adv == adv ? adv : 1e300;
}

__device__ __host__ __forceinline__ double spline_at(const double* c, int m, int i, double dx) {
  // c: [4][m] rows a, b, c, d; pycubicspline.py:47-65 order a + b dx + c dx^2 + d dx^3
  const double dx2 = dx * dx;
  return c[i] + c[m + i] * dx + c[2 * m + i] * dx2 + c[3 * m + i] * (dx2 * dx);
}

// One lane's ConstantSpeed walker.  knots_lds holds the n knots followed by kKnotPad
// entries of +inf (the walk reads up to kAhead knots past its segment unguarded).
constexpr int kAhead = 8;
constexpr int kKnotPad = kAhead;

// mu -> the bracketing speed profiles (planner.py:48-62): below mus[0] -> profile 0, above
// mus[M-1] -> the last; else i = first mus[i] >= mu, lo = i-1 (i == 0 wraps to M-1, as the
// reference's negative index does); v = (v_lo wa) / den + (v_hi wb) / den.
struct MuBracket {
  int lo, hi;
  bool single;               // mu outside [mus[0], mus[M-1]]: one profile, no interpolation
  double wa, wb, den;
};
__device__ __host__ __forceinline__ MuBracket mu_bracket(const double* mus, int M, double mu) {
  MuBracket b;
  b.single = mu < mus[0] || mu > mus[M - 1];        // NaN: the interpolation branch, as the
  if (b.single) {                                   // reference's comparisons fall through
    b.lo = b.hi = (mu > mus[M - 1]) ? M - 1 : 0;
    b.wa = 1.0;
    b.wb = 0.0;
    b.den = 1.0;
  } else {
    // i = the first mus[i] >= mu among i < M - 1, else M - 1 (NaN mu: M - 1): with mus
    // ascending, the count of !(mus[j] >= mu), j < M - 1 — independent reads, no loop
    int i = 0;
    for (int j = 0; j < M - 1; ++j) i += (int)!(mus[j] >= mu);
    b.hi = i;
    b.lo = (i == 0) ? M - 1 : i - 1;
    b.wa = mus[b.hi] - mu;
    b.wb = mu - mus[b.lo];
    b.den = mus[b.hi] - mus[b.lo];
  }
  return b;
}

struct RaceRef {
  double s, v, L, scale, Ts;
  double wa, wb, den;        // v = (v_lo (hi-mu)) / (hi-lo) + (v_hi (mu-lo)) / (hi-lo)
  double kseg;               // knots[seg]
  int lo, hi, seg;
  bool single;               // mu outside [mus[0], mus[M-1]]: one profile, no interpolation

  // mu -> bracketing profiles (mu_bracket).
  // seg0 >= 0: the start segment (the same for every model of a launch: the caller's one
  // bisection); < 0: bisect here.
  __device__ __host__ __forceinline__ void init(const RacelineK& r, const double* knots_lds,
                                       const double* mus_lds, double mu, double s0, double v0,
                                       double scale_, double Ts_, int seg0 = -1) {
    L = knots_lds[r.n - 1];
    scale = scale_;
    Ts = Ts_;
    s = s0;
    v = fmax(v0, 0.01);                                             // planner.py:34
    const MuBracket b = mu_bracket(mus_lds, r.M, mu);
    lo = b.lo;
    hi = b.hi;
    single = b.single;
    wa = b.wa;
    wb = b.wb;
    den = b.den;
    // initial segment: bisect-right on the knots, clamped to the last segment
    if (seg0 >= 0) {
      seg = seg0;
    } else {
      int a = 0, b = r.n - 1;
      while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (knots_lds[m] <= s) a = m;
        else b = m;
      }
      seg = a;
    }
    kseg = knots_lds[seg];
  }

  // Advance one horizon step; returns xref_{k+1} in (xr, yr) and updates v.
  // Latency shape (one lane walks serially, so each step is a chain of LDS round trips):
  // the advance's knot reads are unconditional (the +inf pad, no per-read branch), the
  // segment's own knot is carried from the step before (kseg) and the new one selected
  // from the reads, and the window / global speed reads are separate paths (a merged
  // pointer would be a flat load, which waits on the step's global stores as well): two
  // round trips a step.
  __device__ __host__ __forceinline__ void step(const RacelineK& r, const double* knots_lds,
                                       const double* xy_lds, const SpeedWin& sw, double& xr,
                                       double& yr) {
    double t = s + scale * v * Ts;                                  // planner.py:41
    if (!(t >= 0.0 && t < L)) {                                     // :42 Python float %
      double r = fmod(t, L);                                        // (t - L exactly for
      if (r != 0.0 && r < 0.0) r += L;                              //  L <= t < 2L)
      t = (r == 0.0) ? 0.0 : r;
    }
    s = t;
    const int m = r.n - 1;
    if (t < kseg) {                                                 // wrapped past the lap end
      seg = 0;
      kseg = knots_lds[0];
    }
    // forward to the segment holding t: up to kAhead knots tested at once (the knots
    // ascend, so the count of those <= t is the advance), the loop after a full window.
    // knots[m] = L > t and the +inf pad after it stop the count at the last segment.
    double kk[kAhead + 1];
    kk[0] = kseg;
#pragma unroll
    for (int j = 1; j <= kAhead; ++j) kk[j] = knots_lds[seg + j];
    int adv = 0;
#pragma unroll
    for (int j = 1; j <= kAhead; ++j) adv += (int)(kk[j] <= t);
    double kn = kk[0];
#pragma unroll
    for (int j = 1; j <= kAhead; ++j) kn = adv == j ? kk[j] : kn;
    seg += adv;
    if (adv == kAhead) {
      while (seg < m - 1 && knots_lds[seg + 1] <= t) ++seg;
      kn = knots_lds[seg];
    }
    kseg = kn;
    const double dx = t - kn;
    xr = spline_at(xy_lds, m, seg, dx);                             // :43 calc_position
    yr = spline_at(xy_lds + 4 * m, m, seg, dx);
    int j = seg - sw.seg0;                                          // the window's column
    if (j < 0) j += m;
    const bool inw = sw.w != nullptr && j < sw.W;
    const int jw = inw ? j : 0;                                     // a valid column either way
    const double* wl = inw ? sw.w : xy_lds;                         // (no window: any LDS row)
    const int Ww = inw ? sw.W : m;
    double vb = spline_at(wl + (size_t)(inw ? lo * 4 * Ww : 0), Ww, jw, dx);
    double va = single ? 0.0 : spline_at(wl + (size_t)(inw ? hi * 4 * Ww : 0), Ww, jw, dx);
    if (!inw) {
      vb = spline_at(r.speed + (size_t)lo * 4 * m, m, seg, dx);
      if (!single) va = spline_at(r.speed + (size_t)hi * 4 * m, m, seg, dx);
    }
    v = single ? vb : vb * wa / den + va * wb / den;                // :58-60
  }
};

}  // namespace llampc
