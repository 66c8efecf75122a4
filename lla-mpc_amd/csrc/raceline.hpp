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
// rows); speed [M][4][n-1]; mus [M] ascending.  Knots and xy are staged in LDS per block;
// the speed profiles are read from global memory (M profiles do not fit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llampc {

struct RacelineK {
  const double* knots;   // [n]
  const double* xy;      // [2][4][n-1]
  const double* speed;   // [M][4][n-1]
  const double* mus;     // [M]
  int32_t n, M;
};

__device__ __host__ __forceinline__ double spline_at(const double* c, int m, int i, double dx) {
  // c: [4][m] rows a, b, c, d; pycubicspline.py:47-65 order a + b dx + c dx^2 + d dx^3
  const double dx2 = dx * dx;
  return c[i] + c[m + i] * dx + c[2 * m + i] * dx2 + c[3 * m + i] * (dx2 * dx);
}

// One lane's ConstantSpeed walker.
struct RaceRef {
  double s, v, L, scale, Ts;
  double wa, wb, den;        // v = (v_lo (hi-mu)) / (hi-lo) + (v_hi (mu-lo)) / (hi-lo)
  int lo, hi, seg;
  bool single;               // mu outside [mus[0], mus[M-1]]: one profile, no interpolation

  // mu -> bracketing profiles (planner.py:48-62): below mus[0] -> profile 0, above
  // mus[M-1] -> the last; else i = first mus[i] >= mu, lo = i-1 (i == 0 wraps to M-1, as
  // the reference's negative index does).
  __device__ __host__ __forceinline__ void init(const RacelineK& r, const double* knots_lds, double mu,
                                       double s0, double v0, double scale_, double Ts_) {
    const int M = r.M;
    L = knots_lds[r.n - 1];
    scale = scale_;
    Ts = Ts_;
    s = s0;
    v = fmax(v0, 0.01);                                             // planner.py:34
    single = mu < r.mus[0] || mu > r.mus[M - 1];   // NaN: the interpolation branch, as the
    if (single) {                                   // reference's comparisons fall through
      lo = hi = (mu > r.mus[M - 1]) ? M - 1 : 0;
      wa = 1.0;
      wb = 0.0;
      den = 1.0;
    } else {
      int i = 0;
      while (i < M - 1 && !(r.mus[i] >= mu)) ++i;
      hi = i;
      lo = (i == 0) ? M - 1 : i - 1;
      wa = r.mus[hi] - mu;
      wb = mu - r.mus[lo];
      den = r.mus[hi] - r.mus[lo];
    }
    // initial segment: bisect-right on the knots, clamped to the last segment
    int a = 0, b = r.n - 1;
    while (b - a > 1) {
      const int m = (a + b) >> 1;
      if (knots_lds[m] <= s) a = m;
      else b = m;
    }
    seg = a;
  }

  // Advance one horizon step; returns xref_{k+1} in (xr, yr) and updates v.
  __device__ __host__ __forceinline__ void step(const RacelineK& r, const double* knots_lds,
                                       const double* xy_lds, double& xr, double& yr) {
    double t = s + scale * v * Ts;                                  // planner.py:41
    if (!(t >= 0.0 && t < L)) {                                     // :42 Python float %
      double r = fmod(t, L);                                        // (t - L exactly for
      if (r != 0.0 && r < 0.0) r += L;                              //  L <= t < 2L)
      t = (r == 0.0) ? 0.0 : r;
    }
    s = t;
    const int m = r.n - 1;
    if (t < knots_lds[seg]) seg = 0;                                // wrapped past the lap end
    while (seg < m - 1 && knots_lds[seg + 1] <= t) ++seg;
    const double dx = t - knots_lds[seg];
    xr = spline_at(xy_lds, m, seg, dx);                             // :43 calc_position
    yr = spline_at(xy_lds + 4 * m, m, seg, dx);
    const double vb = spline_at(r.speed + (size_t)lo * 4 * m, m, seg, dx);
    if (single) {
      v = vb;
    } else {
      const double va = spline_at(r.speed + (size_t)hi * 4 * m, m, seg, dx);
      v = vb * wa / den + va * wb / den;                            // :58-60
    }
  }
};

}  // namespace llampc
