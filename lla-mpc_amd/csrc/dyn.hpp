// dyn.hpp — fp64 Pacejka dynamic-bicycle model and its integrators, register-resident,
// for gfx950 (CDNA4).  One lane owns one (model, candidate) state; nothing here touches
// memory.  Operation order follows the reference NumPy expressions so results agree with
// the CPU path to a few ulp (transcendentals: ocml vs NumPy/libm).
//
//   forces()      Dynamic.calc_forces_batch        llampc/models/dynamic.py:117-154
//   rhs<Form>()   Dynamic._diffequation_batch      dynamic.py:98-115   (Form::Ref)
//                 Dynamic.casadi                   dynamic.py:195-226  (Form::Nlp)
//   rk4_step()    odeintRK4_batch, one step        llampc/utils/rk6.py:50-68
//   rk6_step()    odeintRK6, one step              rk6.py:13-28
//   euler_step()  x + Ts*f (NLP transcription)     llampc/mpc/nmpc.py:58-60
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fastmath.hpp"

// Transcendentals of the model: the short-chain versions (fastmath.hpp) by default;
// -DLLAMPC_OCML_MATH selects ocml's for A/B measurements.
#ifdef LLAMPC_OCML_MATH
#define LL_ATAN2P(y, x) atan2((y), (x))
#define LL_ATAN(z) atan(z)
#define LL_SIN(a) sin(a)
#define LL_SINCOS(a, s, c) sincos((a), (s), (c))
#else
#define LL_ATAN2P(y, x) ::llampc::fm::atan2_xpos((y), (x))
#define LL_ATAN(z) ::llampc::fm::atan_(z)
#define LL_SIN(a) ::llampc::fm::sin_(a)
#define LL_SINCOS(a, s, c) ::llampc::fm::sincos_((a), (s), (c))
#endif

namespace llampc {

// Per-bank constants in kernel-argument space (wave-uniform → SGPRs).
struct VehK {
  double lf, lr, mass, inv_mass, inv_Iz;   // inv_* = 1/mass, 1/Iz as the reference's
  double Cm1, Cm2, Cr0, Cr2;               //   `1/self.mass * (...)` (dynamic.py:111-113)
  int32_t input_acc, approx;
};

struct Tire {  // one model's Pacejka coefficients (bank SoA rows, rt.py:179 order)
  double Bf, Cf, Df, Br, Cr, Dr;
};

struct Forces {
  double Ffy, Frx, Fry, af, ar;
};

enum class Form { Ref, Nlp };

// dynamic.py:117-154 (batch) == :156-193 (scalar): tire + motor forces.
template <Form F>
__device__ __host__ __forceinline__ Forces forces(const VehK& v, const Tire& t, double vx,
                                                  double vy, double om, double pwm,
                                                  double delta) {
  Forces f;
  if (v.approx) {                      // dynamic.py:126-136 (Rajamani linear tires)
    f.Frx = v.mass * pwm;
    f.af = delta - (v.lf * om + vy) / vx;
    f.ar = (v.lr * om - vy) / vx;
    f.Ffy = 2 * t.Cf * f.af;
    f.Fry = 2 * t.Cr * f.ar;
    return f;
  }
  f.Frx = v.input_acc ? v.mass * pwm                                   // dynamic.py:141
                      : (v.Cm1 - v.Cm2 * vx) * pwm - v.Cr0 - v.Cr2 * (vx * vx);  // :146
  // Ref form: atan2(., |vx|) (dynamic.py:149-150); NLP form: atan2(., vx) (:215-216)
  const double den = (F == Form::Ref) ? fabs(vx) : vx;
  f.af = delta - LL_ATAN2P(v.lf * om + vy, den);
  f.ar = LL_ATAN2P(v.lr * om - vy, den);
  f.Ffy = t.Df * LL_SIN(t.Cf * LL_ATAN(t.Bf * f.af));                // dynamic.py:151
  f.Fry = t.Dr * LL_SIN(t.Cr * LL_ATAN(t.Br * f.ar));                // dynamic.py:152
  return f;
}

// Input of one integration step: pwm/accel, steering and sin/cos of the steering.
struct Input {
  double a, d, sd, cd;
};

__device__ __host__ __forceinline__ Input make_input(double a, double d) {
  Input u;
  u.a = a;
  u.d = d;
  LL_SINCOS(d, &u.sd, &u.cd);
  return u;
}

// dx/dt.  Form::Ref = dynamic.py:98-115; Form::Nlp = dynamic.py:195-226 (vmin clamp).
template <Form F>
__device__ __host__ __forceinline__ void rhs(const VehK& v, const Tire& t, const double* x,
                                             const Input& u, double* dx) {
  double vx = x[3], vy = x[4], om = x[5];
  double d = u.d, sd = u.sd, cd = u.cd;
  if (F == Form::Nlp) {
    const double vmin = 0.05;                                        // dynamic.py:208
    if (vx < vmin) {                                                 // dynamic.py:209-212
      vy = 0.0;
      om = 0.0;
      d = 0.0;
      sd = 0.0;
      cd = 1.0;
      vx = vmin;
    }
  }
  const Forces f = forces<F>(v, t, vx, vy, om, u.a, d);
  double sp, cp;
  LL_SINCOS(x[2], &sp, &cp);
  dx[0] = vx * cp - vy * sp;
  dx[1] = vx * sp + vy * cp;
  dx[2] = om;
  dx[3] = v.inv_mass * (f.Frx - f.Ffy * sd) + vy * om;
  dx[4] = v.inv_mass * (f.Fry + f.Ffy * cd) - vx * om;
  dx[5] = v.inv_Iz * (f.Ffy * v.lf * cd - f.Fry * v.lr);
}

// One classic RK4 step (rk6.py:58-66).  The weighted sum is accumulated in the
// reference's left-to-right order ((k1 + 2k2) + 2k3) + k4, then / 6.
__device__ __host__ __forceinline__ void rk4_step(const VehK& v, const Tire& t, double* x,
                                                  const Input& u, double h) {
  double y[6], d[6], acc[6];
  rhs<Form::Ref>(v, t, x, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = k;
    y[i] = x[i] + k / 2;
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = acc[i] + 2 * k;
    y[i] = x[i] + k / 2;
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = acc[i] + 2 * k;
    y[i] = x[i] + k;
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = x[i] + (acc[i] + h * d[i]) / 6;
}

// x_{k+1} = x_k + Ts * f_nlp(x_k, u_k)  (nmpc.py:58-60 equality constraints).
__device__ __host__ __forceinline__ void euler_nlp_step(const VehK& v, const Tire& t, double* x,
                                                        const Input& u, double h) {
  double d[6];
  rhs<Form::Nlp>(v, t, x, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = x[i] + h * d[i];
}

// One odeintRK6 step (rk6.py:18-27), stage coefficients as the reference writes them.
__device__ __host__ __forceinline__ void rk6_step(const VehK& v, const Tire& t, double* x,
                                                  const Input& u, double h) {
  double k1[6], k2[6], k3[6], k4[6], k5[6], k6[6], y[6], d[6];
  rhs<Form::Ref>(v, t, x, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) { k1[i] = h * d[i]; y[i] = x[i] + k1[i] / 4; }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    k2[i] = h * d[i];
    y[i] = x[i] + (3.0 / 32) * k1[i] + (9.0 / 32) * k2[i];
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    k3[i] = h * d[i];
    y[i] = x[i] + (1932.0 / 2197) * k1[i] - (7200.0 / 2197) * k2[i] + (7296.0 / 2197) * k3[i];
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    k4[i] = h * d[i];
    y[i] = x[i] + (439.0 / 216) * k1[i] - 8 * k2[i] + (3680.0 / 513) * k3[i] -
           (845.0 / 4104) * k4[i];
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    k5[i] = h * d[i];
    y[i] = x[i] - (8.0 / 27) * k1[i] + 2 * k2[i] - (3544.0 / 2565) * k3[i] +
           (1859.0 / 4104) * k4[i] - (11.0 / 40) * k5[i];
  }
  rhs<Form::Ref>(v, t, y, u, d);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    k6[i] = h * d[i];
    // gamma @ K (rk6.py:14,26): gamma_1 = 0
    const double g = (16.0 / 135) * k1[i] + 0.0 * k2[i] + (6656.0 / 12825) * k3[i] +
                     (28561.0 / 56430) * k4[i] + (-9.0 / 50) * k5[i] + (2.0 / 55) * k6[i];
    x[i] = x[i] + g;
  }
}

template <int INTEG>
__device__ __host__ __forceinline__ void step(const VehK& v, const Tire& t, double* x,
                                              const Input& u, double h) {
  if (INTEG == 0) rk4_step(v, t, x, u, h);
  else if (INTEG == 1) euler_nlp_step(v, t, x, u, h);
  else rk6_step(v, t, x, u, h);
}

// ------------------------------------------------------------------------------------
// Lane-split evaluation (latency regime).  LPM lanes (a pair or a quad of consecutive
// lanes) carry the SAME state; each lane runs ONE transcendental chain of the stage with
// an identical instruction stream (lane-dependent operands via selects, no divergence),
// and the results are exchanged with DPP quad_perm broadcasts:
//   LPM=2: lane 0 front tire   atan2 -> atan -> sin -> Ffy   (+ sincos(psi) in both)
//          lane 1 rear tire    atan2 -> atan -> sin -> Fry
//   LPM=4: lane 0 sin(psi), lane 1 Ffy, lane 2 Fry, lane 3 cos(psi): one
//          atan2 -> atan -> sincos chain per lane (lanes 0/3 discard their atan results)
// Every lane then forms dx/dt and the integrator update redundantly (cheap, identical).
// ------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_bcast(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// quad_perm encodings: broadcast lane k of each quad = k * 0x55; pairs [0,0,2,2] = 0xA0,
// [1,1,3,3] = 0xF5.
constexpr int kQuad0 = 0x00, kQuad1 = 0x55, kQuad2 = 0xAA, kQuad3 = 0xFF;
constexpr int kPair0 = 0xA0, kPair1 = 0xF5;

template <Form F, int LPM>
__device__ __forceinline__ void rhs_split(const VehK& v, const Tire& t, const double* x,
                                          const Input& u, double* dx, int sub) {
  if (LPM == 1 || v.approx) {           // wave-uniform: no transcendental chains to split
    rhs<F>(v, t, x, u, dx);
    return;
  }
  double vx = x[3], vy = x[4], om = x[5];
  double d = u.d, sd = u.sd, cd = u.cd;
  if (F == Form::Nlp) {
    const double vmin = 0.05;
    if (vx < vmin) {                    // same state in every lane of the group: uniform per group
      vy = 0.0;
      om = 0.0;
      d = 0.0;
      sd = 0.0;
      cd = 1.0;
      vx = vmin;
    }
  }
  const bool front = (LPM == 2) ? (sub == 0) : (sub == 1);
  const double den = (F == Form::Ref) ? fabs(vx) : vx;
  const double yy = front ? (v.lf * om + vy) : (v.lr * om - vy);
  const double a2 = LL_ATAN2P(yy, den);
  const double slip = front ? (d - a2) : a2;
  const double B = front ? t.Bf : t.Br, Cc = front ? t.Cf : t.Cr, D = front ? t.Df : t.Dr;
  double arg = Cc * LL_ATAN(B * slip);
  double Ffy, Fry, sp, cp;
  if (LPM == 2) {
    const double r = D * LL_SIN(arg);
    Ffy = dpp_bcast<kPair0>(r);
    Fry = dpp_bcast<kPair1>(r);
    LL_SINCOS(x[2], &sp, &cp);
  } else {
    const bool psi_lane = (sub == 0) | (sub == 3);
    arg = psi_lane ? x[2] : arg;
    double s, c;
    LL_SINCOS(arg, &s, &c);
    const double r = (sub == 3) ? c : (psi_lane ? s : D * s);
    sp = dpp_bcast<kQuad0>(r);
    Ffy = dpp_bcast<kQuad1>(r);
    Fry = dpp_bcast<kQuad2>(r);
    cp = dpp_bcast<kQuad3>(r);
  }
  const double Frx = v.input_acc ? v.mass * u.a : (v.Cm1 - v.Cm2 * vx) * u.a - v.Cr0 - v.Cr2 * (vx * vx);
  dx[0] = vx * cp - vy * sp;
  dx[1] = vx * sp + vy * cp;
  dx[2] = om;
  dx[3] = v.inv_mass * (Frx - Ffy * sd) + vy * om;
  dx[4] = v.inv_mass * (Fry + Ffy * cd) - vx * om;
  dx[5] = v.inv_Iz * (Ffy * v.lf * cd - Fry * v.lr);
}

template <int LPM>
__device__ __forceinline__ void rk4_step_split(const VehK& v, const Tire& t, double* x,
                                               const Input& u, double h, int sub) {
  double y[6], d[6], acc[6];
  rhs_split<Form::Ref, LPM>(v, t, x, u, d, sub);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = k;
    y[i] = x[i] + k / 2;
  }
  rhs_split<Form::Ref, LPM>(v, t, y, u, d, sub);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = acc[i] + 2 * k;
    y[i] = x[i] + k / 2;
  }
  rhs_split<Form::Ref, LPM>(v, t, y, u, d, sub);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double k = h * d[i];
    acc[i] = acc[i] + 2 * k;
    y[i] = x[i] + k;
  }
  rhs_split<Form::Ref, LPM>(v, t, y, u, d, sub);
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = x[i] + (acc[i] + h * d[i]) / 6;
}

template <int INTEG, int LPM>
__device__ __forceinline__ void step_split(const VehK& v, const Tire& t, double* x,
                                           const Input& u, double h, int sub) {
  if (LPM == 1) {
    step<INTEG>(v, t, x, u, h);
  } else if (INTEG == 0) {
    rk4_step_split<LPM>(v, t, x, u, h, sub);
  } else if (INTEG == 1) {
    double d[6];
    rhs_split<Form::Nlp, LPM>(v, t, x, u, d, sub);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = x[i] + h * d[i];
  } else {
    step<INTEG>(v, t, x, u, h);        // RK6 (plant) stays one lane per rollout
  }
}

// ------------------------------------------------------------------------------------
// Ordering keys (value, index).  Total orders; indices are unique so ties never remain.
// NaN-last: np.argsort order (rt.py:360) and the look-ahead argmin.
// NaN-first: np.argmin (rt.py:359) — the first NaN wins.
// ------------------------------------------------------------------------------------
__device__ __host__ __forceinline__ bool less_nan_last(double av, int64_t ai, double bv,
                                                       int64_t bi) {
  const bool an = av != av, bn = bv != bv;
  if (an | bn) return (an & bn) ? (ai < bi) : bn;
  return (av < bv) || (av == bv && ai < bi);
}

__device__ __host__ __forceinline__ bool less_nan_first(double av, int64_t ai, double bv,
                                                        int64_t bi) {
  const bool an = av != av, bn = bv != bv;
  if (an | bn) return (an & bn) ? (ai < bi) : an;
  return (av < bv) || (av == bv && ai < bi);
}

__device__ __host__ __forceinline__ bool key_less(bool nan_first, double av, int64_t ai,
                                                  double bv, int64_t bi) {
  return nan_first ? less_nan_first(av, ai, bv, bi) : less_nan_last(av, ai, bv, bi);
}

constexpr int64_t kNoIndex = INT64_MAX;   // sentinel index: sorts after every real key
                                          // (value +inf under NaN-first, NaN under NaN-last)

}  // namespace llampc
