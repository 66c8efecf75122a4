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

// Transcendentals of the model: the short-chain versions (fastmath.hpp).
#define LL_ATAN2P(y, x) ::llampc::fm::atan2_xpos((y), (x))
#define LL_ATAN(z) ::llampc::fm::atan_(z)
#define LL_SIN(a) ::llampc::fm::sin_(a)
#define LL_SINCOS(a, s, c) ::llampc::fm::sincos_((a), (s), (c))
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
  // Dynamic.casadi (Form::Nlp) always uses the pwm motor model and the Pacejka tires
  // (dynamic.py:214-218), whatever input_acc / approx say
  if (F == Form::Ref && v.approx) {    // dynamic.py:126-136 (Rajamani linear tires)
    f.Frx = v.mass * pwm;
    f.af = delta - (v.lf * om + vy) / vx;
    f.ar = (v.lr * om - vy) / vx;
    f.Ffy = 2 * t.Cf * f.af;
    f.Fry = 2 * t.Cr * f.ar;
    return f;
  }
  f.Frx = (F == Form::Ref && v.input_acc) ? v.mass * pwm              // dynamic.py:141
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
  for (int i = 0; i < 6; ++i) x[i] = x[i] + fm::div6(acc[i] + h * d[i]);
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
// Rollout stage of the look-ahead (the hot loop).  One stage of odeintRK4_batch
// (rk6.py:58-66) is dx/dt of dynamic.py:98-115 (Ref) / :195-226 (Nlp); its cost is two
// serial transcendental chains — front and rear tire, atan2 -> atan -> sin — plus
// sincos(psi).  With ~1 wave per SIMD a wave pays for every instruction it issues and for
// every branch/select latency on its chains (tools/micro), so this path
//  * evaluates each chain with the branch-free cores of fastmath.hpp and re-does the rare
//    lanes whose operands leave the cores' domains with the general rhs<F>, behind ONE
//    wave-uniform branch per stage that is normally not taken.  Which cores a lane used
//    depends only on its own operands, never on the other rollouts sharing the wave;
//  * LPM = 2 splits the two chains over a lane pair (lane 0 front, lane 1 rear; exchanged
//    with DPP) — the latency regime, fewer waves than SIMDs; LPM = 1 runs both chains in
//    one lane — the throughput regime (fewest instructions per rollout).
// ------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_bcast(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
// (The same quad_perm through the LDS crossbar, ds_swizzle_b32 QDMode, measured slower in
// round 2: the broadcasts stay DPP.)
template <int CTRL, int BIT>
__device__ __forceinline__ double quad_bcast(double v) {
  return dpp_bcast<CTRL>(v);
}
// quad_perm broadcasts within lane pairs: [0,0,2,2] = 0xA0, [1,1,3,3] = 0xF5; within a
// quad: lane q to all four = 0x00, 0x55, 0xAA, 0xFF; xor-1 / xor-2 swaps = 0xB1, 0x4E.
constexpr int kPair0 = 0xA0, kPair1 = 0xF5;
constexpr int kQuad0 = 0x00, kQuad1 = 0x55, kQuad2 = 0xAA, kQuad3 = 0xFF;
constexpr int kQuadX1 = 0xB1, kQuadX2 = 0x4E;
// Position split (LPM = 4): lanes with pc = 0 (0, 2) carry X, pc = 1 (1, 3) carry Y.  A =
// [3,2,3,2] (X lanes get h cos psi, Y lanes h sin psi), B = [2,3,2,3] (the other one).
constexpr int kQuadPosA = 0xBB, kQuadPosB = 0xEE;

// One tire's constants in this lane: front (lw = lf, sg = +1) or rear (lw = lr, sg = -1).
struct Chain {
  double lw, sg, B, C, D;
  double nsB;   // -sg B (chain_fold: z = fma(nsB, atan2, B dsel))
};

__device__ __host__ __forceinline__ Chain make_chain(const VehK& v, const Tire& t, bool front) {
  return front ? Chain{v.lf, 1.0, t.Bf, t.Cf, t.Df, -t.Bf} : Chain{v.lr, -1.0, t.Br, t.Cr, t.Dr, t.Br};
}

// Static part of the fast chain's domain: |C atan(.)| <= |C| pi/2 must stay inside
// sin_wide's |a| <= 3 (|C| <= 1.9 -> 2.985; NaN -> false).
// Static part of the domain: |C| <= 1.9 (sin_wide's range), finite B and D (so a NaN in
// the chain always comes from a NaN state or input, which reaches the rollout's result).
__device__ __host__ __forceinline__ bool chain_static_ok(const Chain& c) {
  return (int)(fabs(c.C) <= 1.9) & (int)(fabs(c.B) <= 1e300) & (int)(fabs(c.D) <= 1e300) &
         (int)(fabs(c.lw) <= 1e300);
}

// Running extremes of the fast cores' operands over a rollout (or a look-back step): the
// domain is judged once at the end instead of per stage (a compare + mask OR per operand
// cost ~15 issue slots per stage).  hi / lo = max / min of the atan2 divisors max(|y|, x);
// ps = max |psi|.  ok(): hi in [2^-1000, 2^999] (a larger divisor's reciprocal may flush to
// zero: a wrong finite angle; a smaller one — 0/0 at standstill — gives a NaN that the atan
// core's min/max would swallow) and |psi| <= kSinCosMax (the fold's range).  The atan
// divisor max(|z|, 1) needs no record: |z| > 2^1000 yields pi/2 exactly as atan does and an
// infinite z a NaN that reaches the state (and, through the positions, the cost); the
// callers re-run every lane whose result is not finite.  fmax/fmin skip a NaN operand, but
// a NaN operand comes from a NaN state, input or parameter and reaches the lane's result.
struct Dom {
  double hi, lo, ps;
  __device__ __forceinline__ void init() {
    hi = 0.0;
    lo = __builtin_inf();
    ps = 0.0;
  }
  __device__ __forceinline__ bool ok() const {
    return (int)(hi <= 0x1p999) & (int)(lo >= 0x1p-1000) & (int)(ps <= fm::kSinCosMax);
  }
  // chain_pair (one reciprocal per front/rear pair): the atan2 divisors in [2^-500, 2^499]
  // and the atan divisors' product (>= 1) at most 2^499, so every divisor and product of
  // two stays a normal number (fastmath.hpp atan_ratio_pair)
  __device__ __forceinline__ bool ok_paired() const {
    return (int)(hi <= 0x1p499) & (int)(lo >= 0x1p-500) & (int)(ps <= fm::kSinCosMax);
  }
};

// (Round 3 measured the LPM-1 lane's front and rear chains with one reciprocal per division
// pair, chain_pair: 16 -> 8 v_rcp_f64 but 843 -> 858 instructions per step, C = 64 375-380 ->
// 383-385 us per tick, profiles/r03/v31/ab_pair_c64.log; the rollouts keep two chain_fast.)

// F = D sin(C atan(B slip)) with slip = dsel - atan2(yy, den) for the front tire
// (dsel = delta) and atan2(yy, den) for the rear (dsel = 0); yy = lf om + vy | lr om - vy
// (dynamic.py:149-152 / :215-220).  The divisors go to the lane's Dom.  LO = false: the
// caller records the lower bound itself (the LPM-1 lane: |den| once for both chains — the
// divisor max(|yy|, |den|) is at least |den|, so min |den| >= 2^-1000 is a sufficient test,
// stricter only at a standstill, which then takes the general path).
template <bool LEAN = false, bool LO = true>
__device__ __forceinline__ double chain_fast(const Chain& c, double den, double vy, double om,
                                             double dsel, Dom& dm, const fm::FmK& K) {
  const double yy = fma(c.lw, om, c.sg * vy);
  double h2;
  const double a2 = fm::atan2_fast<LEAN>(yy, den, K, h2);
  const double z = c.B * fma(-c.sg, a2, dsel);
  const double at = fm::atan_fast<LEAN>(z, K);
  if constexpr (LO) dm.lo = fm::vmin(dm.lo, h2);
  dm.hi = fm::vmax(dm.hi, h2);
  return c.D * fm::sin_wide<LEAN>(c.C * at, K);
}

// Both chains of an LPM-1 lane (front: dsel = delta, rear: dsel = 0) with their divisions
// paired (fastmath.hpp atan2_fast_pair / atan_fast_pair): the same lean evaluation as two
// chain_fast<true> up to the division's roundings; the domain is Dom::ok_paired.
__device__ __forceinline__ void chain_pair(const Chain& cf, const Chain& cr, double den, double vy,
                                           double om, double d, Dom& dm, const fm::FmK& K,
                                           double& Ff, double& Fr) {
  const double yf = fma(cf.lw, om, cf.sg * vy), yr = fma(cr.lw, om, cr.sg * vy);
  double af, ar, hf, hr, dp;
  fm::atan2_fast_pair(yf, yr, den, K, af, ar, hf, hr, dp);
  const double zf = cf.B * fma(-cf.sg, af, d), zr = cr.B * fma(-cr.sg, ar, 0.0);
  double tf, tr, dz;
  fm::atan_fast_pair(zf, zr, K, tf, tr, dz);
  dm.lo = fm::vmin(dm.lo, fm::vmin(hf, hr));
  dm.hi = fm::vmax(dm.hi, fm::vmax(hf, hr));
  dm.hi = fm::vmax(dm.hi, dz);
  Ff = cf.D * fm::sin_wide<true>(cf.C * tf, K);
  Fr = cr.D * fm::sin_wide<true>(cr.C * tr, K);
}

// LPM = 4: the quad's lanes run ONE instruction stream — lanes 0/1 the front/rear chain,
// lanes 2/3 the same chains (wasted) up to the final sine, whose argument is theirs:
// lane 2 sin(psi), lane 3 cos(psi), so sincos(psi) costs no polynomial of its own.
// psi = r + k pi (2k = nearest even integer to psi 2/pi, 3-part Cody-Waite by pi/2, |r| <=
// pi/2); sin psi = sin((-1)^k r), cos psi = sin((-1)^k (pi/2 - |r|)).  Per lane:
// c.C = C (lanes 0/1) or 0 (2/3), c.D = D or 1, ra = the |r| mask of the high word (lane 3
// clears the sign), pm = 0 / 1 / -1 and po = 0 / 0 / pi/2 place the angle argument
// po + pm r' (exactly 0 in lanes 0/1, so their argument is C atan(.) as at LPM 1/2).
// SCALED: psi arrives as Psi = (2/pi) psi (the fused quad's state, step_fused): k2 = the
// even integer nearest Psi, r = (Psi - k2) pi/2 — the subtraction is exact (|Psi| < 2^51),
// so the fold is 4 instructions instead of the 3-part Cody-Waite's 5.
template <bool SCALED = false, bool LEAN = false>
__device__ __forceinline__ double chain_fold(const Chain& c, double den, double vy, double om,
                                             double Bd, double psi, int ra, double pm,
                                             double po, Dom& dm, const fm::FmK& K) {
  double t2, r;
  if constexpr (SCALED) {
    t2 = psi + K.rmagic2;                                // 2^53 (1.5 + 2k 2^-53): ulp 2
    const double k2 = t2 - K.rmagic2;
    r = (psi - k2) * K.pio2;
  } else {
    t2 = fma(psi, K.two_pi, K.rmagic2);
    const double k2 = t2 - K.rmagic2;
    r = fma(-k2, K.cw0, psi);
    r = fma(-k2, K.cw1, r);
    r = fma(-k2, K.cw2, r);
  }
  const double rr = __hiloint2double(__double2hiint(r) & ra, __double2loint(r));
  const double pa = fma(pm, rr, po);
  const int fs = __double2loint(t2) << 31;               // (-1)^k on the argument
  const double arg_psi = __hiloint2double(__double2hiint(pa) ^ fs, __double2loint(pa));
  double at;
  {
    const double yy = fma(c.lw, om, c.sg * vy);
    double h2;
    const double a2 = fm::atan2_fast<LEAN>(yy, den, K, h2);
    const double z = fma(c.nsB, a2, Bd);                  // B (dsel - sg a2)
    at = fm::atan_fast<LEAN>(z, K);
    dm.lo = fm::vmin(dm.lo, h2);
    dm.hi = fm::vmax(dm.hi, h2);
  }
  return c.D * fm::sin_wide<LEAN>(fma(c.C, at, arg_psi), K);
}

// Per-rollout constants of the fast stage.  ch[0] is this lane's chain (LPM = 2) or the
// front chain and ch[1] the rear (LPM = 1); fw = 1 for a front lane, 0 for a rear lane;
// sok = the static domain (chain_static_ok of the lane's chains).
struct StageK {
  Chain ch[2];
  double fw;
  double k1, k2, k0, k3;   // Frx = (k1 - k2 vx) a - k0 - k3 vx^2; input_acc: (mass, 0, 0, 0)
  double pm, po;           // LPM = 4: the angle argument of chain_fold
  double psg;              // LPM = 4 position split: -1 on X lanes, +1 on Y lanes
  int ra;
  int pc;                  // LPM = 4 position split: the lane's component (0 = X, 1 = Y)
  bool sok;
};

// psi_scale: LPM = 4 lanes 2/3 return psi_scale sin(psi), psi_scale cos(psi) (the fused RK4
// passes h, so the stage increments need no h vx, h vy products).
template <int LPM>
__device__ __forceinline__ StageK make_stage(const VehK& v, const Tire& t, int sub,
                                             double psi_scale = 1.0) {
  const bool front = (LPM == 1) || (sub & 1) == 0;
  StageK s;
  s.ch[0] = make_chain(v, t, front);
  s.ch[1] = make_chain(v, t, false);
  s.fw = front ? 1.0 : 0.0;
  s.pm = sub == 2 ? 1.0 : (sub == 3 ? -1.0 : 0.0);
  s.po = sub == 3 ? fm::kPio2 : 0.0;
  s.ra = sub == 3 ? 0x7FFFFFFF : -1;
  s.pc = sub & 1;
  s.psg = (sub & 1) ? 1.0 : -1.0;
  // dynamic.py:141 (input_acc: mass * a) as the :146 form with (mass, 0, 0, 0): equal for
  // finite vx (a non-finite vx is outside the chain domain -> the general rhs)
  s.k1 = v.input_acc ? v.mass : v.Cm1;
  s.k2 = v.input_acc ? 0.0 : v.Cm2;
  s.k0 = v.input_acc ? 0.0 : v.Cr0;
  s.k3 = v.input_acc ? 0.0 : v.Cr2;
  s.sok = chain_static_ok(s.ch[0]) && ((LPM >= 2) || chain_static_ok(s.ch[1])) && !v.approx;
  if (LPM == 4 && sub >= 2) {   // lanes 2/3: the chain's sine takes the psi argument alone
    s.ch[0].C = 0.0;
    s.ch[0].D = psi_scale;
    // (their atan2 / atan duplicate lanes 0/1's chains; constant operands there instead
    // — yy = z = 0 — clocked 1.5 % higher but took 4.5 % more cycles)
  }
  return s;
}

// Tire forces and sin/cos(psi) of one fast stage, in every lane of the rollout.
struct StageF {
  double Ffy, Fry, sp, cp;
};
// Bd = B d fw, the chain's steering term (LPM = 4 only; formed once per step).
// SPLIT (LPM = 4, position split): sp/cp carry the split's A/B operands instead (X lanes:
// cos, sin; Y lanes: sin, cos — kQuadPosA/B).
template <int LPM, bool SPLIT = false, bool SCALED = false, bool LEAN = false>
__device__ __forceinline__ StageF forces_fast(const StageK& sk, double den, double vy, double om,
                                              double d, double psi, const fm::FmK& K, Dom& dm,
                                              double Bd = 0.0) {
  StageF f;
  dm.ps = fm::vmax_abs(psi, dm.ps);
  if (LPM == 4) {
    const double r = chain_fold<SCALED, LEAN>(sk.ch[0], den, vy, om, Bd, psi, sk.ra, sk.pm, sk.po, dm, K);
    f.Ffy = quad_bcast<kQuad0, 0>(r);
    f.Fry = quad_bcast<kQuad1, 1>(r);
    if constexpr (SPLIT) {
      f.sp = quad_bcast<kQuadPosA, 2>(r);
      f.cp = quad_bcast<kQuadPosB, 3>(r);
    } else {
      f.sp = quad_bcast<kQuad2, 2>(r);
      f.cp = quad_bcast<kQuad3, 3>(r);
    }
    return f;
  }
  if (LPM == 2) {
    const double r = chain_fast<LEAN>(sk.ch[0], den, vy, om, d * sk.fw, dm, K);
    f.Ffy = dpp_bcast<kPair0>(r);
    f.Fry = dpp_bcast<kPair1>(r);
  } else {
    f.Ffy = chain_fast<LEAN, false>(sk.ch[0], den, vy, om, d, dm, K);
    f.Fry = chain_fast<LEAN, false>(sk.ch[1], den, vy, om, 0.0, dm, K);
    dm.lo = fm::vmin_abs(den, dm.lo);
  }
  if constexpr (SCALED && LPM == 1) {
    // LPM = 1 with the scaled yaw Psi = (2/pi) psi (k_fused): the quad's fold in one lane —
    // psi = r + k pi, sin psi = sin((-1)^k r), cos psi = sin((-1)^k (pi/2 - |r|)), both by
    // sin_wide (|arg| <= pi/2).  As many instructions as sincos_fast, and the sincos
    // polynomials' and Cody-Waite's 17 constants (34 VGPRs) are not live in the loop.
    const double t2 = psi + K.rmagic2;                   // 2^53 (1.5 + 2k 2^-53): ulp 2
    const double k2 = t2 - K.rmagic2;
    const double r = (psi - k2) * K.pio2;
    const int fs = __double2loint(t2) << 31;             // (-1)^k on both arguments
    const double c = K.pio2 - fabs(r);
    f.sp = fm::sin_wide<LEAN>(__hiloint2double(__double2hiint(r) ^ fs, __double2loint(r)), K);
    f.cp = fm::sin_wide<LEAN>(__hiloint2double(__double2hiint(c) ^ fs, __double2loint(c)), K);
  } else {
    fm::sincos_fast(psi, &f.sp, &f.cp, K);
  }
  return f;
}

// dx/dt on the fast path.  No fallback and no domain test here: the operands go to `dm`;
// the caller judges dm (and sk.sok) once and re-runs an out-of-domain lane's rollout with
// the general evaluation (lookahead_block), so the stage has no branch at all.
template <Form F, int LPM>
__device__ __forceinline__ void rhs_fast(const VehK& v, const StageK& sk, const double* x,
                                         const Input& u, double* dx, const fm::FmK& K,
                                         Dom& dm) {
  double vx = x[3], vy = x[4], om = x[5];
  double d = u.d, sd = u.sd, cd = u.cd;
  if (F == Form::Nlp && vx < 0.05) {      // dynamic.py:208-212 (vmin clamp)
    vy = 0.0;
    om = 0.0;
    d = 0.0;
    sd = 0.0;
    cd = 1.0;
    vx = 0.05;
  }
  // den = vx: the fast atan2 takes |den| (Ref: atan2(., |vx|); Nlp: vx >= vmin after the clamp)
  const double Bd = sk.ch[0].B * (d * sk.fw);
  const StageF f = forces_fast<LPM>(sk, vx, vy, om, d, x[2], K, dm, Bd);
  const double Frx = (sk.k1 - sk.k2 * vx) * u.a - sk.k0 - sk.k3 * (vx * vx);
  dx[0] = vx * f.cp - vy * f.sp;
  dx[1] = vx * f.sp + vy * f.cp;
  dx[2] = om;
  dx[3] = v.inv_mass * (Frx - f.Ffy * sd) + vy * om;
  dx[4] = v.inv_mass * (f.Fry + f.Ffy * cd) - vx * om;
  dx[5] = v.inv_Iz * (f.Ffy * v.lf * cd - f.Fry * v.lr);
}

__device__ __forceinline__ Input make_input_fast(double a, double d, const fm::FmK& K,
                                                 bool& bad) {
  Input u;
  u.a = a;
  u.d = d;
  fm::sincos_fast(d, &u.sd, &u.cd, K);
  bad = (int)bad | (int)!fm::sincos_fast_ok(d);
  return u;
}

// Fused RK4 of the look-ahead rollouts: the stage increments k = h f(y) are formed directly
// (h folded into the force and geometry constants, Frx as a polynomial in vx with per-step
// coefficients) and the update is x + (k1 + 2k2 + 2k3 + k4) * (1/6) as one FMA — the
// arithmetic of rk4_step / dynamic.py:98-115 with other roundings of its products and sums
// (~1 ulp per step, the transcendental cores' class; tests/test_gpu_parity.py bounds the
// rollouts at 1e-7 relative).  42 fewer instructions per step than step_fast's reference
// roundings, which the look-back keeps (its errors are ranked, rt.py:359-360).
// The look-ahead's fused stages use the lean cores (fastmath.hpp kAtanRL / kSinWQL, the
// division without its residual step; the FmK of those rollouts is loaded with
// FmK::load<kLeanLA>()): ~1e-13 relative on the tire forces (8 terms, round 4; ~1e-14 with 9);
// 456 instructions per step at LPM 4 (467 with 9 terms, 494 with the precise 10-term cores,
// 507 in round 2), A/B 28.8 -> 27.2 us per tick with 9 terms (profiles/r03/ab_lean), 26.6
// with 8 (profiles/r04/ab_lean8.log).
constexpr bool kLeanLA = true;

struct FusedK {
  double h, hm, hIlf, hIlr, m1, m0, m2, m3;   // hm = h/m; m1 = hm k1, m0 = hm k0,
};                                            // m2 = hm k2, m3 = -hm k3 (StageK)

// The fused rollouts that carry the scaled yaw state (W = h omega, Psi = (2/pi) psi, see
// make_fused): the LPM-4 quad (round 2) and, from round 3, the LPM-1 lane (its sin/cos psi by
// the fold of forces_fast).
// LPM 2 keeps omega and psi.
constexpr bool scaled_yaw(int lpm) {
  return lpm == 4 || lpm == 1;
}
// SCALED (the LPM = 4 quad): the rollout state carries W = h omega and Psi = (2/pi) psi
// instead of omega and psi.  Then the yaw increment IS W (no h omega product), vy W and vx W
// are the h vy omega / h vx omega terms of the velocity increments, the omega increment
// takes one more factor h (hIlf, hIlr), the chains' lw / h turns W back into omega for the
// slip angles, and the yaw's RK4 weights carry 2/pi (FmK inv_pi, two_pi, inv_3pi) — the
// fold then needs no Cody-Waite (chain_fold<true>).  Same arithmetic up to roundings.
__device__ __forceinline__ FusedK make_fused(const VehK& v, const StageK& sk, double h,
                                             bool scaled = false) {
  FusedK q;
  q.h = h;
  q.hm = h * v.inv_mass;
  q.hIlf = h * v.inv_Iz * v.lf;
  q.hIlr = h * v.inv_Iz * v.lr;
  if (scaled) {
    q.hIlf *= h;
    q.hIlr *= h;
  }
  q.m1 = q.hm * sk.k1;
  q.m0 = q.hm * sk.k0;
  q.m2 = q.hm * sk.k2;
  q.m3 = -(q.hm * sk.k3);
  return q;
}

// SPLIT (LPM = 4 only): the quad's lanes integrate ONE position component each — X on pc =
// 0, Y on pc = 1 — in k[0]/x[0] (k[1]/x[1] unused): the position feeds nothing but the cost,
// so the component's increment, stage sums and tracking term are formed once instead of
// twice in every lane.  X: vx hcos - vy hsin; Y: vx hsin + vy hcos = fma(vx, A, psg vy B).
template <int LPM, bool SPLIT = false>
__device__ __forceinline__ void k_fused(const StageK& sk, const FusedK& q, double F0, double F1,
                                        double hmsd, double hmcd, double c5a, double d, double Bd,
                                        const double* y, double* k, const fm::FmK& K, Dom& dm) {
  const double vx = y[3], vy = y[4], om = y[5];
  constexpr bool kScaled = scaled_yaw(LPM);   // om = W = h omega, y[2] = Psi (make_fused)
  const StageF f = forces_fast<LPM, SPLIT, kScaled, kLeanLA>(sk, vx, vy, om, d, y[2], K, dm, Bd);
  // h sin(psi), h cos(psi): LPM = 4 lanes 2/3 scale their sine by h already (make_stage)
  const double hsp = (LPM == 4) ? f.sp : q.h * f.sp, hcp = (LPM == 4) ? f.cp : q.h * f.cp;
  const double hmFrx = fma(vx, fma(q.m3, vx, F1), F0);                     // hm Frx
  k[2] = kScaled ? om : q.h * om;
  if constexpr (SPLIT) {
    k[0] = fma(vx, hsp, (sk.psg * vy) * hcp);                             // (A, B) in (sp, cp)
    k[1] = 0.0;
  } else {
    k[0] = fma(vx, hcp, -(vy * hsp));                                     // h (vx cos - vy sin)
    k[1] = fma(vx, hsp, vy * hcp);
  }
  k[3] = fma(-f.Ffy, hmsd, fma(vy, k[2], hmFrx));                         // h/m (Frx - Ffy sd) + h vy om
  k[4] = fma(f.Ffy, hmcd, fma(-vx, k[2], q.hm * f.Fry));                  // h/m (Fry + Ffy cd) - h vx om
  k[5] = fma(f.Ffy, c5a, -(f.Fry * q.hIlr));                              // h/Iz (Ffy lf cd - Fry lr)
}

// The step's input terms of the fused stages: they depend on the input and the shared
// constants only, so a staged look-ahead forms them once per (step, candidate) per block.
struct FusedIn {
  double F0, F1, hmsd, hmcd, c5a;
};
__device__ __forceinline__ FusedIn fused_in(const FusedK& q, const Input& u) {
  return FusedIn{fma(q.m1, u.a, -q.m0), -(q.m2 * u.a), q.hm * u.sd, q.hm * u.cd, q.hIlf * u.cd};
}

template <int LPM, bool SPLIT = false>
__device__ __forceinline__ void step_fused(const StageK& sk, const FusedK& q, double* x,
                                           const FusedIn& fi, double ud, const fm::FmK& K,
                                           Dom& dm) {
  static_assert(!SPLIT || LPM == 4, "the position split needs the quad");
  const double F0 = fi.F0, F1 = fi.F1, hmsd = fi.hmsd, hmcd = fi.hmcd, c5a = fi.c5a;
  const Input u{0.0, ud, 0.0, 0.0};                       // k_fused reads u.d only
  const double Bd = (LPM == 4) ? sk.ch[0].B * (u.d * sk.fw) : 0.0;
  double y[6], k[6], acc[6];
  y[1] = acc[1] = 0.0;
  k_fused<LPM, SPLIT>(sk, q, F0, F1, hmsd, hmcd, c5a, u.d, Bd, x, k, K, dm);
  // the quad's yaw is Psi = (2/pi) psi with increment W (make_fused): weights x 2/pi
  constexpr bool kScaled = scaled_yaw(LPM);
  const double c2 = kScaled ? K.inv_pi : 0.5, c4 = kScaled ? K.two_pi : 1.0,
               c6 = kScaled ? K.inv_3pi : K.sixth;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (SPLIT && i == 1) continue;
    acc[i] = k[i];
    y[i] = fma(i == 2 ? c2 : 0.5, k[i], x[i]);
  }
  k_fused<LPM, SPLIT>(sk, q, F0, F1, hmsd, hmcd, c5a, u.d, Bd, y, k, K, dm);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (SPLIT && i == 1) continue;
    acc[i] = fma(2.0, k[i], acc[i]);
    y[i] = fma(i == 2 ? c2 : 0.5, k[i], x[i]);
  }
  k_fused<LPM, SPLIT>(sk, q, F0, F1, hmsd, hmcd, c5a, u.d, Bd, y, k, K, dm);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (SPLIT && i == 1) continue;
    acc[i] = fma(2.0, k[i], acc[i]);
    y[i] = (i == 2 && kScaled) ? fma(c4, k[i], x[i]) : x[i] + k[i];
  }
  k_fused<LPM, SPLIT>(sk, q, F0, F1, hmsd, hmcd, c5a, u.d, Bd, y, k, K, dm);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    if (SPLIT && i == 1) continue;
    x[i] = fma(acc[i] + k[i], i == 2 ? c6 : K.sixth, x[i]);
  }
}

template <int LPM, bool SPLIT = false>
__device__ __forceinline__ void step_fused(const StageK& sk, const FusedK& q, double* x,
                                           const Input& u, const fm::FmK& K, Dom& dm) {
  step_fused<LPM, SPLIT>(sk, q, x, fused_in(q, u), u.d, K, dm);
}

// One look-ahead step on the fast path.
//  RK4 (rk6.py:58-66): four explicit stages with rk4_step's roundings — acc = k, acc + 2k,
//    acc + 2k (FMAs by exact weights), y = x + k/2, x + k/2, x + k, and the final sum divided
//    by 6 through fm::div6 (correctly rounded, = x / 6.0).
//  NLP Euler (nmpc.py:58-60): x + Ts f_nlp(x, u).
//  RK6 (rk6.py:13-28): the general rk6_step, one lane per rollout (LPM must be 1).
template <int INTEG, int LPM>
__device__ __forceinline__ void step_fast(const VehK& v, const Tire& t, const StageK& sk,
                                          double* x, const Input& u, double h,
                                          const fm::FmK& K, Dom& dm) {
  if (INTEG == 0) {
    double y[6], d[6], acc[6];
    rhs_fast<Form::Ref, LPM>(v, sk, x, u, d, K, dm);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double k = h * d[i];
      acc[i] = k;
      y[i] = fma(0.5, k, x[i]);
    }
    rhs_fast<Form::Ref, LPM>(v, sk, y, u, d, K, dm);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double k = h * d[i];
      acc[i] = fma(2.0, k, acc[i]);
      y[i] = fma(0.5, k, x[i]);
    }
    rhs_fast<Form::Ref, LPM>(v, sk, y, u, d, K, dm);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double k = h * d[i];
      acc[i] = fma(2.0, k, acc[i]);
      y[i] = x[i] + k;
    }
    rhs_fast<Form::Ref, LPM>(v, sk, y, u, d, K, dm);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = x[i] + fm::div6(acc[i] + h * d[i], K);
  } else if (INTEG == 1) {
    double d[6];
    rhs_fast<Form::Nlp, LPM>(v, sk, x, u, d, K, dm);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = x[i] + h * d[i];
  } else {
    static_assert(INTEG != 2 || LPM == 1, "RK6 look-ahead runs one lane per rollout");
    rk6_step(v, t, x, u, h);
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

// Branch-free forms of the two orders for per-lane loops on the device (the if/else forms
// above compile to nested divergent branches).
template <int NAN_FIRST, typename I>
__device__ __forceinline__ bool less_bf(double av, I ai, double bv, I bi) {
  const int an = av != av, bn = bv != bv, na = an ^ 1, nb = bn ^ 1;
  const int first = NAN_FIRST ? (an & nb) : (na & bn);
  return first | ((na & nb) & (int)(av < bv)) | (((an & bn) | (int)(av == bv)) & (int)(ai < bi));
}

constexpr int64_t kNoIndex = INT64_MAX;   // sentinel index: sorts after every real key
                                          // (value +inf under NaN-first, NaN under NaN-last)

}  // namespace llampc
