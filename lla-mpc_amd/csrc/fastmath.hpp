// fastmath.hpp — lean fp64 atan2 / atan / sin / sincos for the rollout kernels.
//
// Why: the rollout is VALU-issue-bound (rocprofv3 PMC: SQ_ACTIVE_INST_VALU ~ 1 quad-cycle
// per fp64 instruction, SQ_WAIT_INST_ANY ~3% of wave cycles), so what costs is the NUMBER of
// instructions per transcendental chain atan2 -> atan -> sin.  The same accuracy
// class (<= 1 ulp for each polynomial core, measured in tools/fit_fastmath.py; <= 4 ulp end
// to end, tested against libm) comes with fewer instructions: an atan2 specialised to
// x >= 0, which is all the model needs (the reference form uses |vx|, dynamic.py:149-150;
// the NLP form clamps vx >= vmin, dynamic.py:208-216), and no inlined Payne-Hanek path
// except behind a branch for |a| > 2^20 pi/2.
//
// Evaluation: Horner (the kernels are issue-bound, see atan_q), a reciprocal-Newton
// division, and a wave-uniform small-argument path for sin.
// Coefficients: Chebyshev fits in 60-digit mpmath (tools/fit_fastmath.py):
//   atan(t) = t + t*s*QA(s),          s = t^2, |t| <= 1      (QA: 22 terms)
//   sin(r)  = r + r*s*QS(s),          s = r^2, |r| <= pi/4   (QS: 7 terms)
//   cos(r)  = 1 - s/2 + s^2*QC(s)                            (QC: 7 terms)
// with a 3-part Cody-Waite reduction by pi/2 for |a| <= 2^20 (ocml beyond, or non-finite).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace llampc {
namespace fm {

constexpr double kAtanQ[22] = {
    -0.3333333333333333,     0.1999999999999992,     -0.14285714285701234,
    0.11111111110268297,     -0.0909090906193528,    0.07692307078827029,
    -0.06666657934573768,    0.05882264416776449,    -0.052624922290256754,
    0.04758080083637821,     -0.043306538430670664,  0.03938687540798632,
    -0.035271331066871296,   0.030330719265790507,   -0.024191345810140718,
    0.01718398172211335,     -0.010412153260359241,  0.005140912856746939,
    -0.0019612554271685326,  0.0005376839297396244,  -9.371186345052626e-05,
    7.767624330289919e-06};
constexpr double kSinQ[7] = {-0.16666666666666666,    0.008333333333333331,
                             -0.00019841269841265065, 2.7557319219339167e-06,
                             -2.5052106232447578e-08, 1.6058531618986147e-10,
                             -7.586697117706918e-13};
constexpr double kCosQ[7] = {0.041666666666666664,   -0.0013888888888888887,
                             2.4801587301584645e-05, -2.7557319221402824e-07,
                             2.087675579108042e-09,  -1.1470460887609959e-11,
                             4.7458719020432915e-14};
constexpr double kPio2Hi = 1.570796325802803, kPio2Mid = 9.920935184482005e-10,
                 kPio2Lo = 6.123233995736766e-17;
constexpr double kTwoOverPi = 0.6366197723675814, kPio2 = 1.5707963267948966,
                 kPio4 = 0.7853981633974483;
constexpr double kPio2Tail = 6.123233995736766e-17;   // pi/2 - (double)(pi/2)
constexpr double kSinCosMax = 1647099.3291652855;      // 2^20 * pi/2

// Horner evaluation throughout: the kernels are issue-bound (Estrin's
// shorter dependency chains cost more instructions and measured slower).
__device__ __host__ __forceinline__ double atan_q(double s) {
  const double* c = kAtanQ;
  double p = c[21];
#pragma unroll
  for (int i = 20; i >= 0; --i) p = fma(p, s, c[i]);
  return p;
}

// atan(t) for |t| <= 1.
__device__ __host__ __forceinline__ double atan_core(double t) {
  const double s = t * t;
  return fma(t * s, atan_q(s), t);
}

// num / den by reciprocal + two Newton steps + one residual correction (8 VALU instead of
// the 11 of the scaled IEEE sequence); exact-division fallback, wave-uniform, when some
// |den| is outside [2^-1000, 2^1000] or not finite.
__device__ __host__ __forceinline__ double div_(double num, double den) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double ad = fabs(den);
  if (__any(!(ad >= 0x1p-1000 && ad <= 0x1p1000))) return num / den;
  double r = __builtin_amdgcn_rcp(den);
  double e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  const double q = num * r;
  return fma(r, fma(-den, q, num), q);
#else
  return num / den;
#endif
}

// atan2(y, x) for x >= +0 (or NaN): one division, no quadrant branches.  Special cases
// follow C99 atan2 for x >= 0: (+-0, +0) -> +-0, (+-inf, +inf) -> +-pi/4.
__device__ __host__ __forceinline__ double atan2_xpos(double y, double x) {
  const bool swap = fabs(y) > x;
  const double num = swap ? x : y, den = swap ? y : x;
  const double r = atan_core(div_(num, den));
  double out = swap ? (copysign(kPio2, y) - r) + copysign(kPio2Tail, y) : r;
  if (x == 0.0 && y == 0.0) out = y;
  if (isinf(x) && isinf(y)) out = copysign(kPio4, y);
  return out;
}

// atan(z): the division only when some |z| > 1.
__device__ __host__ __forceinline__ double atan_(double z) {
  const bool swap = fabs(z) > 1.0;
  double t = z;
  if (swap) t = 1.0 / z;
  const double r = atan_core(t);
  return swap ? (copysign(kPio2, z) - r) + copysign(kPio2Tail, z) : r;
}

__device__ __host__ __forceinline__ double poly7(const double* a, double s1) {
  double p = a[6];
#pragma unroll
  for (int i = 5; i >= 0; --i) p = fma(p, s1, a[i]);
  return p;
}

__device__ __host__ __forceinline__ double sin_poly(double r, double s1) {
  return fma(r * s1, poly7(kSinQ, s1), r);
}

__device__ __host__ __forceinline__ double cos_poly(double s1) {
  return fma(s1 * s1, poly7(kCosQ, s1), fma(-0.5, s1, 1.0));
}

__device__ __host__ __forceinline__ void sincos_core(double r, double* s, double* c) {
  const double s1 = r * r;
  *s = sin_poly(r, s1);
  *c = cos_poly(s1);
}

__device__ __host__ __forceinline__ void sincos_(double a, double* s, double* c) {
  if (!(fabs(a) <= kSinCosMax)) {       // huge or non-finite: ocml (Payne-Hanek)
    sincos(a, s, c);
    return;
  }
  const double k = rint(a * kTwoOverPi);
  double r = fma(-k, kPio2Hi, a);
  r = fma(-k, kPio2Mid, r);
  r = fma(-k, kPio2Lo, r);
  const int q = (int)k & 3;
  double sr, cr;
  sincos_core(r, &sr, &cr);
  double so = (q & 1) ? cr : sr, co = (q & 1) ? sr : cr;
  so = (q & 2) ? -so : so;
  co = ((q + 1) & 2) ? -co : co;
  *s = so;
  *c = co;
}

// sin(a): wave-uniform fast path when every |a| <= pi/4 (no reduction, one polynomial) —
// the common case for the tire argument C*atan(B*alpha) at moderate slip.
__device__ __host__ __forceinline__ double sin_(double a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (__all(fabs(a) <= kPio4)) return sin_poly(a, a * a);
#endif
  double s, c;
  sincos_(a, &s, &c);
  return s;
}

// ------------------------------------------------------------------------------------
// Branch-free cores for the rollout stage (dyn.hpp rhs_fast).
//
// Measured on gfx950 with ONE wave per SIMD (the regime of a tick at N*C ~ 1e4):
// a dependent fp64 FMA costs ~6 cycles, but a compare+select ~25, a wave-uniform branch
// ~70, v_rcp_f64 / v_rndne_f64 ~40 (tools/micro/lat_bench.hip).  So these cores carry no
// branches and as few selects as possible, and are valid only on a stated domain; the
// caller evaluates the domain predicate (the *_ok helpers, off the critical path) and
// re-does the rare out-of-domain lanes with the general functions above, behind ONE
// wave-uniform branch per stage that is normally not taken.
// ------------------------------------------------------------------------------------
constexpr double kSinWQ[10] = {
    -0.16666666666666666,  0.008333333333333328,  -0.00019841269841267895,
    2.7557319223709e-06,  -2.505210836542107e-08,  1.6059043004898195e-10,
    -7.647142668717314e-13,  2.8111267068839815e-15,  -8.18919565437741e-18,
    1.790528073907954e-20};
// atan(t) = t + t*s*QR(s) for |t| <= tan(pi/8) (10 terms: fit error 1.5e-16 relative, <= 1 ulp): the fast cores reduce their
// ratio r in [0, 1] by atan(r) = pi/4 + atan((r - 1)/(r + 1)) when r > tan(pi/8), so the
// polynomial is half as long as QA's on [0, 1] for 6 more instructions
// (tools/fit_fastmath.py).
constexpr double kAtanR[10] = {
    -0.3333333333333325,  0.19999999999898407,  -0.1428571426609662,
    0.11111109636534361,  -0.09090852557176049,  0.0769105515839315,
    -0.06649613695291669,  0.05736332165907643,  -0.04483334622272886,
    0.02275052699336167};
constexpr double kTanPi8 = 0.41421356237309503;
// Lean cores of the look-ahead rollouts (kLeanLA): 8-term atan (1.1e-13 relative on |t| <=
// tan(pi/8)) and 8-term sin_wide (2.6e-13 absolute to |a| = 3), and the division without its
// residual correction (<= 18 ulp), against the <= 4 ulp of the precise cores, which the
// look-back keeps (its errors are ranked).  Round 3 shipped 9 terms, round 4 went to 8 and then
// 7 (-12 / -32 instructions per LPM-4 / LPM-1 step, 26.3 -> 26.0 us per tick).  Round 5 measured
// the cost of that on ill-conditioned rollouts (tools/diag/accuracy_headroom.py,
// profiles/r05/accuracy_lean.txt): on config 3's own Mobil scenario states, where a ONE-ulp
// change of x0 moves a cost by 1.5e-8 relative in NumPy itself, the 7-term cores
// were 9.3e-5 off (6,400 ulp-equivalents: past the north star's 1e-5), 8 terms 6.8e-7 (47),
// 9 terms 1.6e-8 (1.1); every well-conditioned shape stays within 1e-10 with 8 terms.  So 8
// terms again (+0.2-0.4 us per tick at C = 1, +2 % at C = 64).
// -DLLAMPC_LEAN_TERMS=7 / 9 build the other cores (tools/fit_fastmath.py fits them).
#ifndef LLAMPC_LEAN_TERMS
#define LLAMPC_LEAN_TERMS 8
#endif
constexpr int kLeanTerms = LLAMPC_LEAN_TERMS;
#if LLAMPC_LEAN_TERMS == 7
constexpr double kAtanRL[7] = {-0.3333333333144073, 0.1999999891728858, -0.14285612511387016,
                               0.11107495135714474, -0.09028983500350463, 0.07135325122330678,
                               -0.04043224825887161};
constexpr double kSinWQL[7] = {-0.1666666666651697, 0.008333333317028357, -0.00019841266938549256,
                               2.755712516942648e-06, -2.5045917650344973e-08, 1.5957259420467993e-10,
                               -6.809345001958508e-13};
#elif LLAMPC_LEAN_TERMS == 8
constexpr double kAtanRL[8] = {-0.33333333333266196, 0.19999999949854794, -0.142857081103604,
                               0.11110819716745676, -0.09084101895346429, 0.07604800046078292,
                               -0.06027307460946675, 0.03295679541870136};
constexpr double kSinWQL[8] = {-0.16666666666665675, 0.008333333333192344, -0.0001984126980834366,
                               2.7557316292288437e-06, -2.5051980053729585e-08, 1.6055987705856629e-10,
                               -7.606702398667312e-13, 2.530093775325291e-15};
#else
constexpr double kAtanRL[9] = {-0.3333333333333093, 0.19999999997724888, -0.14285713930378566,
                               0.11111089649211055, -0.09090255952690657, 0.07681045202742948,
                               -0.0655090730756309, 0.05168834935919362, -0.02723288406057488};
constexpr double kSinWQL[9] = {-0.1666666666666666, 0.008333333333332372, -0.00019841269840984845,
                               2.755731919144023e-06, -2.5052106522437073e-08, 1.605898387304835e-10,
                               -7.646028139181475e-13, 2.7988830742041364e-15, -7.463851483197331e-18};
#endif
constexpr double kSinWideMax = 3.0;   // sin(a) = a + a*s*QW(s) (10 terms, fit error 6e-18), |a| <= 3:
                                       // <= 3 ulp up to |a| = 2, then <= 2^-50 absolute (cancellation)

// Constants of the fast cores, held in VGPRs for the whole kernel (FmK::load pins them
// with an empty asm so the compiler cannot rematerialise them): a VOP3 v_fma_f64 reads a
// VGPR constant for free, while a rematerialised 64-bit constant costs two v_mov/s_mov
// issue slots per use — 2.5x on a Horner chain in the one-wave-per-SIMD regime.
struct FmK {
  double ar[10];
  double tp8, pio4;
  double sw[10], sq[7], cq[7];
  double pio2, two_pi, cw0, cw1, cw2, sixth, six, rmagic, rmagic2, one;
  double inv_pi, inv_3pi;                 // (2/pi)/2, (2/pi)/6: the scaled yaw's RK4 weights

  __device__ __forceinline__ static void pin(double& x) { asm volatile("" : "+v"(x)); }
  // LEAN: the kLeanTerms-term coefficient sets in ar / sw (the lean cores read no more)
  template <bool LEAN = false>
  __device__ __forceinline__ static FmK load() {
    FmK k;
    constexpr int nA = LEAN ? kLeanTerms : 10;
#pragma unroll
    for (int i = 0; i < nA; ++i) { k.ar[i] = LEAN ? kAtanRL[i] : kAtanR[i]; pin(k.ar[i]); }
    k.tp8 = kTanPi8;
    k.pio4 = kPio4;
    pin(k.tp8);
    pin(k.pio4);
#pragma unroll
    for (int i = 0; i < nA; ++i) { k.sw[i] = LEAN ? kSinWQL[i] : kSinWQ[i]; pin(k.sw[i]); }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      k.sq[i] = kSinQ[i];
      k.cq[i] = kCosQ[i];
      pin(k.sq[i]);
      pin(k.cq[i]);
    }
    k.pio2 = kPio2;
    k.two_pi = kTwoOverPi;
    k.cw0 = kPio2Hi;
    k.cw1 = kPio2Mid;
    k.cw2 = kPio2Lo;
    k.sixth = 1.0 / 6.0;
    k.six = 6.0;
    k.rmagic = 0x1.8p52;
    k.rmagic2 = 0x1.8p53;
    k.one = 1.0;
    pin(k.pio2); pin(k.two_pi); pin(k.cw0); pin(k.cw1); pin(k.cw2);
    pin(k.sixth); pin(k.six); pin(k.rmagic); pin(k.rmagic2); pin(k.one);
    k.inv_pi = kTwoOverPi * 0.5;
    k.inv_3pi = kTwoOverPi / 6.0;
    pin(k.inv_pi); pin(k.inv_3pi);
    return k;
  }
};

template <int N>
__device__ __forceinline__ double horner(const double* c, double s) {
  double p = c[N - 1];
#pragma unroll
  for (int i = N - 2; i >= 0; --i) p = fma(p, s, c[i]);
  return p;
}

// num / den, den in [2^-1001, 2^1000]: reciprocal + one Newton step + residual.  With the
// reciprocal's relative error e0, r has e0^2 and the corrected quotient e0^4 + 1/2 ulp:
// one step is enough for any e0 <= 2^-14 (v_rcp_f64 is far better; the atan2/atan ULP
// tests, whose every call divides, bound the result).
template <bool LEAN = false>
__device__ __forceinline__ double div_fast(double num, double den) {
  double r = __builtin_amdgcn_rcp(den);
  const double e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  if constexpr (LEAN) return num * r;         // lean cores: no residual step (<= 18 ulp)
  // the residual correction is needed: without it atan2 reaches 18 ulp for divisors just
  // below powers of two (v_rcp_f64 is least accurate there; tools/diag/ulp_probe.py)
  const double q = num * r;
  return fma(r, fma(-den, q, num), q);
}

// v / 6 correctly rounded (Markstein: q = RN(v/6 approx), exact residual, one correction;
// checked bit-exact against v / 6.0 in tests/test_host_cpu.py::test_div6_correctly_rounded).
__device__ __host__ __forceinline__ double div6(double v) {
  const double y = 1.0 / 6.0;
  const double q = v * y;
  return fma(fma(-6.0, q, v), y, q);
}
__device__ __forceinline__ double div6(double v, const FmK& K) {
  const double q = v * K.sixth;
  return fma(fma(-K.six, q, v), K.sixth, q);
}

// IEEE maxNum / minNum as ONE instruction.  fmax/fmin compile to v_max_f64/v_min_f64 plus a
// canonicalising v_max_f64 x, x of every operand the compiler cannot prove canonical (loop-
// carried values, fabs results): 5 extra instructions per rollout stage.  The operands here
// are arithmetic results, never signalling NaNs, so the raw instruction has fmax's meaning
// (a NaN operand yields the other one).  |a| by the source modifier.
__device__ __forceinline__ double vmax(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmax_abs(double a, double b) {   // max(|a|, b)
  double r;
  asm("v_max_f64 %0, |%1|, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmin_abs(double a, double b) {   // min(|a|, b)
  double r;
  asm("v_min_f64 %0, |%1|, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmax_abs2(double a, double b) {  // max(|a|, |b|)
  double r;
  asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double vmin_abs2(double a, double b) {  // min(|a|, |b|)
  double r;
  asm("v_min_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// atan(n / d) for 0 <= n <= d, d in [2^-1001, 2^1000].  Reduced form: s = n > tan(pi/8) d
// selects t = (n - d)/(n + d) and the offset pi/4 (sf = 1.0 or 0.0: the select is the high
// word only), so the polynomial covers |t| <= tan(pi/8).  n - d and n + d are rounded once
// each (relative 2^-53 on t); the offset add rounds once: <= 2 ulp before the callers'
// fix-ups (tests: test_fast_cores_ulp_on_domain).
template <bool LEAN = false>
__device__ __forceinline__ double atan_ratio_k(double n, double d, const FmK& K) {
  const bool red = n > K.tp8 * d;
  const double sf = __hiloint2double(red ? 0x3FF00000 : 0, 0);
  const double t = div_fast<LEAN>(fma(-sf, d, n), fma(sf, n, d));
  const double s = t * t;
  return fma(sf, K.pio4, fma(t * s, horner<LEAN ? kLeanTerms : 10>(K.ar, s), t));
}

// atan2(y, x) for x >= 0 on the domain atan2_fast_ok(y, x): the sum |y| + x in
// [2^-1000, 2^1000] (so max(|y|, x) is a safe divisor; NaN -> not ok).
__device__ __host__ __forceinline__ bool atan2_fast_ok(double y, double x) {
  const double s = fabs(y) + x;
  return s >= 0x1p-1000 && s <= 0x1p1000;
}
// hi = max(|y|, |x|), the divisor: hi in [2^-1000, 2^999] lies inside the domain (the
// rollout checks its running extremes once, dyn.hpp Dom).  x enters as |x| (the callers'
// x is |vx| or the clamped vx >= vmin, so passing vx itself saves materialising |vx|).
template <bool LEAN = false>
__device__ __forceinline__ double atan2_fast(double y, double x, const FmK& K, double& hi) {
  const double ay = fabs(y);
  hi = vmax_abs2(y, x);
  const double r = atan_ratio_k<LEAN>(vmin_abs2(y, x), hi, K);
  const double o = (ay > fabs(x)) ? K.pio2 - r : r;   // no pi/2 tail: <= 2 ulp (measured)
  return copysign(o, y);
}
template <bool LEAN = false>
__device__ __forceinline__ double atan2_fast(double y, double x, const FmK& K) {
  double hi;
  return atan2_fast<LEAN>(y, x, K, hi);
}

// atan(z) on the domain |z| <= 2^1000: the reciprocal branch as a division by max(|z|, 1)
// (exact when |z| <= 1).
__device__ __host__ __forceinline__ bool atan_fast_ok(double z) { return fabs(z) <= 0x1p1000; }
// hz = max(|z|, 1), the divisor: hz <= 2^1000 is the domain.
template <bool LEAN = false>
__device__ __forceinline__ double atan_fast(double z, const FmK& K, double& hz) {
  const double az = fabs(z);
  hz = vmax_abs(z, K.one);
  const double r = atan_ratio_k<LEAN>(vmin_abs(z, K.one), hz, K);
  const double o = (az > 1.0) ? K.pio2 - r : r;   // no pi/2 tail: <= 2 ulp (measured)
  return copysign(o, z);
}
template <bool LEAN = false>
__device__ __forceinline__ double atan_fast(double z, const FmK& K) {
  double hz;
  return atan_fast<LEAN>(z, K, hz);
}

// Two independent reduced-ratio atans with ONE reciprocal (the LPM-1 lane's front and rear
// chains, lean cores only): 1/den_f = den_r / (den_f den_r) and 1/den_r = den_f / (den_f
// den_r), the product's reciprocal with one Newton step.  v_rcp_f64 issues for 16 cycles
// against 4 for an FMA, so the pair costs 44 VALU cycles instead of 56.  Valid while both
// divisors lie in [2^-500, 2^500] (the product then stays a normal number): the callers'
// domain record (dyn.hpp Dom::ok_paired) checks that.  dprod = the product, for that record.
__device__ __forceinline__ void atan_ratio_pair(double nf, double df, double nr, double dr,
                                                const FmK& K, double& of, double& orr,
                                                double& dprod) {
  const bool redf = nf > K.tp8 * df, redr = nr > K.tp8 * dr;
  const double sff = __hiloint2double(redf ? 0x3FF00000 : 0, 0);
  const double sfr = __hiloint2double(redr ? 0x3FF00000 : 0, 0);
  const double denf = fma(sff, nf, df), denr = fma(sfr, nr, dr);
  const double D = denf * denr;
  double r = __builtin_amdgcn_rcp(D);
  const double e = fma(-D, r, 1.0);
  r = fma(r, e, r);
  const double tf = fma(-sff, df, nf) * (denr * r);
  const double tr = fma(-sfr, dr, nr) * (denf * r);
  const double sf2 = tf * tf, sr2 = tr * tr;
  of = fma(sff, K.pio4, fma(tf * sf2, horner<kLeanTerms>(K.ar, sf2), tf));
  orr = fma(sfr, K.pio4, fma(tr * sr2, horner<kLeanTerms>(K.ar, sr2), tr));
  dprod = D;
}

// atan2(y_f, x) and atan2(y_r, x) (x >= 0) by atan_ratio_pair; hf / hr = the divisors
// max(|y|, |x|) for the domain record, dprod the reciprocal's product.
__device__ __forceinline__ void atan2_fast_pair(double yf, double yr, double x, const FmK& K,
                                                double& af, double& ar, double& hf, double& hr,
                                                double& dprod) {
  hf = vmax_abs2(yf, x);
  hr = vmax_abs2(yr, x);
  double rf, rr;
  atan_ratio_pair(vmin_abs2(yf, x), hf, vmin_abs2(yr, x), hr, K, rf, rr, dprod);
  const double of = (fabs(yf) > fabs(x)) ? K.pio2 - rf : rf;
  const double orr = (fabs(yr) > fabs(x)) ? K.pio2 - rr : rr;
  af = copysign(of, yf);
  ar = copysign(orr, yr);
}

// atan(z_f) and atan(z_r) by atan_ratio_pair; dprod = the product of the divisors
// max(|z|, 1) (+ the reduction's share), >= 1: the domain record bounds it from above.
__device__ __forceinline__ void atan_fast_pair(double zf, double zr, const FmK& K, double& af,
                                               double& ar, double& dprod) {
  double rf, rr;
  atan_ratio_pair(vmin_abs(zf, K.one), vmax_abs(zf, K.one), vmin_abs(zr, K.one),
                  vmax_abs(zr, K.one), K, rf, rr, dprod);
  const double of = (fabs(zf) > 1.0) ? K.pio2 - rf : rf;
  const double orr = (fabs(zr) > 1.0) ? K.pio2 - rr : rr;
  af = copysign(of, zf);
  ar = copysign(orr, zr);
}

// sin(a) for |a| <= kSinWideMax, one polynomial (the Pacejka argument C*atan(.) is
// bounded by |C| pi/2, so |C| <= 1.9 keeps every call in range).
template <bool LEAN = false>
__device__ __forceinline__ double sin_wide(double a, const FmK& K) {
  const double s = a * a;
  return fma(a * s, horner<LEAN ? kLeanTerms : 10>(K.sw, s), a);
}

// sincos(a) for |a| <= kSinCosMax (NaN/inf -> not ok): Cody-Waite reduction, quadrant
// fix-up with integer sign flips.
__device__ __host__ __forceinline__ bool sincos_fast_ok(double a) { return fabs(a) <= kSinCosMax; }
__device__ __forceinline__ void sincos_fast(double a, double* s, double* c, const FmK& K) {
  // k = round(a 2/pi) by adding 1.5*2^52 (|a 2/pi| < 2^51 on the domain): the integer lands
  // in the mantissa's low bits, so the quadrant is the low word — no v_rndne / v_cvt
  const double t = fma(a, K.two_pi, K.rmagic);
  const double k = t - K.rmagic;
  double r = fma(-k, K.cw0, a);
  r = fma(-k, K.cw1, r);
  r = fma(-k, K.cw2, r);
  const int q = __double2loint(t);
  const double s1 = r * r;
  const double sr = fma(r * s1, horner<7>(K.sq, s1), r);
  const double cr = fma(s1 * s1, horner<7>(K.cq, s1), fma(-0.5, s1, 1.0));
  const bool odd = q & 1;
  const double so = odd ? cr : sr, co = odd ? sr : cr;
  const int fs = (q & 2) << 30, fc = ((q + 1) & 2) << 30;
  *s = __hiloint2double(__double2hiint(so) ^ fs, __double2loint(so));
  *c = __hiloint2double(__double2hiint(co) ^ fc, __double2loint(co));
}

}  // namespace fm
}  // namespace llampc
