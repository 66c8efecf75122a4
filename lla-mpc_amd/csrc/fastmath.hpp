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

// The kernels are VALU-issue-bound (rocprofv3: ~1 fp64 instruction per 4 cycles, few
// dependency stalls), so the cores use Horner (one SGPR constant per v_fmac, no moves)
// rather than Estrin.
__device__ __host__ __forceinline__ double atan_q(double s) {
  double p = kAtanQ[21];
#pragma unroll
  for (int i = 20; i >= 0; --i) p = fma(p, s, kAtanQ[i]);
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

__device__ __host__ __forceinline__ double sin_poly(double r, double s1) {
  double p = kSinQ[6];
#pragma unroll
  for (int i = 5; i >= 0; --i) p = fma(p, s1, kSinQ[i]);
  return fma(r * s1, p, r);
}

__device__ __host__ __forceinline__ double cos_poly(double s1) {
  double p = kCosQ[6];
#pragma unroll
  for (int i = 5; i >= 0; --i) p = fma(p, s1, kCosQ[i]);
  return fma(s1 * s1, p, fma(-0.5, s1, 1.0));
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

}  // namespace fm
}  // namespace llampc
