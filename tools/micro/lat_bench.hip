// Diagnostic: fp64 dependent-latency and constant-placement costs on gfx950 (one wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "fastmath.hpp"
using namespace llampc;

__device__ __forceinline__ void pin(double& x) { asm volatile("" : "+v"(x)); }

// atan_q with coefficients held in (opaque) VGPRs
template <bool EST>
__device__ __forceinline__ double atan_qv(double s, const double* c) {
  if (!EST) {
    double p = c[21];
#pragma unroll
    for (int i = 20; i >= 0; --i) p = fma(p, s, c[i]);
    return p;
  }
  const double s2 = s * s, s4 = s2 * s2, s8 = s4 * s4, s16 = s8 * s8;
  const double p0 = fma(c[1], s, c[0]), p1 = fma(c[3], s, c[2]), p2 = fma(c[5], s, c[4]),
               p3 = fma(c[7], s, c[6]), p4 = fma(c[9], s, c[8]), p5 = fma(c[11], s, c[10]),
               p6 = fma(c[13], s, c[12]), p7 = fma(c[15], s, c[14]), p8 = fma(c[17], s, c[16]),
               p9 = fma(c[19], s, c[18]), p10 = fma(c[21], s, c[20]);
  const double q0 = fma(p1, s2, p0), q1 = fma(p3, s2, p2), q2 = fma(p5, s2, p4),
               q3 = fma(p7, s2, p6), q4 = fma(p9, s2, p8);
  const double r0 = fma(q1, s4, q0), r1 = fma(q3, s4, q2), r2 = fma(p10, s4, q4);
  return fma(r2, s16, fma(r1, s8, r0));
}

__device__ __forceinline__ double div_nochk(double num, double den) {
  double r = __builtin_amdgcn_rcp(den);
  double e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  const double q = num * r;
  return fma(r, fma(-den, q, num), q);
}
// one Newton step then residual correction
__device__ __forceinline__ double div_1n(double num, double den) {
  double r = __builtin_amdgcn_rcp(den);
  double e = fma(-den, r, 1.0);
  r = fma(r, e, r);
  const double q = num * r;
  return fma(r, fma(-den, q, num), q);
}

template <int OP, int ILP>
__global__ void chain(const double* in, double* out, long long* cyc, int iters) {
  double v[ILP];
  for (int i = 0; i < ILP; ++i) v[i] = in[threadIdx.x] + 0.01 * i;
  double c[22];
  for (int i = 0; i < 22; ++i) { c[i] = fm::kAtanQ[i]; pin(c[i]); }
  double k1 = 0.999, k2 = 0.001;
  pin(k1); pin(k2);
  __syncthreads();
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      double x = v[i];
      if (OP == 0) { for (int j = 0; j < 16; ++j) x = fma(x, k1, k2); }            // 16 dep fma, vgpr const
      if (OP == 1) { for (int j = 0; j < 16; ++j) x = fma(x, 0.999 + j * 1e-9, 0.001 + j * 1e-9); }  // sgpr consts
      if (OP == 2) { for (int j = 0; j < 16; ++j) x = x * k1; }                     // 16 dep mul
      if (OP == 3) { for (int j = 0; j < 16; ++j) x = x + k2; }                     // 16 dep add
      if (OP == 4) x = atan_qv<false>(x * 0.5, c);
      if (OP == 5) x = atan_qv<true>(x * 0.5, c);
      if (OP == 6) x = fm::atan_q<false>(x * 0.5);
      if (OP == 7) x = fm::atan_q<true>(x * 0.5);
      if (OP == 8) x = div_nochk(x, 1.5 + x * k2);
      if (OP == 9) x = div_1n(x, 1.5 + x * k2);
      if (OP == 10) x = x / (1.5 + x * k2);
      if (OP == 11) x = 1.0 + __builtin_amdgcn_rcp(x);
      if (OP == 12) { for (int j = 0; j < 16; ++j) x = (x > k2) ? x * k1 : x + k2; }  // 16 cmp+cndmask+op
      if (OP == 13) x = rint(x * k1) + k2;
      if (OP == 20) {                                  // 64 dependent fp64 FMAs
#pragma unroll
        for (int j = 0; j < 64; ++j) x = fma(x, k1, c[j % 22]);
      }
      if (OP == 21) {                                  // 8 independent chains x 8 FMAs
        double y[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) y[q] = x + q;
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int q = 0; q < 8; ++q) y[q] = fma(y[q], k1, c[(j + q) % 22]);
        x = ((y[0] + y[1]) + (y[2] + y[3])) + ((y[4] + y[5]) + (y[6] + y[7]));
      }
      if (OP == 22) {                                  // 2 independent chains x 32 FMAs
        double y0 = x, y1 = x + 1;
#pragma unroll
        for (int j = 0; j < 32; ++j) { y0 = fma(y0, k1, c[j % 22]); y1 = fma(y1, k1, c[(j + 5) % 22]); }
        x = y0 + y1;
      }
      v[i] = x;
    }
  }
  long long t1 = clock64();
  double acc = 0;
  for (int i = 0; i < ILP; ++i) acc += v[i];
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP, int ILP>
void run(const char* name, double* din, double* dout, long long* dcyc, double div) {
  const int iters = 200;
  hipLaunchKernelGGL((chain<OP, ILP>), dim3(1), dim3(64), 0, 0, din, dout, dcyc, iters);
  hipLaunchKernelGGL((chain<OP, ILP>), dim3(1), dim3(64), 0, 0, din, dout, dcyc, iters);
  long long c = 0;
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  printf("%-34s ILP=%d  %8.1f cycles\n", name, ILP, (double)c / iters / ILP / div);
}

int main() {
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, 64 * 8); hipMalloc(&dout, 64 * 8); hipMalloc(&dcyc, 8);
  double h[64];
  for (int i = 0; i < 64; ++i) h[i] = 0.1 + 0.01 * i;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
#define R(op, name, d) run<op, 1>(name, din, dout, dcyc, d); run<op, 4>(name, din, dout, dcyc, d);
  R(0, "dep fma (vgpr const) per op", 16)
  R(1, "dep fma (sgpr consts) per op", 16)
  R(2, "dep mul per op", 16)
  R(3, "dep add per op", 16)
  R(12, "cmp+cndmask+op per op", 16)
  R(4, "atan_q Horner vgpr", 1)
  R(5, "atan_q Estrin vgpr", 1)
  R(6, "atan_q Horner sgpr", 1)
  R(7, "atan_q Estrin sgpr", 1)
  R(8, "div rcp+2N no check", 1)
  R(9, "div rcp+1N no check", 1)
  R(10, "div IEEE", 1)
  R(11, "rcp only", 1)
  R(13, "rint", 1)
  run<20, 1>("64 dep fma (per fma)", din, dout, dcyc, 64);
  run<21, 1>("8x8 indep fma (per fma)", din, dout, dcyc, 71);
  run<22, 1>("2x32 fma (per fma)", din, dout, dcyc, 65);
  return 0;
}
