// Diagnostic microbenchmark (not product): cycles per call of the model's building blocks
// as a dependent chain in ONE wave (the latency regime of the tick), and with 4 independent
// chains per lane (ILP).  s_memtime around the loop.  Build: see tools/micro/build.sh
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dyn.hpp"

using namespace llampc;

template <int OP, int ILP>
__global__ void chain(const double* in, double* out, long long* cyc, int iters, const double* prm) {
  double v[ILP];
  for (int i = 0; i < ILP; ++i) v[i] = in[threadIdx.x] + 0.01 * i;
  VehK vk{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], prm[8], 0, 0};
  Tire t{prm[9 + (threadIdx.x & 7)], prm[18], prm[19], prm[20], prm[21], prm[22]};
  const fm::FmK K = fm::FmK::load();
  __syncthreads();
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) {
      double x = v[i];
      if (OP == 0) x = fm::atan2_xpos<false>(x * 0.3, 1.0 + x * x);
      if (OP == 1) x = fm::atan2_xpos<true>(x * 0.3, 1.0 + x * x);
      if (OP == 2) x = fm::atan_<false>(x * 0.7);
      if (OP == 3) x = fm::atan_<true>(x * 0.7);
      if (OP == 4) x = fm::sin_<false>(x * 0.5) + 0.3;
      if (OP == 5) { double s, c; fm::sincos_<false>(x * 3.0, &s, &c); x = s + c * 0.1; }
      if (OP == 6) x = fm::div_(x, 1.5 + x * x);
      if (OP == 7) x = x / (1.5 + x * x);
      if (OP == 8) x = atan2(x * 0.3, 1.0 + x * x);                 // ocml
      if (OP == 9) x = atan(x * 0.7);                               // ocml
      if (OP == 10) x = sin(x * 0.5) + 0.3;                         // ocml
      if (OP == 11) x = fma(x, 0.999, 0.001);                       // one dependent fma
      if (OP == 13) {                                               // one full rhs (LPM=1)
        double xs[6] = {x, 0.2, 0.3 + x * 0.01, 1.5, 0.05, 0.3}, d[6];
        const Input u = make_input(0.5, 0.05);
        rhs<Form::Ref>(vk, t, xs, u, d);
        x = x + 1e-3 * (d[0] + d[3] + d[5] * 1e-3);
      }
      if (OP == 15) {                                               // full RK4 step, LPM=4
        double xs[6] = {x, 0.2, 0.3 + x * 0.01, 1.5, 0.05, 0.3};
        bool bad = false; const Input u = make_input_fast(0.5, 0.05 + 1e-3 * x, K, bad);
        const StageK sk = make_stage<2>(vk, t, threadIdx.x & 1);
        step_fast<0, 2>(vk, t, sk, xs, u, 0.02, K, bad);
        x = xs[0] * 0.5 + xs[3] * 1e-3;
      }
      if (OP == 16) {                                               // full RK4 step, LPM=1
        double xs[6] = {x, 0.2, 0.3 + x * 0.01, 1.5, 0.05, 0.3};
        bool bad = false; const Input u = make_input_fast(0.5, 0.05 + 1e-3 * x, K, bad);
        const StageK sk = make_stage<1>(vk, t, 0);
        step_fast<0, 1>(vk, t, sk, xs, u, 0.02, K, bad);
        x = xs[0] * 0.5 + xs[3] * 1e-3;
      }
      if (OP == 17) x = fm::atan2_fast(x * 0.3, 1.0 + x * x, K);
      if (OP == 18) x = fm::atan_fast(x * 0.7, K);
      if (OP == 19) x = fm::sin_wide(x * 0.5, K) + 0.3;
      if (OP == 20) { double s, c; fm::sincos_fast(x * 3.0, &s, &c, K); x = s + c * 0.1; }
      if (OP == 21) x = fm::div6(x, K) + 0.9;
      if (OP == 14) {                                               // dpp exchange only
        x = dpp_bcast<kPair1>(x) * 0.999 + 0.001;
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
void run(const char* name, double* din, double* dout, long long* dcyc, const double* prm) {
  const int iters = 200;
  hipLaunchKernelGGL((chain<OP, ILP>), dim3(1), dim3(64), 0, 0, din, dout, dcyc, iters, prm);
  hipLaunchKernelGGL((chain<OP, ILP>), dim3(1), dim3(64), 0, 0, din, dout, dcyc, iters, prm);
  long long c = 0;
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  printf("%-26s ILP=%d  %8.1f cycles/call (per chain element)\n", name, ILP, (double)c / iters / ILP);
}

int main() {
  double *din, *dout;
  long long* dcyc;
  hipMalloc(&din, 64 * 8);
  hipMalloc(&dout, 64 * 8);
  hipMalloc(&dcyc, 8);
  double h[64];
  for (int i = 0; i < 64; ++i) h[i] = 0.1 + 0.01 * i;
  hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  double hp[32] = {0.029, 0.033, 0.041, 1 / 0.041, 1 / 27.8e-6, 0.287, 0.0545, 0.0518, 0.00035,
                   2.579, 2.58, 2.57, 2.6, 2.55, 2.59, 2.579, 2.5, 0,
                   1.2, 0.192, 3.3852, 1.2691, 0.1737};
  double* prm;
  hipMalloc(&prm, sizeof hp);
  hipMemcpy(prm, hp, sizeof hp, hipMemcpyHostToDevice);
#define R(op, name) run<op, 1>(name, din, dout, dcyc, prm); run<op, 4>(name, din, dout, dcyc, prm);
  R(11, "fma (dependent)")
  R(6, "div_ (rcp-newton)")
  R(7, "a/b (IEEE)")
  R(0, "atan2_xpos Horner")
  R(1, "atan2_xpos Estrin")
  R(8, "atan2 ocml")
  R(2, "atan_ Horner")
  R(3, "atan_ Estrin")
  R(9, "atan ocml")
  R(4, "sin_ Horner")
  R(10, "sin ocml")
  R(5, "sincos_ Horner")
  R(14, "dpp bcast + fma")
  R(17, "atan2_fast")
  R(18, "atan_fast")
  R(19, "sin_wide")
  R(20, "sincos_fast")
  R(21, "div6")
  R(15, "fast rk4 step LPM=2 (/4)")
  R(16, "fast rk4 step LPM=1 (/4)")
  return 0;
}
