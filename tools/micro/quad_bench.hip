// Diagnostic: shader cycles per look-ahead step of the fused LPM-4 quad (dyn.hpp step_fused
// <4, SPLIT>, the plan kernel's hot loop body) for ONE wave on its SIMD, s_memtime around
// 200 steps.  ROLL=2 interleaves two independent rollouts per lane in the same loop: if a
// step of two costs about one step of one, the loop is latency-bound (dependency chain),
// if it costs two, issue-bound.  Built by tools/micro/quad_bench.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dyn.hpp"
using namespace llampc;

#ifndef ROLL
#define ROLL 1
#endif

__global__ __launch_bounds__(64) void steps(const double* prm, double* out, long long* cyc, int H) {
  VehK vk{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], prm[8], 0, 0};
  const int sub = threadIdx.x & 3;
  const fm::FmK K = fm::FmK::load();
  StageK sk[ROLL];
  FusedK q[ROLL];
  double x[ROLL][6];
  Dom dm[ROLL];
  for (int r = 0; r < ROLL; ++r) {
    Tire t{prm[9] + 1e-3 * (threadIdx.x >> 2) + 1e-4 * r, prm[10], prm[11], prm[12], prm[13], prm[14]};
    sk[r] = make_stage<4>(vk, t, sub, prm[25]);
    sk[r].ch[0].lw = sk[r].ch[0].lw / prm[25];
    if (sub >= 2) sk[r].ch[0].lw = sk[r].ch[0].sg = sk[r].ch[0].B = sk[r].ch[0].nsB = 0.0;
    q[r] = make_fused(vk, sk[r], prm[25], true);
    const double x0[6] = {prm[15], prm[16], prm[17], prm[18], prm[19] + 1e-4 * threadIdx.x + 1e-5 * r, prm[20]};
    for (int m = 0; m < 6; ++m) x[r][m] = x0[m];
    x[r][0] = (sub & 1) ? x0[1] : x0[0];
    x[r][2] = x0[2] * K.two_pi;
    x[r][5] = x0[5] * prm[25];
    dm[r].init();
  }
  const FusedIn fi = fused_in(q[0], Input{prm[21], prm[22], prm[23], prm[24]});
  __syncthreads();
  const long long t0 = clock64();
  for (int k = 0; k < H; ++k) {
#pragma unroll
    for (int r = 0; r < ROLL; ++r) step_fused<4, true>(sk[r], q[r], x[r], fi, prm[22], K, dm[r]);
  }
  const long long t1 = clock64();
  double acc = 0.0;
  for (int r = 0; r < ROLL; ++r) acc += x[r][0] + x[r][2] + x[r][3] + x[r][4] + x[r][5] + dm[r].ok();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double hp[32] = {0.029, 0.033, 0.041, 1 / 0.041, 1 / 27.8e-6, 0.287, 0.0545, 0.0518, 0.00035,
                   2.579, 1.2, 0.192, 3.3852, 1.2691, 0.1737,
                   0.5, -1.0, -0.6, 1.8, 0.05, 0.4, 0.5, 0.05, 0.04998, 0.99875, 0.02};
  double *prm, *out;
  long long* cyc;
  (void)hipMalloc(&prm, sizeof hp);
  (void)hipMalloc(&out, 64 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(prm, hp, sizeof hp, hipMemcpyHostToDevice);
  const int H = 200;
  long long c = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(steps, dim3(1), dim3(64), 0, 0, prm, out, cyc, H);
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  }
  double o[64];
  (void)hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
  printf("%s ROLL=%d %.1f cycles/step (%.1f per rollout-step)  check %.6g\n", VARIANT, ROLL, (double)c / H,
         (double)c / H / ROLL, o[0]);
  return 0;
}
