// Diagnostic: cycles per look-ahead step (step_fast<RK4, LPM=2>, the kernel's hot loop body)
// for ONE wave, s_memtime around 200 steps; built in ablation variants by tools/micro/ablate.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "dyn.hpp"
using namespace llampc;

__global__ __launch_bounds__(64) void steps(const double* prm, double* out, long long* cyc, int H) {
  VehK vk{prm[0], prm[1], prm[2], prm[3], prm[4], prm[5], prm[6], prm[7], prm[8], 0, 0};
  Tire t{prm[9] + 1e-3 * (threadIdx.x >> 1), prm[10], prm[11], prm[12], prm[13], prm[14]};
  const fm::FmK K = fm::FmK::load();
  const StageK sk = make_stage<2>(vk, t, threadIdx.x & 1);
  double x[6] = {prm[15], prm[16], prm[17], prm[18], prm[19] + 1e-4 * threadIdx.x, prm[20]};
  Input u;
  u.a = prm[21];
  u.d = prm[22];
  u.sd = prm[23];
  u.cd = prm[24];
  bool bad = false;
  __syncthreads();
  long long t0 = clock64();
  for (int k = 0; k < H; ++k) step_fast<0, 2>(vk, t, sk, x, u, 0.02, K, bad);
  long long t1 = clock64();
  out[threadIdx.x] = x[0] + x[1] + x[2] + x[3] + x[4] + x[5] + bad;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double hp[32] = {0.029, 0.033, 0.041, 1 / 0.041, 1 / 27.8e-6, 0.287, 0.0545, 0.0518, 0.00035,
                   2.579, 1.2, 0.192, 3.3852, 1.2691, 0.1737,
                   0.5, -1.0, -0.6, 1.8, 0.05, 0.4, 0.5, 0.05, 0.04998, 0.99875};
  double *prm, *out;
  long long* cyc;
  hipMalloc(&prm, sizeof hp);
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(prm, hp, sizeof hp, hipMemcpyHostToDevice);
  const int H = 200;
  long long c = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(steps, dim3(1), dim3(64), 0, 0, prm, out, cyc, H);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  }
  printf("%s %.1f cycles/step\n", VARIANT, (double)c / H);
  return 0;
}
