// Diagnostic: issue cost (shader cycles per wave-instruction) of the VALU instructions of
// the rollout stage, one wave alone on its SIMD.  Each case: a loop of 16 INDEPENDENT
// instructions (8 register pairs, no dependency inside a group) x 8 per iteration x iters.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void issue(double* io, long long* cyc, int iters) {
  double a0 = io[threadIdx.x], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
         a6 = a0 + 6, a7 = a0 + 7;
  double b = io[64 + threadIdx.x], c = io[128 + threadIdx.x];
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define FMA(i) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a##i) : "v"(b), "v"(c));
#define MUL(i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a##i) : "v"(b));
#define RCP(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(a##i));
#define MAX(i) asm volatile("v_max_f64 %0, %0, %1" : "+v"(a##i) : "v"(b));
#define DPP(i) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[2,3,2,3] row_mask:0xf bank_mask:0xf" : "=v"(*((int*)&a##i)) : "v"(*((int*)&b)));
#define CND(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(*((int*)&a##i)) : "v"(*((int*)&b)));
#define XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(*((int*)&a##i)) : "v"(*((int*)&b)));
#define DEPFMA(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
    if (OP == 0) { R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) R8(FMA) }
    if (OP == 1) { R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) R8(MUL) }
    if (OP == 2) { R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) R8(RCP) }
    if (OP == 3) { R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) R8(MAX) }
    if (OP == 4) { R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) R8(DPP) }
    if (OP == 5) { R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) R8(CND) }
    if (OP == 6) { R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) R8(XOR) }
    if (OP == 7) { R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) R8(DEPFMA) }
    if (OP == 8) { R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) R8(FMA) R8(XOR) }           // 8 fp64 + 8 32-bit
    if (OP == 9) { R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) R8(FMA) R8(DPP) }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  io[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP>
static double run(double* io, long long* cyc, int iters) {
  issue<OP><<<1, 64>>>(io, cyc, iters);
  issue<OP><<<1, 64>>>(io, cyc, iters);
  long long h;
  hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
  return (double)h / (128.0 * iters);
}

int main() {
  double* io;
  long long* cyc;
  hipMalloc(&io, 192 * 8);
  hipMalloc(&cyc, 8);
  double h[192];
  for (int i = 0; i < 192; ++i) h[i] = 1.0 + 1e-3 * i;
  hipMemcpy(io, h, sizeof h, hipMemcpyHostToDevice);
  const int it = 500;
  printf("cycles per wave-instruction (one wave alone, 16 independent per group):\n");
  printf("v_fma_f64 %.2f\n", run<0>(io, cyc, it));
  printf("v_mul_f64 %.2f\n", run<1>(io, cyc, it));
  printf("v_rcp_f64 %.2f\n", run<2>(io, cyc, it));
  printf("v_max_f64 %.2f\n", run<3>(io, cyc, it));
  printf("v_mov_b32_dpp %.2f\n", run<4>(io, cyc, it));
  printf("v_cndmask_b32 %.2f\n", run<5>(io, cyc, it));
  printf("v_xor_b32 %.2f\n", run<6>(io, cyc, it));
  printf("v_fma_f64 dependent %.2f\n", run<7>(io, cyc, it));
  printf("fma_f64+xor_b32 mix (per instr) %.2f\n", run<8>(io, cyc, it));
  printf("fma_f64+dpp mix (per instr) %.2f\n", run<9>(io, cyc, it));
  return 0;
}
