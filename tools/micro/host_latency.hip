// Host-side latency breakdown of one synchronous tick (diagnostic, not shipped).
// Variants, 1,000 timed iterations after 50 warm-up each, p50/p99 in microseconds:
//   plan       llampc_plan (host pointers: H2D pack, plan kernel, D2H record, stream sync)
//   plan_dev   llampc_plan_device on resident inputs + hipStreamSynchronize
//   empty_sync empty kernel + hipStreamSynchronize
//   empty_spin empty kernel that stores a tag into pinned host memory; host spins on it
//   copies     H2D of the input pack + D2H of one record + hipStreamSynchronize (no kernel)
//   plan_spin  llampc_plan_device + a 1-thread kernel after it that copies the record into
//              pinned host memory with a tag; the host spins on the tag
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude tools/micro/host_latency.hip
//        -Llla-mpc_amd/llampc/_lib -lllampc_hip -Wl,-rpath,$PWD/lla-mpc_amd/llampc/_lib
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
#include "llampc.h"

#define CK(x)                                                                         \
  do {                                                                                \
    int rc_ = (int)(x);                                                               \
    if (rc_) {                                                                        \
      std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,      \
                   llampc_last_error());                                              \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void empty_kernel() {}

__global__ void tag_kernel(volatile unsigned long long* tag, unsigned long long v) {
  __threadfence_system();
  *tag = v;
}

// copies the record (as 8-B words) to pinned host memory, then publishes the tag
__global__ void rec_copy_kernel(const unsigned long long* rec, unsigned long long* host, int words,
                                volatile unsigned long long* tag, unsigned long long v) {
  for (int i = threadIdx.x; i < words; i += blockDim.x) host[i] = rec[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) *tag = v;
}

using clk = std::chrono::steady_clock;

static void report(const char* name, std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  std::printf("{\"variant\": \"%s\", \"p50_us\": %.2f, \"p99_us\": %.2f, \"n\": %zu}\n", name,
              v[v.size() / 2], v[(size_t)(v.size() * 0.99)], v.size());
  std::fflush(stdout);
}

template <class F>
static void run(const char* name, F f, int warm = 50, int iters = 1000) {
  std::vector<double> t;
  for (int i = 0; i < warm + iters; ++i) {
    auto a = clk::now();
    f(i);
    auto b = clk::now();
    if (i >= warm) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  report(name, t);
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? std::atoll(argv[1]) : 10000;
  const int H = 20, C = 1, W = 10;
  std::mt19937_64 rng(0);
  std::normal_distribution<double> z(0.0, 1.0);
  // Pacejka rows (Bf, Cf, Df, Br, Cr, Dr) around the ORCA nominal (orca.py:13-27)
  const double nom[6] = {2.579, 1.2, 0.192, 3.3852, 1.2691, 0.1737};
  const double sig[6] = {0.2, 0.1, 0.5, 0.2, 0.1, 0.5};
  std::vector<double> params(6 * N);
  for (int64_t i = 0; i < N; ++i)
    for (int k = 0; k < 6; ++k) params[k * N + i] = nom[k] * (1.0 + sig[k] * 0.3 * z(rng));
  llampc_vehicle veh{0.029, 0.033, 0.041, 27.8e-6, 0.287, 0.0545, 0.0518, 0.00035, 0, 0};
  llampc_bank* bank = nullptr;
  CK(llampc_bank_create(params.data(), N, 0, &veh, W, 0, &bank));

  // inputs: a straight-ish state, small steering, xref ahead of the car
  std::vector<double> xp = {0.1, 0.2, 0.3, 1.5, 0.01, 0.2}, up = {0.4, 0.05}, xn(6), uprev = {0.4, 0.05};
  for (int m = 0; m < 6; ++m) xn[m] = xp[m] + 0.01 * (m + 1);
  std::vector<double> U(2 * C * H), xref(2 * (H + 1));
  for (int k = 0; k < H; ++k) {
    U[2 * k] = 0.4;
    U[2 * k + 1] = 0.05 * std::sin(0.3 * k);
  }
  for (int k = 0; k <= H; ++k) {
    xref[k] = xn[0] + 0.03 * k;
    xref[(H + 1) + k] = xn[1] + 0.01 * k;
  }
  llampc_plan_in in{};
  in.x_prev = xp.data();
  in.u_prev = up.data();
  in.x_now = xn.data();
  in.U = U.data();
  in.xref = xref.data();
  in.uprev = uprev.data();
  in.C = C;
  in.H = H;
  in.K = 10;
  in.integrator = LLAMPC_RK4;
  in.do_lookback = 1;
  in.do_lookahead = 1;
  in.nan_policy = LLAMPC_NAN_FIRST;
  in.xref_mode = LLAMPC_XREF_GIVEN;
  in.current_model = 0;
  in.Ts = 0.02;
  in.cost.Q[0] = in.cost.Q[3] = 1.0;
  in.cost.R[0] = 5e-3;
  in.cost.R[3] = 1.0;
  in.cost.umin[0] = -0.1;
  in.cost.umin[1] = -0.35;
  in.cost.umax[0] = 1.0;
  in.cost.umax[1] = 0.35;
  in.cost.rate_max[0] = -1.0;
  in.cost.rate_max[1] = 5.0;
  llampc_plan_out out{};

  run("plan", [&](int) { CK(llampc_plan(bank, &in, &out, nullptr, nullptr, nullptr)); });

  // resident inputs for the device API
  const size_t L = 16 + 2 * (H + 1) + 2 * C * H;
  std::vector<double> pack(L, 0.0);
  std::memcpy(&pack[0], xp.data(), 48);
  std::memcpy(&pack[6], up.data(), 16);
  std::memcpy(&pack[8], xn.data(), 48);
  std::memcpy(&pack[14], uprev.data(), 16);
  std::memcpy(&pack[16], xref.data(), 8 * 2 * (H + 1));
  std::memcpy(&pack[16 + 2 * (H + 1)], U.data(), 8 * 2 * C * H);
  double* dpack = nullptr;
  void* dout = nullptr;
  CK(hipMalloc(&dpack, L * 8));
  CK(hipMalloc(&dout, sizeof(llampc_plan_out)));
  CK(hipMemcpy(dpack, pack.data(), L * 8, hipMemcpyHostToDevice));
  llampc_plan_in din = in;
  din.x_prev = dpack;
  din.u_prev = dpack + 6;
  din.x_now = dpack + 8;
  din.uprev = dpack + 14;
  din.xref = dpack + 16;
  din.U = dpack + 16 + 2 * (H + 1);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  run("plan_dev", [&](int) {
    CK(llampc_plan_device(bank, &din, dout, nullptr, nullptr, nullptr, s));
    CK(hipStreamSynchronize(s));
  });
  run("empty_sync", [&](int) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
    CK(hipStreamSynchronize(s));
  });
  unsigned long long* htag = nullptr;
  unsigned long long* hrec = nullptr;
  CK(hipHostMalloc((void**)&htag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&hrec, sizeof(llampc_plan_out), hipHostMallocCoherent | hipHostMallocMapped));
  unsigned long long *dtag = nullptr, *drec = nullptr;
  CK(hipHostGetDevicePointer((void**)&dtag, htag, 0));
  CK(hipHostGetDevicePointer((void**)&drec, hrec, 0));
  *htag = 0;
  unsigned long long seq = 0;
  auto spin = [&](unsigned long long v) {
    auto t0 = clk::now();
    while (__atomic_load_n(htag, __ATOMIC_ACQUIRE) != v) {
      if (std::chrono::duration<double>(clk::now() - t0).count() > 2.0) {
        std::fprintf(stderr, "spin timeout\n");
        std::exit(2);
      }
    }
  };
  run("empty_spin", [&](int) {
    ++seq;
    hipLaunchKernelGGL(tag_kernel, dim3(1), dim3(64), 0, s, dtag, seq);
    spin(seq);
  });
  CK(hipStreamSynchronize(s));
  llampc_plan_out* hin = nullptr;
  CK(hipHostMalloc((void**)&hin, 4096, hipHostMallocDefault));
  std::memcpy(hin, pack.data(), L * 8);
  run("copies", [&](int) {
    CK(hipMemcpyAsync(dpack, hin, L * 8, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(hrec, dout, sizeof(llampc_plan_out), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
  });
  const int words = (int)(sizeof(llampc_plan_out) / 8);
  run("plan_spin", [&](int) {
    ++seq;
    CK(llampc_plan_device(bank, &din, dout, nullptr, nullptr, nullptr, s));
    hipLaunchKernelGGL(rec_copy_kernel, dim3(1), dim3(256), 0, s, (const unsigned long long*)dout, drec,
                       words, dtag, seq);
    spin(seq);
  });
  CK(hipStreamSynchronize(s));
  run("plan_dev_again", [&](int) {
    CK(llampc_plan_device(bank, &din, dout, nullptr, nullptr, nullptr, s));
    CK(hipStreamSynchronize(s));
  });
  CK(llampc_bank_destroy(bank));
  return 0;
}
