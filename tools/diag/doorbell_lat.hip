// Diagnostic (not product): host -> device doorbell round trips for the armed controller tick.
// One persistent launch per mode answers N rings; the host rings (stores seq into the doorbell
// word) and spins until the kernel's answer (seq in a pinned tag) arrives; p50 / p99 of the
// round trip.  Modes:
//   0  pinned host memory, polled by block 0 (system-scope loads), answered by block 0
//   1  fine-grained device memory (hipDeviceMallocFinegrained) written by the host through its
//      pointer, polled by block 0
//   2  pinned host memory polled by block 0, relayed to device memory (sc1 store), polled by
//      block 1, which answers (the armed tick's relay)
// Every poll is bounded (s_memrealtime); the launch ends after N rings or on a timeout.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/diag/doorbell_lat tools/diag/doorbell_lat.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void ring_kernel(int mode, const uint64_t* door, uint64_t* relay, uint64_t* tag, int n) {
  if (threadIdx.x != 0) return;
  const uint64_t bound = 100000000ull;   // 1 s per ring at 100 MHz
  for (int i = 1; i <= n; ++i) {
    const uint64_t want = (uint64_t)i;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (mode == 2 && blockIdx.x == 0) {
      while (ld_sys(door) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) return;
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(relay, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (mode == 2) {                      // block 1
      while (ld_agent(relay) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) return;
        __builtin_amdgcn_s_sleep(1);
      }
    } else {
      while (ld_sys(door) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) return;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __hip_atomic_store(tag, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// mode 3: the armed tick's pattern — 13 tagged words (x_t halves + status) in pinned memory,
// block 0 polls them and relays them to device memory, blocks 1..B-1 poll the 13 device words;
// each block stores when it saw ring i (s_memrealtime) into seen[i][blk]; the last arrival
// (a counter) answers the host.
__global__ void relay13_kernel(const uint64_t* door, uint64_t* relay, uint64_t* tag, unsigned* cnt,
                               unsigned long long* seen, int n, int variant) {
  __shared__ int go;
  const uint64_t bound = 100000000ull;
  for (int i = 1; i <= n; ++i) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 0;
      for (;;) {
        uint64_t w[13];
        bool all = true;
        if (blockIdx.x == 0) {
#pragma unroll
          for (int q = 0; q < 13; ++q) w[q] = ld_sys(&door[q]);
        } else if (variant == 0) {
#pragma unroll
          for (int q = 0; q < 13; ++q) w[q] = ld_agent(&relay[q]);
        } else {                          // variant 1: the status word alone, then the rest
          w[12] = ld_agent(&relay[12]);
          if ((uint32_t)(w[12] >> 32) == (uint32_t)i) {
#pragma unroll
            for (int q = 0; q < 12; ++q) w[q] = ld_agent(&relay[q]);
          } else {
            all = false;
          }
        }
#pragma unroll
        for (int q = 0; q < 13; ++q) all = all && (uint32_t)(w[q] >> 32) == (uint32_t)i;
        if (all) {
          if (blockIdx.x == 0) {
            if (variant == 1) {
#pragma unroll
              for (int q = 0; q < 12; ++q) __hip_atomic_store(&relay[q], w[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __builtin_amdgcn_s_waitcnt(0);
              __hip_atomic_store(&relay[12], w[12], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
#pragma unroll
              for (int q = 0; q < 13; ++q) __hip_atomic_store(&relay[q], w[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          ok = 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) break;
        __builtin_amdgcn_s_sleep(1);
      }
      seen[(size_t)i * gridDim.x + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
      go = ok;
      if (ok) {
        const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)i * gridDim.x - 1)
          __hip_atomic_store(tag, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
    if (!go) return;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  uint64_t *h_door = nullptr, *d_door = nullptr, *h_tag = nullptr, *d_tag = nullptr, *fg = nullptr, *relay = nullptr;
  CHECK(hipHostMalloc((void**)&h_door, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc((void**)&h_tag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer((void**)&d_door, h_door, 0));
  CHECK(hipHostGetDevicePointer((void**)&d_tag, h_tag, 0));
  CHECK(hipMalloc((void**)&relay, 64));
  const bool have_fg = hipExtMallocWithFlags((void**)&fg, 64, hipDeviceMallocFinegrained) == hipSuccess;
  for (int mode = 0; mode < 3; ++mode) {
    if (mode == 1 && !have_fg) {
      std::printf("mode 1: hipExtMallocWithFlags(fine-grained) failed\n");
      continue;
    }
    uint64_t* host_door = mode == 1 ? fg : h_door;      // what the host stores into
    const uint64_t* dev_door = mode == 1 ? fg : d_door;  // what the kernel polls
    if (mode == 1) {
      // the host writes device memory through the pointer: if the BAR does not map it, this faults
      CHECK(hipMemset(fg, 0, 64));
      CHECK(hipDeviceSynchronize());
    }
    *(volatile uint64_t*)host_door = 0;
    *(volatile uint64_t*)h_tag = 0;
    CHECK(hipMemset(relay, 0, 64));
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(ring_kernel, dim3(mode == 2 ? 2 : 1), dim3(64), 0, 0, mode, dev_door, relay, d_tag, n);
    CHECK(hipGetLastError());
    std::vector<double> us;
    bool ok = true;
    for (int i = 1; i <= n && ok; ++i) {
      // the kernel is polling: give it a moment, as a paced tick would
      const auto w = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - w < std::chrono::microseconds(20)) {
      }
      const auto t0 = std::chrono::steady_clock::now();
      __atomic_store_n(host_door, (uint64_t)i, __ATOMIC_RELEASE);
      while (__atomic_load_n(h_tag, __ATOMIC_ACQUIRE) != (uint64_t)i) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
          ok = false;
          break;
        }
      }
      us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CHECK(hipDeviceSynchronize());
    std::sort(us.begin(), us.end());
    std::printf("mode %d: %s rings %zu  round trip p50 %.2f us  p10 %.2f  p99 %.2f\n", mode, ok ? "ok" : "TIMEOUT",
                us.size(), us[us.size() / 2], us[us.size() / 10], us[us.size() * 99 / 100]);
  }
  // mode 3: the armed tick's relay pattern, B blocks
  for (int variant = 0; variant < 2; ++variant) {
    const int B = 64, R = 400;
    unsigned* cnt = nullptr;
    unsigned long long* seen = nullptr;
    uint64_t* rel13 = nullptr;
    CHECK(hipMalloc((void**)&cnt, 4));
    CHECK(hipMalloc((void**)&rel13, 13 * 8));
    CHECK(hipMalloc((void**)&seen, (size_t)(R + 1) * B * 8));
    CHECK(hipMemset(cnt, 0, 4));
    CHECK(hipMemset(rel13, 0, 13 * 8));
    for (int q = 0; q < 16; ++q) h_door[q % 8] = 0;
    *(volatile uint64_t*)h_tag = 0;
    uint64_t* door13 = nullptr;
    uint64_t* d_door13 = nullptr;
    CHECK(hipHostMalloc((void**)&door13, 16 * 8, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostGetDevicePointer((void**)&d_door13, door13, 0));
    for (int q = 0; q < 16; ++q) door13[q] = 0;
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(relay13_kernel, dim3(B), dim3(64), 0, 0, d_door13, rel13, d_tag, cnt, seen, R, variant);
    CHECK(hipGetLastError());
    std::vector<double> us;
    bool ok = true;
    for (int i = 1; i <= R && ok; ++i) {
      const auto w = std::chrono::steady_clock::now();
      while (std::chrono::steady_clock::now() - w < std::chrono::microseconds(50)) {
      }
      const auto t0 = std::chrono::steady_clock::now();
      const uint64_t tg = (uint64_t)i << 32;
      for (int q = 0; q < 12; ++q) __atomic_store_n(&door13[q], tg | (uint64_t)(q + 1), __ATOMIC_RELAXED);
      __atomic_store_n(&door13[12], tg | 1u, __ATOMIC_RELEASE);
      while (__atomic_load_n(h_tag, __ATOMIC_ACQUIRE) != (uint64_t)i) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
          ok = false;
          break;
        }
      }
      us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> sv((size_t)(R + 1) * B);
    CHECK(hipMemcpy(sv.data(), seen, sv.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> spread;
    for (int i = 1; i <= R; ++i) {
      unsigned long long mx = 0;
      for (int b = 1; b < B; ++b) mx = std::max(mx, sv[(size_t)i * B + b]);
      spread.push_back((double)(mx - sv[(size_t)i * B]) / 100.0);
    }
    std::sort(us.begin(), us.end());
    std::sort(spread.begin(), spread.end());
    std::printf("mode 3 variant %d (%s): %s round trip p50 %.2f us p99 %.2f; block 0 -> last block p50 %.2f us p99 %.2f\n",
                variant, variant ? "status word first" : "13 words per poll", ok ? "ok" : "TIMEOUT", us[us.size() / 2],
                us[us.size() * 99 / 100], spread[spread.size() / 2], spread[spread.size() * 99 / 100]);
  }
  return 0;
}
