// nlp.hip — the setupNLP.solve drop-in (llampc_nlp_*, include/llampc.h): the selected model's
// NMPC (nmpc.py:14-203: Euler transcription of Dynamic.casadi, nmpc.py:58-60; the objective
// nmpc.py:44-111; input bounds and the steering-rate bound nmpc.py:102-105) solved on the
// device by the cross-entropy method — no IPOPT here (casadi is absent; its optimum is parity
// unpinned).  One launch per iteration, all enqueued back to back, then the Euler trajectory
// of the best sequence (integrate_kernel) and ONE copy back:
//
//   sample blocks   each draws 64 sequences from the iteration's (mean, std) — Philox noise
//                   (ctl.hpp), the bounds, the rate chain in order over the horizon; sample 0 is
//                   the mean itself, sample 1 of the first iteration holds uprev — and rolls
//                   them out (the plan kernel's rollout, NLP-Euler, four lanes per rollout,
//                   candidates in LDS), writing each sample's objective (+inf if infeasible);
//   the last block  (ticket) sorts the samples' objectives (bitonic in LDS, NaN last, ties to
//                   the lower index), regenerates the E elite sequences and sets the next mean /
//                   std to their mean / standard deviation (NumPy's axis-0 order), keeping the
//                   best sequence seen so far.
#include "plan_dev.hpp"
#include "nlp.hpp"

namespace llampc {

namespace {

// sample s of iteration `it` before the rate chain (the bounds applied)
__device__ __forceinline__ double nlp_raw(const NlpLaunch& a, const NlpState* st, int s, int k, int j) {
#pragma clang fp contract(off)
  const double m = st->mean[k][j];
  double u;
  if (s == 0) {
    u = m;
  } else if (s == 1 && a.it == 0 && a.has_hold) {
    u = j ? a.up1 : a.up0;
  } else {
    const double z = ctl_z((uint32_t)((s * a.H + k) * 2 + j), a.call, a.seed, (uint32_t)(a.it + 1));
    const double zu = z * 1.7320508075688772;       // unit variance (sqrt(3), as np.sqrt(3.0))
    const double d = zu * st->std_[k][j];
    u = m + d;
  }
  return np_clip(u, j ? a.umin1 : a.umin0, j ? a.umax1 : a.umax0);
}

// u_k <- clip(u_k, u_{k-1} + lo, u_{k-1} + hi) in order over k (nmpc.py:104-105 as the host
// sampler applies it); lo > hi: no rate bound on this input
__device__ __forceinline__ void nlp_rate_chain(double* u, int H, double up, double lo, double hi) {
#pragma clang fp contract(off)
  if (!(lo <= hi)) return;
  double prev = up;
  for (int k = 0; k < H; ++k) {
    const double a = prev + lo, b = prev + hi;
    prev = np_clip(u[2 * k], a, b);
    u[2 * k] = prev;
  }
}

// order-preserving key of an objective: NaN above +inf (a diverged rollout sorts last)
__device__ __forceinline__ uint64_t nlp_key(double v) {
  const double w = (v != v) ? __builtin_nan("") : v + 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(w);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ void nlp_complete(const NlpLaunch& a, unsigned char* smem) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, H = a.H, S = a.samples, E = a.elite;
  NlpState* st = a.st;
  uint64_t* key = reinterpret_cast<uint64_t*>(smem + kScratchBytes);      // [S]
  uint32_t* idx = reinterpret_cast<uint32_t*>(key + S);                    // [S]
  double* eu = reinterpret_cast<double*>(idx + S + (S & 1));                // [E][H][2]
  for (int i = tid; i < S; i += kBlock) {
    key[i] = nlp_key(ld_wt(&a.cost[i]));
    idx[i] = (uint32_t)i;
  }
  __syncthreads();
  // bitonic sort of (key, index) ascending
  for (int k = 2; k <= S; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < S; i += kBlock) {
        const int l = i ^ j;
        if (l > i) {
          const uint64_t ki = key[i], kl = key[l];
          const uint32_t ii = idx[i], il = idx[l];
          const bool l_less = (kl < ki) || (kl == ki && il < ii);
          const bool up = (i & k) == 0;
          if (up ? l_less : !l_less) {
            key[i] = kl;
            key[l] = ki;
            idx[i] = il;
            idx[l] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  // the elite sequences, regenerated (the sample blocks' generator), then their rate chains
  for (int e = tid; e < E * H * 2; e += kBlock) {
    const int r = e / (2 * H), q = e - r * 2 * H;
    eu[e] = nlp_raw(a, st, (int)idx[r], q >> 1, q & 1);
  }
  __syncthreads();
  if (tid < 2 * E) {
    const int r = tid >> 1, j = tid & 1;
    nlp_rate_chain(eu + 2 * (size_t)r * H + j, H, j ? a.up1 : a.up0, j ? a.rlo1 : a.rlo0, j ? a.rhi1 : a.rhi0);
  }
  __syncthreads();
  const double c0 = ld_wt(&a.cost[idx[0]]);
  const bool better = c0 < st->best_j;              // the best sequence so far (NaN never)
  __syncthreads();                                  // every thread has read best_j
  if (tid < 2 * H) {
    // mean / std over the elite in np.mean(axis=0) / np.std(axis=0)'s order: an axis-0
    // reduction adds the rows in sequence (checked against NumPy), std = sqrt(mean((x - m)^2))
    const int k = tid >> 1, j = tid & 1;
    auto at = [&](int e) { return eu[(2 * (size_t)e * H) + 2 * k + j]; };
    double acc = 0.0;
    for (int e = 0; e < E; ++e) acc += at(e);
    const double m = acc / E;
    double s = 0.0;
    for (int e = 0; e < E; ++e) {
      const double d = at(e) - m;
      s += d * d;
    }
    st->mean[k][j] = m;
    st->std_[k][j] = sqrt(s / E) + a.std_floor;
    if (better) st->best_u[k][j] = eu[2 * k + j];
  }
  if (tid == 0) {
    if (better) {
      st->best_j = c0;
      st->best_it = a.it;
    }
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

__global__ __launch_bounds__(kBlock) void nlp_kernel(NlpLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Scratch sc(smem);
  int* flag = reinterpret_cast<int*>(smem + kFlagOff);
  const int tid = threadIdx.x, H = a.H, blk = (int)blockIdx.x;
  constexpr int LPM = 4, kPerBlock = kBlock / LPM;   // 64 samples per block
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);            // xref [H+1][2]
  double* Ul = sx + 2 * (H + 1);                                            // [64][H][2]
  double* x0 = Ul + 2 * (size_t)kPerBlock * H;                              // [6]
  const NlpState* st = a.st;
  for (int e = tid; e <= H; e += kBlock) {
    sx[2 * e] = a.xref[e];
    sx[2 * e + 1] = a.xref[(H + 1) + e];
  }
  if (tid < 6) x0[tid] = a.x0[tid];
  for (int e = tid; e < kPerBlock * H * 2; e += kBlock) {
    const int r = e / (2 * H), q = e - r * 2 * H;
    Ul[e] = nlp_raw(a, st, blk * kPerBlock + r, q >> 1, q & 1);
  }
  __syncthreads();
  if (tid < 2 * kPerBlock) {
    const int r = tid >> 1, j = tid & 1;
    nlp_rate_chain(Ul + 2 * (size_t)r * H + j, H, j ? a.up1 : a.up0, j ? a.rlo1 : a.rlo0, j ? a.rhi1 : a.rhi0);
  }
  __syncthreads();
  // rollouts: a quad per sample (the plan kernel's NLP-Euler fast stage + the general re-run)
  const int sub = tid % LPM, c = tid / LPM;
  const Tire t = load_tire(a.la.params, 1, 0);
  CostK q = a.la.cost;
  VehK veh = a.la.veh;
  double Ts = a.la.Ts;
  for (int m = 0; m < 4; ++m) {
    pin_vgpr(q.Q[m]);
    pin_vgpr(q.R[m]);
    pin_vgpr(q.P[m]);
  }
  for (int m = 0; m < 2; ++m) {
    pin_vgpr(q.umin[m]);
    pin_vgpr(q.umax[m]);
    pin_vgpr(q.dmax[m]);
  }
  pin_vgpr(Ts);
  const StageK sk = make_stage<LPM>(veh, t, sub, 1.0);
  const FusedK fq = make_fused(veh, sk, Ts, false);
  const fm::FmK K = fm::FmK::load();
  bool bad = false;
  double J = rollout<1, false, LPM, 0, true, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K,
                                                          fq, bad);
  int bi = bad;
  bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
  bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
  if (__builtin_expect(__any(bi), 0)) {
    bool unused = false;
    if (bi) J = rollout<1, false, LPM, 0, false, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K,
                                                              fq, unused);
  }
  if (sub == 0) st_wt(&a.cost[blk * kPerBlock + c], J);
  if (!ticket_last(a.ticket, gridDim.x, flag)) return;
  nlp_complete(a, smem);
}

size_t nlp_lds_bytes(int H, int samples, int elite) {
  const size_t blocks = kScratchBytes + 16 * (size_t)(H + 1) + 16 * 64 * (size_t)H + 64;
  const size_t last = kScratchBytes + 12 * (size_t)samples + 8 + 16 * (size_t)elite * H;
  return std::max(blocks, last);
}

hipError_t launch_nlp(const NlpLaunch& a, hipStream_t s) {
  const size_t lds = std::max<size_t>(nlp_lds_bytes(a.H, a.samples, a.elite), 82 * 1024);
  allow_lds(nlp_kernel);
  hipLaunchKernelGGL(nlp_kernel, dim3(a.samples / 64), dim3(kBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace llampc
