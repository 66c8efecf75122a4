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
//                   Each block then sorts its 64 (objective, index) keys in one wave (a bitonic
//                   network of DPP / shuffle exchanges: NaN last, ties to the lower index) and
//                   publishes its best len = next_pow2(E) sorted;
//   the last block  (ticket) merges the blocks' lists pairwise up a tree — the lower len of two
//                   sorted lists is min(a_i, b_(len-1-i)), bitonic, then one half-cleaner
//                   network in registers per level — to the E best overall in order,
//                   regenerates the E elite sequences and sets the next mean / std to their mean
//                   / standard deviation (NumPy's axis-0 order), keeping the best sequence seen
//                   so far.  (A bitonic sort of all samples in LDS took 36 us of the 62 us
//                   round: 55 barrier-separated passes.)
#include "plan_dev.hpp"
#include "nlp.hpp"

namespace llampc {

#ifdef LLAMPC_STAMPS
// Diagnostic build only: s_memrealtime per block and phase of the last launch
// (tools/diag/nlp_phases.py): 0 entry, 1 drawn, 2 rate-clipped, 3 rolled out; the completing
// block: 4 keyed, 5 sorted, 6 elite drawn, 7 elite clipped, 8 done; 9 staged (sample blocks).
static __device__ unsigned long long g_nlp_ph[32][12];
#define NLP_STAMP(slot)                                                                               \
  do {                                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < 32) g_nlp_ph[blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" int llampc_debug_nlp_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nlp_ph), sizeof(g_nlp_ph)) == hipSuccess ? 0 : -2;
}
#else
#define NLP_STAMP(slot) \
  do {                  \
  } while (0)
#endif

namespace {

// The search's noise: one Philox4x32-10 call per PAIR of values, the counter (i / 2, call lo,
// call hi, round + 1): value i takes the 16-bit halves (low for even i, high for odd) of the
// four words, z = (h0 + h1 + h2 + h3 + 2) 2^-16 - 2 — the 4-term Irwin-Hall variate on
// 16-bit cells of the controller's candidates too (ctl.hpp ctl_z2; centred: mean 0, variance
// 1/3 - 1/(3 2^32)), at half the Philox calls of one per value (the sample blocks' draw was
// 4.3 of a 26 us round).
__device__ __forceinline__ void nlp_z2(uint32_t pair, uint64_t call, uint64_t seed, uint32_t stream, double& z0,
                                       double& z1) {
  const Philox4 w = philox4x32_10(Philox4{pair, (uint32_t)call, (uint32_t)(call >> 32), stream}, (uint32_t)seed,
                                  (uint32_t)(seed >> 32));
  const uint32_t lo = (w.x & 0xFFFFu) + (w.y & 0xFFFFu) + (w.z & 0xFFFFu) + (w.w & 0xFFFFu) + 2u;
  const uint32_t hi = (w.x >> 16) + (w.y >> 16) + (w.z >> 16) + (w.w >> 16) + 2u;
  z0 = (double)lo * 0x1p-16 - 2.0;      // exact: integers < 2^19 and a power-of-two scale
  z1 = (double)hi * 0x1p-16 - 2.0;
}

// sample s of round `it` before the rate chain (the bounds applied), given its variate z;
// ms = the round's mean [H][2] then std [H][2] (LDS)
__device__ __forceinline__ double nlp_raw_z(const NlpLaunch& a, const double* ms, int it, int s, int k, int j,
                                            double z) {
#pragma clang fp contract(off)
  const double m = ms[2 * k + j];
  double u;
  if (s == 0) {
    u = m;
  } else if (s == 1 && it == 0 && a.has_hold) {
    u = j ? a.up1 : a.up0;
  } else {
    const double zu = z * 1.7320508075688772;       // unit variance (sqrt(3), as np.sqrt(3.0))
    const double d = zu * ms[2 * (a.H + k) + j];
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
__device__ __forceinline__ double nlp_unkey(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// (key, index) exchange step of a bitonic network across lanes lane ^ j: the lane keeps the
// smaller pair when `low`, else the larger (indices are distinct, so the order is total)
__device__ __forceinline__ void nlp_cx(uint64_t& k, uint32_t& i, int j, bool low) {
  const uint64_t pk = __shfl_xor(k, j, 64);
  const uint32_t pi = __shfl_xor(i, j, 64);
  const bool pless = pk < k || (pk == k && pi < i);
  if (low == pless) {
    k = pk;
    i = pi;
  }
}

__device__ __forceinline__ void nlp_traj_quad(const NlpLaunch& a, const double* sx, const double* ub, const double* x0);

// xmpc (nmpc.py:58-60): the NLP's Euler trajectory of the best sequence over all rounds, by
// one quad of the completing block (the sample blocks' fast rollout, the general re-run when
// its domain check fails) — it was a separate one-lane launch of the general evaluation, 32 us.
__device__ __forceinline__ void nlp_trajectory(const NlpLaunch& a, unsigned char* smem, double* ub, bool better,
                                               double bj, int bit) {
  const int tid = threadIdx.x, H = a.H;
  const NlpState* st = a.st;
  NlpResult* res = a.res;
  __syncthreads();                      // the elite rows are read; best_u is final
  double* sx = ub + 2 * (size_t)H;      // after the sequence: xref [H+1][2], x0 [6]
  double* x0 = sx + 2 * (size_t)(H + 1);
  for (int e = tid; e < 2 * H; e += kBlock) {
    const double v = better ? ub[e] : ld_wt(&st->best_u[0][0] + e);   // an earlier round's completion
    ub[e] = v;
    (&res->best_u[0][0])[e] = v;
  }
  if (tid == 0) {
    res->best_j = bj;
    res->best_it = bit;
  }
  for (int e = tid; e <= H; e += kBlock) {
    sx[2 * e] = a.xref[e];
    sx[2 * e + 1] = a.xref[(H + 1) + e];
  }
  if (tid < 6) x0[tid] = a.x0[tid];
  __syncthreads();
  if (tid < 4) nlp_traj_quad(a, sx, ub, x0);
  __threadfence_system();               // the result's host-memory stores, then the tag
  __syncthreads();
  if (tid == 0) __hip_atomic_store(a.host_tag, a.host_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one quad: the rollout with the trajectory written (lane 0) into the host result
__device__ __forceinline__ void nlp_traj_quad(const NlpLaunch& a, const double* sx, const double* ub, const double* x0) {
  const int tid = threadIdx.x;
  constexpr int LPM = 4;
  const int sub = tid;
  const Tire t = load_tire(a.la.params, 1, 0);
  const CostK q = a.la.cost;
  const VehK veh = a.la.veh;
  const double Ts = a.la.Ts;
  const StageK sk = make_stage<LPM>(veh, t, sub, 1.0);
  const FusedK fq = make_fused(veh, sk, Ts, false);
  const fm::FmK K = fm::FmK::load();
  double* out = sub == 0 ? &a.res->traj[0][0] : nullptr;
  if (sub == 0)
    for (int m = 0; m < 6; ++m) out[m] = x0[m];
  bool bad = false;
  (void)rollout<1, false, LPM, 0, true, false, true, true>(a.la, 0, 0, x0, sx, ub, veh, t, sk, q, Ts, a.up0, a.up1, K, fq,
                                                           bad, out);
  int bi = bad;
  bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
  bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
  if (bi) {
    bool unused = false;
    (void)rollout<1, false, LPM, 0, false, false, true, true>(a.la, 0, 0, x0, sx, ub, veh, t, sk, q, Ts, a.up0, a.up1, K,
                                                              fq, unused, out);
  }
}

// Round `it`'s completion (the block that added the last ticket): the elite, the next mean /
// std, the best so far.  The state is handed to the next round's blocks (other CUs, other
// XCDs) by sc1 stores and loads, as the sample blocks' lists (st_wt / ld_wt).
__device__ __forceinline__ void nlp_complete(const NlpLaunch& a, unsigned char* smem, int it) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, H = a.H, E = a.elite;
  const int len = nlp_list_len(E), nl = (int)gridDim.x;
  NlpState* st = a.st;
  uint64_t* kA = reinterpret_cast<uint64_t*>(smem + kScratchBytes);       // [nl * len] x 2
  uint64_t* kB = kA + (size_t)nl * len;
  uint32_t* iA = reinterpret_cast<uint32_t*>(kB + (size_t)nl * len);
  uint32_t* iB = iA + (size_t)nl * len;
  double* eu = reinterpret_cast<double*>(smem + kScratchBytes + 24 * (size_t)nl * len);   // [E][H][2]
  for (int e = tid; e < nl * len; e += kBlock) {
    kA[e] = ld_wt(&a.top_key[e]);
    iA[e] = ld_wt(&a.top_idx[e]);
  }
  __syncthreads();
  NLP_STAMP(4);
  // merge tree: lists 2g, 2g + 1 -> list g; a group of len lanes (inside one wave) per pair
  for (int n = nl; n > 1; n >>= 1) {
    const int pairs = n >> 1, gpp = kBlock / len, i = tid & (len - 1);
    for (int g0 = 0; g0 < pairs; g0 += gpp) {                      // block-uniform
      const int g = g0 + tid / len;
      if (g < pairs) {
        uint64_t k = kA[(size_t)(2 * g) * len + i];
        uint32_t x = iA[(size_t)(2 * g) * len + i];
        const uint64_t kb = kA[(size_t)(2 * g + 1) * len + (len - 1 - i)];
        const uint32_t xb = iA[(size_t)(2 * g + 1) * len + (len - 1 - i)];
        if (kb < k || (kb == k && xb < x)) {
          k = kb;
          x = xb;
        }
        for (int j = len >> 1; j > 0; j >>= 1) nlp_cx(k, x, j, (i & j) == 0);
        kB[(size_t)g * len + i] = k;
        iB[(size_t)g * len + i] = x;
      }
    }
    __syncthreads();
    uint64_t* tk = kA;
    kA = kB;
    kB = tk;
    uint32_t* ti = iA;
    iA = iB;
    iB = ti;
  }
  NLP_STAMP(5);
  const uint32_t* idx = iA;                                        // the E best, in order
  // the elite sequences (the sample blocks' rate-clipped candidates)
  for (int e = tid; e < E * H * 2; e += kBlock) {
    const int r = e / (2 * H), q = e - r * 2 * H;
    eu[e] = ld_wt(&a.cand[2 * (size_t)idx[r] * H + q]);
  }
  __syncthreads();
  NLP_STAMP(6);
  const double c0 = nlp_unkey(kA[0]);
  const double bj0 = ld_wt(&st->best_j);
  const int bit0 = ld_wt(&st->best_it);
  const bool better = c0 < bj0;                     // the best sequence so far (NaN never)
  __syncthreads();                                  // every thread has read best_j
  if (tid < 2 * H) {
    // mean / std over the elite in np.mean(axis=0) / np.std(axis=0)'s order: an axis-0
    // reduction adds the rows in sequence (checked against NumPy), std = sqrt(mean((x - m)^2))
    const int k = tid >> 1, j = tid & 1;
    auto at = [&](int e) { return eu[(2 * (size_t)e * H) + 2 * k + j]; };
    // in row order, eight LDS reads issued ahead of their adds (one read per dependent add
    // waited an LDS round trip per row)
    double acc = 0.0;
    int e = 0;
    for (; e + 8 <= E; e += 8) {
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = at(e + i);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += v[i];
    }
    for (; e < E; ++e) acc += at(e);
    const double m = acc / E;
    double s = 0.0;
    for (e = 0; e + 8 <= E; e += 8) {
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = at(e + i);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double d = v[i] - m;
        s += d * d;
      }
    }
    for (; e < E; ++e) {
      const double d = at(e) - m;
      s += d * d;
    }
    st_wt(&st->mean[k][j], m);
    st_wt(&st->std_[k][j], sqrt(s / E) + a.std_floor);
    if (better) st_wt(&st->best_u[k][j], eu[2 * k + j]);
  }
  // the result (the last round): best objective and round, before this round's update
  const double bj = better ? c0 : bj0;
  const int bit = better ? it : bit0;
  if (tid == 0) {
    if (better) {
      st_wt(&st->best_j, c0);
      st_wt(&st->best_it, it);
    }
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  NLP_STAMP(8);
  if (it == a.iters - 1) nlp_trajectory(a, smem, eu, better, bj, bit);
}

}  // namespace

// ST: the candidates' per-step input terms staged in LDS once per block (pwm, delta, sin /
// cos delta, the input-rate cost term, feasibility: the plan kernel's staged Euler layout,
// [k][c][kStageW]), so the rollout loop reads them instead of forming them per step; when
// 64 x H x 64 B fit beside the rest (H <= kNlpStageH).
constexpr int kNlpStageH = 28;

// s_memrealtime ticks (100 MHz) a block waits for a round's state before it gives up (never
// expected: the solve then reports that its completion tag did not arrive)
constexpr uint64_t kNlpRoundWait = 5000000;

template <bool ST>
__global__ __launch_bounds__(kBlock) void nlp_kernel(NlpLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Scratch sc(smem);
  int* flag = reinterpret_cast<int*>(smem + kFlagOff);
  const int tid = threadIdx.x, H = a.H, blk = (int)blockIdx.x;
  constexpr int LPM = 4, kPerBlock = kBlock / LPM;   // 64 samples per block
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);            // xref [H+1][2]
  double* Ul = sx + 2 * (H + 1);                                            // [64][H][2]
  double* x0 = Ul + 2 * (size_t)kPerBlock * H;                              // [6]
  uint64_t* ks = reinterpret_cast<uint64_t*>(x0 + 6);                       // [64] the samples' keys
  double* ms = reinterpret_cast<double*>(ks + 64);                          // the round's mean, std [2][H][2]
  double* su = ms + 4 * (size_t)H;                                          // ST: [H][64][kStageW]
  int* rflag = flag + 1;                // the round wait's verdict (flag is ticket_last's)
  const NlpState* st = a.st;
  for (int r = 0; r < a.rounds; ++r) {
    const int it = a.it + r;
    if (r > 0) {                        // the previous round's completion published round it
      if (tid == 0) {
        const uint64_t want = tag_word((uint32_t)a.host_seq, (uint32_t)it);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (ld_wt(a.round_tag) != want)
          if (__builtin_amdgcn_s_memrealtime() - t0 > kNlpRoundWait) {
            ok = 0;
            break;
          }
        *rflag = ok;
      }
      __syncthreads();
      if (!*rflag) return;
    }
    NLP_STAMP(0);
    // the round's inputs (the completing block of the previous round used this LDS)
    for (int e = tid; e <= H; e += kBlock) {
      sx[2 * e] = a.xref[e];
      sx[2 * e + 1] = a.xref[(H + 1) + e];
    }
    if (tid < 6) x0[tid] = a.x0[tid];
    for (int e = tid; e < 4 * H; e += kBlock)
      ms[e] = ld_wt(e < 2 * H ? &st->mean[0][0] + e : &st->std_[0][0] + (e - 2 * H));
    __syncthreads();
    // value i = (s H + k) 2 + j of the round; pair i / 2 = (s H + k): the (j = 0, 1) values of
    // one (sample, step) share a Philox call
    for (int e = tid; e < kPerBlock * H; e += kBlock) {
      const int rr = e / H, k = e - rr * H, s = blk * kPerBlock + rr;
      double z0, z1;
      nlp_z2((uint32_t)(s * H + k), a.call, a.seed, (uint32_t)(it + 1), z0, z1);
      Ul[2 * e] = nlp_raw_z(a, ms, it, s, k, 0, z0);
      Ul[2 * e + 1] = nlp_raw_z(a, ms, it, s, k, 1, z1);
    }
    __syncthreads();
    NLP_STAMP(1);
    if (tid < 2 * kPerBlock) {
      const int rr = tid >> 1, j = tid & 1;
      nlp_rate_chain(Ul + 2 * (size_t)rr * H + j, H, j ? a.up1 : a.up0, j ? a.rlo1 : a.rlo0, j ? a.rhi1 : a.rhi0);
    }
    __syncthreads();
    NLP_STAMP(2);
    for (int e = tid; e < kPerBlock * H * 2; e += kBlock) st_wt(&a.cand[(size_t)blk * kPerBlock * 2 * H + e], Ul[e]);
    const fm::FmK K = fm::FmK::load();
    if constexpr (ST) {
      const CostK& q0 = a.la.cost;
      // consecutive threads take consecutive candidates of one step: their 64-B records are
      // adjacent in LDS (one step per thread-row was a 4 KB stride: every write one bank)
      for (int f = tid; f < kPerBlock * H; f += kBlock) {
        const int k = f >> 6, c = f & (kPerBlock - 1), e = c * H + k;
        const double ua = Ul[2 * e], dl = Ul[2 * e + 1];
        double sd, cd;
        if (fm::sincos_fast_ok(dl)) fm::sincos_fast(dl, &sd, &cd, K);
        else LL_SINCOS(dl, &sd, &cd);
        const double p0 = k ? Ul[2 * e - 2] : a.up0, p1 = k ? Ul[2 * e - 1] : a.up1;
        const double d0 = ua - p0, d1 = dl - p1;
        double* o = su + kStageW * (k * kPerBlock + c);
        o[0] = ua;
        o[1] = dl;
        o[2] = sd;
        o[3] = cd;
        o[6] = act_term(q0, d0, d1);
        o[7] = (!q0.enforce || input_feasible(q0, ua, dl, d0, d1)) ? 1.0 : 0.0;
      }
      __syncthreads();
      NLP_STAMP(9);
    }
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
    bool bad = false;
    double J;
    if constexpr (ST)
      J = rollout<1, true, LPM, 0, true>(a.la, c, 0, x0, sx, su, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, bad);
    else
      J = rollout<1, false, LPM, 0, true, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, bad);
    int bi = bad;
    bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
    bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
    if (__builtin_expect(__any(bi), 0)) {
      bool unused = false;
      if (bi) {
        if constexpr (ST)
          J = rollout<1, true, LPM, 0, false>(a.la, c, 0, x0, sx, su, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, unused);
        else
          J = rollout<1, false, LPM, 0, false, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K,
                                                            fq, unused);
      }
    }
    NLP_STAMP(3);
    if (sub == 0) ks[c] = nlp_key(J);
    __syncthreads();
    if (tid < 64) {                     // wave 0: the block's 64 keys sorted (bitonic, in registers)
      uint64_t k = ks[tid];
      uint32_t x = (uint32_t)(blk * kPerBlock + tid);
      for (int w = 2; w <= 64; w <<= 1)
        for (int j = w >> 1; j > 0; j >>= 1) nlp_cx(k, x, j, ((tid & j) == 0) == ((tid & w) == 0));
      const int len = nlp_list_len(a.elite);
      if (tid < len) {
        st_wt(&a.top_key[(size_t)blk * len + tid], k);
        st_wt(&a.top_idx[(size_t)blk * len + tid], x);
      }
    }
    if (!ticket_last(a.ticket, gridDim.x, flag)) continue;
    nlp_complete(a, smem, it);
    if (r + 1 < a.rounds) {             // publish the next round: its state stored sc1, drained
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) st_wt(a.round_tag, tag_word((uint32_t)a.host_seq, (uint32_t)(it + 1)));
    }
  }
}

size_t nlp_lds_bytes(int H, int samples, int elite) {
  const size_t blocks = kScratchBytes + 16 * (size_t)(H + 1) + 16 * 64 * (size_t)H + 48 + 8 * 64 + 32 * (size_t)H +
                        (H <= kNlpStageH ? 8 * kStageW * 64 * (size_t)H : 0);
  const size_t nll = (size_t)(samples / 64) * nlp_list_len(elite);
  const size_t last = kScratchBytes + 24 * nll + 16 * (size_t)elite * H + 16 * (size_t)(H + 1) + 48;
  return std::max(blocks, last);
}

hipError_t launch_nlp(const NlpLaunch& a, hipStream_t s) {
  const size_t lds = std::max<size_t>(nlp_lds_bytes(a.H, a.samples, a.elite), 82 * 1024);
  if (a.H <= kNlpStageH) {
    allow_lds(nlp_kernel<true>);
    hipLaunchKernelGGL(nlp_kernel<true>, dim3(a.samples / 64), dim3(kBlock), lds, s, a);
  } else {
    allow_lds(nlp_kernel<false>);
    hipLaunchKernelGGL(nlp_kernel<false>, dim3(a.samples / 64), dim3(kBlock), lds, s, a);
  }
  return hipGetLastError();
}

}  // namespace llampc
