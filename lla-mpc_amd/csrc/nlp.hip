// nlp.hip — the setupNLP.solve drop-in (llampc_nlp_*, include/llampc.h): the selected model's
// NMPC (nmpc.py:14-203: Euler transcription of Dynamic.casadi, nmpc.py:58-60; the objective
// nmpc.py:44-111; input bounds and the steering-rate bound nmpc.py:102-105) solved on the
// device by the cross-entropy method — no IPOPT here (casadi is absent; its optimum is parity
// unpinned).  Every round in one launch (or one launch per round, nlp.hpp), then the Euler
// trajectory of the best sequence and the result into pinned host memory:
//
//   sample blocks   each draws 64 sequences from the round's (mean, std) — Philox noise
//                   (ctl.hpp), the bounds, the rate chain in order over the horizon; sample 0 is
//                   the mean itself, sample 1 of the first round holds uprev — and rolls them out
//                   (the plan kernel's rollout, NLP-Euler, four lanes per rollout, candidates in
//                   LDS), writing each sample's objective (+inf if infeasible).  Each block then
//                   sorts its 64 (objective, index) keys in one wave (a bitonic network of
//                   shuffle exchanges: NaN last, ties to the lower index) and publishes its best
//                   len = next_pow2(E) sorted, as tagged words;
//   every block     then completes the round itself (round 6; until then one completion block
//                   did and handed the next mean / std back through tagged words, ~1.5 us a
//                   round), in registers where it can (E <= 32, nlp_complete32): waves 0-3 each
//                   poll four blocks' lists straight into registers and merge them two levels
//                   in the wave — the lower len of two sorted lists is min(a_i, b_(len-1-i)),
//                   bitonic, then one half-cleaner network of lane exchanges per level — and
//                   hand wave 0 the result through LDS (a counter, no block barrier), which
//                   merges those the same way to the E best overall in order, loads the E elite
//                   sequences (32 loads in flight per lane) and sets the next mean / std as
//                   their mean / standard deviation (NumPy's axis-0 order).  Every block
//                   computes the same values in the same order, so all hold the same next
//                   distribution.  Block 0 keeps the state (the best sequence so far) and
//                   writes the result.  The lists and the sequences are double-buffered by
//                   round parity: a block can be a round ahead of another, never two.  The next
//                   round's Philox variates (they do not depend on the mean / std) are drawn by
//                   helper waves 5-7 while waves 0-3 complete the round.  (A bitonic sort
//                   of all samples in LDS took 36 us of the 62 us round: 55 barrier-separated
//                   passes; the barrier-separated merge tree of round 6's first version 2.5 us.)
#include "plan_dev.hpp"
#include "nlp.hpp"

namespace llampc {

#ifdef LLAMPC_STAMPS
// Diagnostic build only: s_memrealtime per block and phase of the last launch
// (tools/diag/nlp_phases.py): 0 round start, 10 mean / std in, 1 samples formed, 2 rate-clipped,
// 9 staged, 3 wave 0's rollouts done, 12 every wave's, 11 list published; the completion (wave
// 0): 4 its four lists in and merged, 13 every group in, 5 merged, 6 elite loads issued, 14 the
// elite mean, 8 next mean / std.
static __device__ unsigned long long g_nlp_ph[32][16];
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

// s_memrealtime ticks (100 MHz) a block waits for a round's state before it gives up (never
// expected: the solve then reports that its completion tag did not arrive)
constexpr uint64_t kNlpRoundWait = 5000000;

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
// sampler applies it); lo > hi: no rate bound on this input.  Eight steps at a time in
// registers: their LDS reads issue together.  A batch free of NaN (every one unless the mean /
// std is NaN) takes np_clip's non-NaN branch as plain compare-selects: the NaN tests' lane-mask
// logic (vector compares combined in the scalar unit) was most of each step's dependent chain.
// (Forming the samples inside this pass too, on its two waves instead of the block's four,
// measured 3.8 us against 1.8 + 1.7 us split.)
__device__ __forceinline__ void nlp_rate_chain(double* u, int H, double up, double lo, double hi) {
#pragma clang fp contract(off)
  if (!(lo <= hi)) return;
  double prev = up;
  int k0 = 0;
  for (; k0 + 8 <= H; k0 += 8) {
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = u[2 * (k0 + i)];
    bool fin = prev == prev;
#pragma unroll
    for (int i = 0; i < 8; ++i) fin = fin && v[i] == v[i];
    if (fin) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double a = prev + lo, b = prev + hi;
        const double y = v[i] > a ? v[i] : a;
        prev = y < b ? y : b;
        v[i] = prev;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        prev = np_clip(v[i], prev + lo, prev + hi);
        v[i] = prev;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) u[2 * (k0 + i)] = v[i];
  }
  for (; k0 < H; ++k0) {
    prev = np_clip(u[2 * k0], prev + lo, prev + hi);
    u[2 * k0] = prev;
  }
}

// e / d for 0 <= e < 2^16, 1 <= d <= 2^8, without the integer division's software sequence:
// (e + 1/2) / d is at least 1 / (2 d) from an integer, far beyond the float product's error
__device__ __forceinline__ int nlp_div(int e, float rd) { return (int)(((float)e + 0.5f) * rd); }

// order-preserving key of an objective: NaN above +inf (a diverged rollout sorts last)
__device__ __forceinline__ uint64_t nlp_key(double v) {
  const double w = (v != v) ? __builtin_nan("") : v + 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(w);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double nlp_unkey(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k));
}

// a block-uniform double held in scalar registers (the best so far lives across the rollouts)
__device__ __forceinline__ double nlp_uni(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// lane ^ J's value, in VALU ops only: DPP quad_perm for J = 1, 2, DPP row shifts for J = 4 (left
// or right by the lane's bit 2), DPP row_ror:8 for J = 8, and gfx950's v_permlane16_swap /
// v_permlane32_swap for J = 16, 32 (the swap's two results; the lane's bit picks).  ds_swizzle
// and ds_bpermute (LDS-pipe round trips) made every step of the block sort and the merges an
// LDS-latency chain: the 21-step sort of 64 keys took ~1 us.
template <int J>
__device__ __forceinline__ uint32_t nlp_xor32(uint32_t v) {
  static_assert(J >= 1 && J <= 32 && (J & (J - 1)) == 0, "a power of two below the wave size");
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  } else if constexpr (J == 4) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xF, 0xF, false);   // row_shl:4
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    return (__lane_id() & 4) ? dn : up;
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);                       // row_ror:8
  } else if constexpr (J == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (__lane_id() & 16) ? p[0] : p[1];
  } else {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() & 32) ? p[0] : p[1];
  }
}

// (key, index) exchange step of a bitonic network across lanes lane ^ J: the lane keeps the
// smaller pair when `low`, else the larger (indices are distinct, so the order is total)
template <int J>
__device__ __forceinline__ void nlp_cx(uint64_t& k, uint32_t& i, bool low) {
  const uint64_t pk = ((uint64_t)nlp_xor32<J>((uint32_t)(k >> 32)) << 32) | nlp_xor32<J>((uint32_t)k);
  const uint32_t pi = nlp_xor32<J>(i);
  const bool pless = pk < k || (pk == k && pi < i);
  if (low == pless) {
    k = pk;
    i = pi;
  }
}

// the half-cleaner steps J, J / 2, .., 1 of a bitonic merge of blocks of W lanes
// (W = 0: the merge tree's, each lane keeping the lower when its bit J is clear)
template <int W, int J>
__device__ __forceinline__ void nlp_clean(uint64_t& k, uint32_t& i, int lane) {
  nlp_cx<J>(k, i, W ? (((lane & J) == 0) == ((lane & W) == 0)) : ((lane & J) == 0));
  if constexpr (J > 1) nlp_clean<W, J / 2>(k, i, lane);
}

// the wave's 64 (key, index) pairs sorted ascending across the lanes (bitonic)
template <int W = 2>
__device__ __forceinline__ void nlp_sort64(uint64_t& k, uint32_t& i, int lane) {
  nlp_clean<W, W / 2>(k, i, lane);
  if constexpr (W < 64) nlp_sort64<2 * W>(k, i, lane);
}

// a bitonic sequence of len lanes (a group inside the wave) sorted ascending
__device__ __forceinline__ void nlp_clean_len(uint64_t& k, uint32_t& i, int lane, int len) {
  switch (len) {                        // block-uniform
    case 64: nlp_clean<0, 32>(k, i, lane); break;
    case 32: nlp_clean<0, 16>(k, i, lane); break;
    case 16: nlp_clean<0, 8>(k, i, lane); break;
    case 8: nlp_clean<0, 4>(k, i, lane); break;
    case 4: nlp_clean<0, 2>(k, i, lane); break;
    case 2: nlp_clean<0, 1>(k, i, lane); break;
    default: break;
  }
}

__device__ __forceinline__ void nlp_traj_quad(const NlpLaunch& a, const double* sx, const double* ub, const double* x0);

// xmpc (nmpc.py:58-60): the NLP's Euler trajectory of the best sequence over all rounds, by
// one quad of the completing block (the sample blocks' fast rollout, the general re-run when
// its domain check fails) — it was a separate one-lane launch of the general evaluation, 32 us.
// The block that writes the result: the best sample's if it is from the last round (its states
// are in that block's LDS), else block 0.
__device__ __forceinline__ int nlp_owner(const NlpLaunch& a, int bit, int bs) {
  return a.ltraj && bit == a.iters - 1 ? bs / 64 : 0;
}

// sx, x0: the block's LDS copies of the solve's xref [H+1][2] and x0 [6] (nlp_kernel).
// trl: the block's LDS states of its samples' rollouts in the solve's last round (NlpLaunch.ltraj)
// — a best from that round is written by its own block, from there; an earlier round's best by
// block 0, re-running its rollout.
// bu: the block's LDS copy of the best sequence so far.
__device__ __forceinline__ void nlp_trajectory(const NlpLaunch& a, double* bu, double bj, int bit, int bs, int it,
                                               const double* trl, const double* sx, const double* x0) {
  const int tid = threadIdx.x, H = a.H;
  NlpResult* res = a.res;
  __syncthreads();                      // bu is final
  for (int e = tid; e < 2 * H; e += (int)blockDim.x) {
    const double v = bit < 0 ? 0.0 : bu[e];   // none: no finite objective, the result's zeros
    bu[e] = v;
    (&res->best_u[0][0])[e] = v;
  }
  if (tid == 0) {
    res->best_j = bj;
    res->best_it = bit;
  }
  if (a.ltraj && bit == it) {
    const double* src = trl + (size_t)(bs & 63) * 6 * H;
    for (int e = tid; e < 6 * (H + 1); e += (int)blockDim.x) (&res->traj[0][0])[e] = e < 6 ? x0[e] : src[e - 6];
  } else {
    __syncthreads();
    if (tid < 4) nlp_traj_quad(a, sx, bu, x0);
  }
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

// A round's lists and sequences, double-buffered by round parity (every block completes every
// round, so a block may run one round ahead of another — never two: round r + 2's stores follow
// the writer's completion of round r + 1, which needs every block's list of round r + 1, which
// each block publishes only after it has read round r's buffers).
__device__ __forceinline__ uint64_t* nlp_lists(const NlpLaunch& a, int it) {
  return a.list_tag + (size_t)(it & 1) * 3 * (size_t)a.samples;
}
__device__ __forceinline__ double* nlp_cand(const NlpLaunch& a, int it) {
  return a.cand + (size_t)(it & 1) * 2 * (size_t)a.samples * a.H;
}

// The completion's LDS (every block): the lists' keys kA | kB and indices iA | iB ([m] each: the
// merge tree's two buffers, or nlp_complete32's wave results), then the elite sequences [E][H][2]
// (nlp_complete32: row 0 only, the trajectory's).
struct NlpCompLds {
  uint64_t *kA, *kB;
  uint32_t *iA, *iB;
  double* eu;
};
__host__ __device__ __forceinline__ int nlp_comp_m(int nl, int len) {
  const int ng = (nl + 3) >> 2, m32 = 32 * (ng + ((ng + 3) >> 2));   // nlp_complete32's two levels
  return nl * len > m32 ? nl * len : m32;
}
__device__ __forceinline__ NlpCompLds nlp_comp_lds(unsigned char* base, int nl, int len) {
  const size_t m = (size_t)nlp_comp_m(nl, len);
  NlpCompLds L;
  L.kA = reinterpret_cast<uint64_t*>(base);
  L.kB = L.kA + m;
  L.iA = reinterpret_cast<uint32_t*>(L.kB + m);
  L.iB = L.iA + m;
  L.eu = reinterpret_cast<double*>(base + 24 * m);
  return L;
}
// its bytes: the lists, the elite rows, and the trajectory's reference and x0 after them
__host__ __device__ __forceinline__ size_t nlp_comp_bytes(int H, int nl, int elite) {
  return 24 * (size_t)nlp_comp_m(nl, nlp_list_len(elite)) + 16 * (size_t)elite * H + 16 * (size_t)(H + 1) + 48;
}

// Waits (bounded) for tagged words; returns the block's verdict (every thread the same).
__device__ __forceinline__ bool nlp_block_ok(int ok, int* rflag) {
  if (threadIdx.x == 0) *rflag = 1;
  __syncthreads();
  if (!ok) *rflag = 0;
  __syncthreads();
  return *rflag != 0;
}

// The completion block: every sample block's sorted list of the round (tag sq) into kA / iA.
__device__ __forceinline__ bool nlp_poll_lists(const NlpLaunch& a, const NlpCompLds& L, int nl, int it, uint32_t sq,
                                               int* rflag) {
  const int nbl = nl * nlp_list_len(a.elite);
  const uint64_t* lt = nlp_lists(a, it);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  int ok = 1;
  for (int e = threadIdx.x; e < nbl && ok; e += (int)blockDim.x) {
    for (;;) {
      const uint64_t hi = ld_wt(&lt[e]), lo = ld_wt(&lt[nbl + e]), ix = ld_wt(&lt[2 * nbl + e]);
      if ((int)tag_ok(hi, sq) & (int)tag_ok(lo, sq) & (int)tag_ok(ix, sq)) {
        L.kA[e] = join_words(hi, lo);
        L.iA[e] = (uint32_t)ix;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > kNlpRoundWait) {
        ok = 0;
        break;
      }
    }
  }
  return nlp_block_ok(ok, rflag);
}

// Round `it`'s completion, run by every block (the lists in kA / iA): the elite, the next mean /
// std into ms (this block's LDS: every block computes the same), the best so far.  Block 0 alone
// writes the state and, on the solve's last round, the result; on a launch's last round it also
// publishes the next mean / std as tagged words for the next launch (one launch per round).
// bj / bit: the best objective so far and its round, carried in registers across the launch's
// rounds; stored to the state too, for the next launch.
__device__ __forceinline__ void nlp_complete(const NlpLaunch& a, unsigned char* cbase, int it, int nl, double& bjv,
                                             int& bitv, int& bsv, double* ms, double* bu, bool last_of_launch,
                                             const double* trl, const double* sx, const double* x0) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, H = a.H, E = a.elite;
  const int len = nlp_list_len(E);
  const bool b0 = blockIdx.x == 0;
  const NlpCompLds L = nlp_comp_lds(cbase, nl, len);
  uint64_t* kA = L.kA;
  uint64_t* kB = L.kB;
  uint32_t* iA = L.iA;
  uint32_t* iB = L.iB;
  double* eu = L.eu;                                                  // [E][H][2]
  // merge tree: lists 2g, 2g + 1 -> list g; a group of len lanes (inside one wave) per pair
  for (int n = nl; n > 1; n >>= 1) {
    const int pairs = n >> 1, gpp = (int)blockDim.x / len, i = tid & (len - 1);
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
        nlp_clean_len(k, x, i, len);
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
  // the elite sequences (the sample blocks' rate-clipped candidates of this round's buffer)
  const double* cand = nlp_cand(a, it);
  for (int e = tid; e < E * H * 2; e += (int)blockDim.x) {
    const int r = e / (2 * H), q = e - r * 2 * H;
    eu[e] = ld_wt(&cand[2 * (size_t)idx[r] * H + q]);
  }
  __syncthreads();
  NLP_STAMP(6);
  const double c0 = nlp_unkey(kA[0]);
  const double bj0 = bjv;
  const int bit0 = bitv, bs0 = bsv;
  const bool better = c0 < bj0;                     // the best sequence so far (NaN never)
  double* msn = ms;
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
    const double sd = sqrt(s / E) + a.std_floor;
    const int im = 2 * k + j, is = 2 * H + 2 * k + j;
    if (it + 1 < a.iters) {             // the next round's mean / std
      if (b0 && last_of_launch) {       // into the next launch: tagged halves (low, high)
        const uint32_t sq1 = nlp_seq(a.host_seq, it + 1);
        const uint64_t mb = (uint64_t)__double_as_longlong(m);
        const uint64_t sb = (uint64_t)__double_as_longlong(sd);
        st_wt(&a.ms_tag[2 * im], tag_word(sq1, (uint32_t)mb));
        st_wt(&a.ms_tag[2 * im + 1], tag_word(sq1, (uint32_t)(mb >> 32)));
        st_wt(&a.ms_tag[2 * is], tag_word(sq1, (uint32_t)sb));
        st_wt(&a.ms_tag[2 * is + 1], tag_word(sq1, (uint32_t)(sb >> 32)));
      }
    }
    if (better) bu[2 * k + j] = eu[2 * k + j];   // this block's copy of the best so far
    msn[im] = m;                        // this block's copy (ms is read again only after a barrier)
    msn[is] = sd;
  }
  // the result (the last round): best objective and round, before this round's update
  const double bj = better ? c0 : bj0;
  const int bit = better ? it : bit0;
  const int bs = better ? (int)idx[0] : bs0;
  bjv = nlp_uni(bj);
  bitv = __builtin_amdgcn_readfirstlane(bit);
  bsv = __builtin_amdgcn_readfirstlane(bs);
  NLP_STAMP(8);
  if (it == a.iters - 1 && (int)blockIdx.x == nlp_owner(a, bit, bs)) nlp_trajectory(a, bu, bj, bit, bs, it, trl, sx, x0);
  __syncthreads();                      // ms (the next round's) and the LDS lists (the next poll)
}

// LDS words of nlp_complete32's hand-off between its waves (the scratch's pad, plan_dev.hpp
// kScratchBytes): the Phase-A waves done (counted over the launch's rounds), a poll that timed
// out, the round's best key and its sample.
constexpr int kNlpDoneOff = 176, kNlpFailOff = 180, kNlpBestOff = 184, kNlpBestSOff = 164;
constexpr int kNlpMergeWaves = 4;       // waves 0-3 poll and merge (5-7 draw, ST)

__device__ __forceinline__ bool nlp_less(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
  return ka < kb || (ka == kb && ia < ib);
}

// Four sorted lists of at most 32 -> their 32 smallest (key, index) pairs, ascending, in lanes
// 0-31.  On entry lane i of half h (i = lane & 31, h = lane >> 5) holds (ka, ia) = entry i of
// list 2h and (kb, ib) = entry 31 - i of list 2h + 1 (pads: all ones, after every real pair).
// min(a_i, b_(31-i)) is bitonic and holds the two lists' 32 smallest; a half-cleaner sorts each
// half; then each lane against lane ^ 63 (lane i < 32 meets the other half's 31 - i) the same way.
__device__ __forceinline__ void nlp_merge4(uint64_t& ka, uint32_t& ia, uint64_t kb, uint32_t ib, int lane) {
  if (nlp_less(kb, ib, ka, ia)) {
    ka = kb;
    ia = ib;
  }
  nlp_clean<0, 16>(ka, ia, lane);
  // lane ^ 63 = ((lane ^ 15) ^ 16) ^ 32: row_mirror, then the two swaps
  auto x63 = [](uint32_t v) {
    return nlp_xor32<32>(nlp_xor32<16>((uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false)));
  };
  const uint64_t pk = ((uint64_t)x63((uint32_t)(ka >> 32)) << 32) | x63((uint32_t)ka);
  const uint32_t pi = x63(ia);
  if (nlp_less(pk, pi, ka, ia)) {
    ka = pk;
    ia = pi;
  }
  nlp_clean<0, 16>(ka, ia, lane);
}

// entry e of a round's lists, polled until its words carry the round's tag; false: timed out
__device__ __forceinline__ bool nlp_poll2(const uint64_t* lt, int nbl, int ea, int eb, uint32_t sq, uint64_t& ka,
                                          uint32_t& ia, uint64_t& kb, uint32_t& ib) {
  bool ra = ea < 0, rb = eb < 0;        // < 0: a pad
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (!ra) {
      const uint64_t hi = ld_wt(&lt[ea]), lo = ld_wt(&lt[nbl + ea]), ix = ld_wt(&lt[2 * nbl + ea]);
      if ((int)tag_ok(hi, sq) & (int)tag_ok(lo, sq) & (int)tag_ok(ix, sq)) {
        ka = join_words(hi, lo);
        ia = (uint32_t)ix;
        ra = true;
      }
    }
    if (!rb) {
      const uint64_t hi = ld_wt(&lt[eb]), lo = ld_wt(&lt[nbl + eb]), ix = ld_wt(&lt[2 * nbl + eb]);
      if ((int)tag_ok(hi, sq) & (int)tag_ok(lo, sq) & (int)tag_ok(ix, sq)) {
        kb = join_words(hi, lo);
        ib = (uint32_t)ix;
        rb = true;
      }
    }
    if (ra && rb) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > kNlpRoundWait) return false;
  }
}

// Round `it`'s completion for len <= 32 (E <= 32), run by every block after its list is
// published.  Phase A, waves 0-3: each polls groups of four lists into registers and merges them
// (nlp_merge4) into the group's 32 best, written to LDS.  Phase B, wave 0: merges the groups'
// lists up the same way, loads the E elite rows (32 loads per lane in flight together) and forms
// the next mean / std in NumPy's order.  The other waves are free (helpers 5-7 draw the next round's variates).  Ends
// with the block's barrier; returns false if a poll timed out (every thread the same).
// (Phase A's waves loading their groups' 32 best rows into LDS beside Phase B measured slower:
// four times the bytes through the one CU, 1.8 us against 1.0 for wave 0's own loads.)
__device__ __forceinline__ bool nlp_complete32(const NlpLaunch& a, unsigned char* smem, unsigned char* cbase, int it,
                                               int r, int nl, double& bjv, int& bitv, int& bsv, double* ms,
                                               double* bu, bool last_of_launch, const double* trl,
                                               const double* sx, const double* x0) {
#pragma clang fp contract(off)
  // an opaque copy of the thread index: the lane arithmetic below stays here instead of being
  // hoisted out of the round loop, where it would live across the rollouts (VGPR spills)
  int tid = (int)threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6, h = lane >> 5, i = lane & 31;
  const int H = a.H, E = a.elite, len = nlp_list_len(E), nbl = nl * len, H2 = 2 * H;
  const bool b0 = blockIdx.x == 0;
  int* done = reinterpret_cast<int*>(smem + kNlpDoneOff);
  int* fail = reinterpret_cast<int*>(smem + kNlpFailOff);
  uint64_t* bestk = reinterpret_cast<uint64_t*>(smem + kNlpBestOff);
  int* bests = reinterpret_cast<int*>(smem + kNlpBestSOff);
  const NlpCompLds L = nlp_comp_lds(cbase, nl, len);
  const double* cand = nlp_cand(a, it);
  const int ng = (nl + 3) >> 2, nact = ng < kNlpMergeWaves ? ng : kNlpMergeWaves;
  if (w < nact) {                       // Phase A
    const uint64_t* lt = nlp_lists(a, it);
    bool ok = true;
    for (int g = w; g < ng; g += nact) {
      const int la = 4 * g + 2 * h, lb = la + 1;
      uint64_t ka = ~0ull, kb = ~0ull;
      uint32_t ia = ~0u, ib = ~0u;
      ok = ok && nlp_poll2(lt, nbl, la < nl && i < len ? la * len + i : -1,
                           lb < nl && 31 - i < len ? lb * len + 31 - i : -1, nlp_seq(a.host_seq, it), ka, ia, kb, ib);
      nlp_merge4(ka, ia, kb, ib, lane);
      if (h == 0) {
        L.kA[g * 32 + i] = ka;
        L.iA[g * 32 + i] = ia;
      }
    }
    if (!ok) *fail = 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  NLP_STAMP(4);
  if (w == 0) {                         // Phase B, the elite, the next mean / std
    while (__hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < (r + 1) * nact)
      __builtin_amdgcn_s_sleep(1);
    NLP_STAMP(13);
    if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      uint64_t fk = ~0ull;
      uint32_t fi = ~0u;
      uint64_t *sk = L.kA, *dk = L.kB;
      uint32_t *si = L.iA, *di = L.iB;
      for (int cnt = ng;;) {             // wave-uniform
        const int ng2 = (cnt + 3) >> 2;
        for (int g = 0; g < ng2; ++g) {
          const int la = 4 * g + 2 * h, lb = la + 1;
          uint64_t ka = la < cnt ? sk[la * 32 + i] : ~0ull, kb = lb < cnt ? sk[lb * 32 + 31 - i] : ~0ull;
          uint32_t ia = la < cnt ? si[la * 32 + i] : ~0u, ib = lb < cnt ? si[lb * 32 + 31 - i] : ~0u;
          nlp_merge4(ka, ia, kb, ib, lane);
          if (h == 0) {
            dk[g * 32 + i] = ka;
            di[g * 32 + i] = ia;
          }
          fk = ka;
          fi = ia;
        }
        if (ng2 == 1) break;
        uint64_t* tk = sk;
        sk = dk;
        dk = tk;
        uint32_t* ti = si;
        si = di;
        di = ti;
        cnt = ng2;
      }
      NLP_STAMP(5);
      // lanes 0..E-1 hold the E best in order; the elite rows (this round's rate-clipped
      // candidates), a column q = 2 k + j per lane
      const uint64_t k0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fk >> 32), 0) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fk, 0);
      const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)fi, 0);
      const double c0 = nlp_unkey(k0);
      const bool better = c0 < bjv;     // the best sequence so far (NaN never)
      // the rows past E read row 0's (their values are not used); E through an opaque copy, so
      // that its 32 comparisons stay here instead of being hoisted out of the round loop
      int Eo = E;
      asm volatile("" : "+s"(Eo));
      // each lane its row's offset (one multiply for all 32), then one read-lane per load
      const uint32_t ro = (lane < Eo ? fi : s0) * (uint32_t)H2;
      for (int q0 = 0; q0 < H2; q0 += 64) {
        const int q = q0 + lane;
        const bool act = q < H2;
        // straight-line loads, all in flight together (the lanes past the columns read the last)
        const double* col = cand + (act ? q : H2 - 1);
        double v[32];
#pragma unroll
        for (int e = 0; e < 32; ++e) v[e] = ld_wt(col + (uint32_t)__builtin_amdgcn_readlane((int)ro, e));
        NLP_STAMP(6);
        // np.mean / np.std over axis 0: the rows added in sequence, std = sqrt(mean((x - m)^2))
        double acc = 0.0;
#pragma unroll
        for (int e = 0; e < 32; ++e) acc = e < Eo ? acc + v[e] : acc;
        const double m = acc / E;
        NLP_STAMP(14);
        double sv = 0.0;
#pragma unroll
        for (int e = 0; e < 32; ++e) {
          const double d = v[e] - m;
          sv = e < Eo ? sv + d * d : sv;
        }
        const double sd = sqrt(sv / E) + a.std_floor;
        if (act) {
          const int im = q, is = H2 + q;
          if (it + 1 < a.iters && b0 && last_of_launch) {   // into the next launch (tagged halves)
            const uint32_t sq1 = nlp_seq(a.host_seq, it + 1);
            const uint64_t mb = (uint64_t)__double_as_longlong(m);
            const uint64_t sb = (uint64_t)__double_as_longlong(sd);
            st_wt(&a.ms_tag[2 * im], tag_word(sq1, (uint32_t)mb));
            st_wt(&a.ms_tag[2 * im + 1], tag_word(sq1, (uint32_t)(mb >> 32)));
            st_wt(&a.ms_tag[2 * is], tag_word(sq1, (uint32_t)sb));
            st_wt(&a.ms_tag[2 * is + 1], tag_word(sq1, (uint32_t)(sb >> 32)));
          }
          if (better) bu[q] = v[0];     // this block's copy of the best so far
          ms[im] = m;                   // read by the next round after the barrier below
          ms[is] = sd;
        }
      }
      if (lane == 0) {
        *bestk = k0;
        *bests = (int)s0;
      }
      NLP_STAMP(8);
    }
  }
  __syncthreads();
  if (*fail) return false;
  const double c0 = nlp_unkey(*bestk);
  const double bj0 = bjv;
  const int bit0 = bitv;
  const bool better = c0 < bj0;
  bjv = nlp_uni(better ? c0 : bj0);
  bitv = __builtin_amdgcn_readfirstlane(better ? it : bit0);
  bsv = __builtin_amdgcn_readfirstlane(better ? *bests : bsv);
  // the result by the block of the best sample (its states are this block's)
  if (it == a.iters - 1 && (int)blockIdx.x == nlp_owner(a, bitv, bsv))
    nlp_trajectory(a, bu, bjv, bitv, bsv, it, trl, sx, x0);
  return true;
}

}  // namespace

// ST: the candidates' per-step input terms staged in LDS once per block (pwm, delta, sin /
// cos delta, the input-rate cost term, feasibility: the plan kernel's staged Euler layout,
// [k][c][kNlpStageW]), so the rollout loop reads them instead of forming them per step; when
// 64 x H x 64 B fit beside the rest (H <= kNlpStageH).
constexpr int kNlpStageH = 28;
constexpr int kNlpStageW = 6;           // the compact Euler record: a, delta, sin, cos, act, feasible

// The round's Philox variates z of this block's samples into Ul (sample rr's row at rr us, its
// value (k, j) at 2 k + j; the pair (s H + k) shares one call): independent of the round's mean /
// std, so a block draws the next round's while it completes this one.
__device__ __forceinline__ void nlp_draw(const NlpLaunch& a, int blk, int it, double* Ul, int us, int t0, int stride) {
  constexpr int kPerBlock = 64;
  const int H = a.H;
  const float rH = 1.0f / (float)H;
  for (int e = t0; e < kPerBlock * H; e += stride) {
    const int rr = nlp_div(e, rH), k = e - rr * H, s = blk * kPerBlock + rr;
    double z0, z1;
    nlp_z2((uint32_t)(s * H + k), a.call, a.seed, (uint32_t)(it + 1), z0, z1);
    Ul[rr * us + 2 * k] = z0;
    Ul[rr * us + 2 * k + 1] = z1;
  }
}

// The sample block's LDS after the scratch: xref [H+1][2] | Ul [64][us] (us = 2 H + 1 staged,
// an odd row stride in doubles: the rate chain's and the staging's row-per-lane accesses are
// then free of bank conflicts; 2 H unstaged, the rollouts' layout) | x0 [6] | keys [64] | mean /
// std [2][H][2] | the best sequence so far [H][2] | ST: the staged terms [H][64][kNlpStageW] — the completion's region
// (nlp_comp_bytes) reuses them once the rollouts are done — else the completion's region |
// ltraj: the samples' rollout states [64][H][6] (nlp_traj_off).
__host__ __device__ __forceinline__ size_t nlp_su_off(int H) {
  return kScratchBytes + 16 * (size_t)(H + 1) + 8 * 64 * (2 * (size_t)H + 1) + 48 + 8 * 64 + 48 * (size_t)H;
}
// ltraj: the samples' rollout states [64][H][6] after the staged terms / the completion's region
__host__ __device__ __forceinline__ size_t nlp_traj_off(int H, int nl, int elite) {
  const size_t su = H <= kNlpStageH ? 8 * kNlpStageW * 64 * (size_t)H : 0, cb = nlp_comp_bytes(H, nl, elite);
  return nlp_su_off(H) + (su > cb ? su : cb);
}

// NT threads: the rollouts take the first 256 (a quad per sample); the other waves share the
// blocks' per-round loops (bounds, staging, the completion) and draw the next round's variates
// while the rollouts run (ST), two waves per SIMD
template <bool ST, int NT>
__global__ __launch_bounds__(NT) void nlp_kernel(NlpLaunch a, NlpInline pk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* rflag = reinterpret_cast<int*>(smem + kFlagOff);   // a bounded wait's block verdict
  const int tid = threadIdx.x, H = a.H, blk = (int)blockIdx.x;
  const int nl = (int)gridDim.x;        // every block samples, every block completes every round
  constexpr int LPM = 4, kPerBlock = 64;             // 64 samples per block, a quad each
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);            // xref [H+1][2]
  const int us = ST ? 2 * H + 1 : 2 * H;                                    // Ul's row stride
  double* Ul = sx + 2 * (H + 1);                                            // [64][us]
  double* x0 = Ul + (size_t)kPerBlock * us;                                 // [6]
  uint64_t* ks = reinterpret_cast<uint64_t*>(x0 + 6);                       // [64] the samples' keys
  double* ms = reinterpret_cast<double*>(ks + 64);                          // the round's mean, std [2][H][2]
  double* bu = ms + 4 * H;                                                  // the best sequence so far [H][2]
  double* su = reinterpret_cast<double*>(smem + nlp_su_off(H));             // ST: [H][64][kNlpStageW]
  unsigned char* cbase = smem + nlp_su_off(H);                              // the completion's region
  double* trl = reinterpret_cast<double*>(smem + nlp_traj_off(H, nl, a.elite));   // ltraj: [64][H][6]
  NlpState* st = a.st;
  const int len = nlp_list_len(a.elite), nbl = nl * len;
  const double* xin = pk.v;             // the inputs in the kernarg segment (NlpInline)
  const double* mean0 = pk.v + 6 + 2 * (H + 1);
  if (tid == 0) {
    *reinterpret_cast<int*>(smem + kNlpDoneOff) = 0;
    *reinterpret_cast<int*>(smem + kNlpFailOff) = 0;
  }
  for (int e = tid; e <= H; e += NT) {   // the solve's inputs (this block's LDS only)
    sx[2 * e] = xin[6 + e];
    sx[2 * e + 1] = xin[6 + (H + 1) + e];
  }
  if (tid < 6) x0[tid] = xin[tid];
  nlp_draw(a, blk, a.it, Ul, us, tid, NT);   // the first round's variates
  // the best so far as the launch starts (none, or an earlier launch's rounds)
  double bjv = nlp_uni(a.it == 0 ? HUGE_VAL : ld_wt(&st->best_j));
  int bitv = __builtin_amdgcn_readfirstlane(a.it == 0 ? -1 : ld_wt(&st->best_it));
  int bsv = __builtin_amdgcn_readfirstlane(a.it == 0 ? -1 : ld_wt(&st->best_s));
  if (a.it > 0)
    for (int e = tid; e < 2 * H; e += NT) bu[e] = ld_wt(&st->best_u[0][0] + e);
  for (int r = 0; r < a.rounds; ++r) {
    const int it = a.it + r;
    const uint32_t sq = nlp_seq(a.host_seq, it);
    NLP_STAMP(0);
    // the round's mean / std: the launch's inputs (round 0: mean0, sigma0), this block's
    // completion of the previous round (in ms already), or — a launch's first round after round
    // 0 — the previous launch's block 0's tagged halves
    if (it == 0) {
      for (int e = tid; e < 4 * H; e += NT) ms[e] = e < 2 * H ? mean0[e] : (e & 1) ? a.sig1 : a.sig0;
    } else if (r == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int ok = 1;
      for (int i = tid; i < 4 * H && ok; i += NT) {
        for (;;) {
          const uint64_t lo = ld_wt(&a.ms_tag[2 * i]), hi = ld_wt(&a.ms_tag[2 * i + 1]);
          if ((int)tag_ok(lo, sq) & (int)tag_ok(hi, sq)) {
            ms[i] = __longlong_as_double((long long)join_words(hi, lo));
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > kNlpRoundWait) {
            ok = 0;
            break;
          }
        }
      }
      if (!nlp_block_ok(ok, rflag)) return;
    }
    __syncthreads();
    NLP_STAMP(10);
    // the samples from their variates (drawn ahead): the bounds
    const float rH = 1.0f / (float)H;
    for (int e = tid; e < kPerBlock * H; e += NT) {
      const int rr = nlp_div(e, rH), k = e - rr * H, s = blk * kPerBlock + rr;
      double* u = Ul + rr * us + 2 * k;
      u[0] = nlp_raw_z(a, ms, it, s, k, 0, u[0]);
      u[1] = nlp_raw_z(a, ms, it, s, k, 1, u[1]);
    }
    __syncthreads();
    NLP_STAMP(1);
    if (tid < 2 * kPerBlock) {
      const int rr = tid >> 1, j = tid & 1;
      nlp_rate_chain(Ul + rr * us + j, H, j ? a.up1 : a.up0, j ? a.rlo1 : a.rlo0, j ? a.rhi1 : a.rhi0);
    }
    __syncthreads();
    NLP_STAMP(2);
    // the rate-clipped sequences for every block's elite read (each wave drains these stores
    // before its list is published, below): staged, by the helper waves during the rollouts
    // (stored here, by every wave, they took ~1.5 us of the round); unstaged, here
    double* cand = nlp_cand(a, it);
    auto store_cand = [&](int t0, int stride) {
      for (int e = t0; e < kPerBlock * H * 2; e += stride) {
        const int rr = nlp_div(e, 0.5f * rH);
        st_wt(&cand[(size_t)blk * kPerBlock * 2 * H + e], Ul[e + rr * (us - 2 * H)]);
      }
    };
    if constexpr (!ST) store_cand(tid, NT);
    NLP_STAMP(15);
    const fm::FmK K = fm::FmK::load();
    if constexpr (ST) {
      const CostK& q0 = a.la.cost;
      // consecutive threads take consecutive candidates of one step: their 64-B records are
      // adjacent in LDS (one step per thread-row was a 4 KB stride: every write one bank)
      for (int f = tid; f < kPerBlock * H; f += NT) {
        const int k = f >> 6, c = f & (kPerBlock - 1);
        const double* u = Ul + c * us + 2 * k;
        const double ua = u[0], dl = u[1];
        double sd, cd;
        if (fm::sincos_fast_ok(dl)) fm::sincos_fast(dl, &sd, &cd, K);
        else LL_SINCOS(dl, &sd, &cd);
        const double p0 = k ? u[-2] : a.up0, p1 = k ? u[-1] : a.up1;
        const double d0 = ua - p0, d1 = dl - p1;
        double* o = su + kNlpStageW * (k * kPerBlock + c);
        o[0] = ua;
        o[1] = dl;
        o[2] = sd;
        o[3] = cd;
        o[4] = act_term(q0, d0, d1);
        o[5] = (!q0.enforce || input_feasible(q0, ua, dl, d0, d1)) ? 1.0 : 0.0;
      }
      __syncthreads();
      NLP_STAMP(9);
    }
    // rollouts: a quad per sample (the plan kernel's NLP-Euler fast stage + the general re-run)
    if (ST && tid >= kPerBlock * LPM) store_cand(tid - kPerBlock * LPM, NT - kPerBlock * LPM);
    if (tid < kPerBlock * LPM) {        // whole waves
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
    // the solve's last round: the sample's states after each step (the quad's lane 0, into LDS)
    // for the result's trajectory — the best's block copies them instead of re-running the
    // best's rollout at the end (8.6 us; keeping every round's states cost the rollouts ~1.4 us a
    // round, in LDS or in global memory alike)
    double* tj = ST && a.ltraj && sub == 0 && it == a.iters - 1 ? trl + (size_t)c * 6 * H - 6 : nullptr;
    if constexpr (ST)
      J = rollout<1, true, LPM, 0, true, false, false, true, false, false, kNlpStageW>(
          a.la, c, 0, x0, sx, su, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, bad, tj);
    else
      J = rollout<1, false, LPM, 0, true, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, bad);
    int bi = bad;
    bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
    bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
    if (__builtin_expect(__any(bi), 0)) {
      bool unused = false;
      if (bi) {
        if constexpr (ST)
          J = rollout<1, true, LPM, 0, false, false, false, true, false, false, kNlpStageW>(
              a.la, c, 0, x0, sx, su, veh, t, sk, q, Ts, a.up0, a.up1, K, fq, unused, tj);
        else
          J = rollout<1, false, LPM, 0, false, false, true>(a.la, c, 0, x0, sx, Ul, veh, t, sk, q, Ts, a.up0, a.up1, K,
                                                            fq, unused);
      }
    }
    NLP_STAMP(3);
    if (sub == 0) ks[c] = nlp_key(J);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's candidate stores (above)
    __syncthreads();
    NLP_STAMP(12);
    if (tid < 64) {                     // wave 0: the block's 64 keys sorted (bitonic, in registers)
      uint64_t k = ks[tid];
      uint32_t x = (uint32_t)(blk * kPerBlock + tid);
      nlp_sort64(k, x, tid);
      if (tid < len) {                  // the list as tagged words (nlp.hpp NlpLaunch.list_tag)
        uint64_t* lt = nlp_lists(a, it);
        const int e = blk * len + tid;
        st_wt(&lt[e], tag_word(sq, (uint32_t)(k >> 32)));
        st_wt(&lt[nbl + e], tag_word(sq, (uint32_t)k));
        st_wt(&lt[2 * nbl + e], tag_word(sq, x));
      }
    }
    // the next round's variates: helper waves 5-7 while waves 0-3 complete the round (ST: Ul is
    // dead, staged above and stored to cand) — not wave 4, which shares wave 0's SIMD, and wave 0
    // carries the completion's critical path (its sort, merges and elite loads slowed ~1 us
    // when wave 4 drew beside it, as the rollouts did when the helpers drew during them);
    // unstaged (H > kNlpStageH), every wave before the completion (the rollouts read Ul)
    constexpr int kDraw0 = kPerBlock * LPM + 64;
    if (r + 1 < a.rounds) {
      if (!ST) nlp_draw(a, blk, it + 1, Ul, us, tid, NT);
      else if (tid >= kDraw0) nlp_draw(a, blk, it + 1, Ul, us, tid - kDraw0, NT - kDraw0);
    }
    NLP_STAMP(11);
    // the round's completion, in every block
    NLP_STAMP(7);
    if (len <= 32) {
      if (!nlp_complete32(a, smem, cbase, it, r, nl, bjv, bitv, bsv, ms, bu, r + 1 == a.rounds, trl, sx, x0)) return;
    } else {
      const NlpCompLds L = nlp_comp_lds(cbase, nl, len);
      if (!nlp_poll_lists(a, L, nl, it, sq, rflag)) return;
      NLP_STAMP(4);
      nlp_complete(a, cbase, it, nl, bjv, bitv, bsv, ms, bu, r + 1 == a.rounds, trl, sx, x0);
    }
    // one launch per round: the best so far into the state for the next launch (block 0; kept in
    // registers and LDS within a launch — per-round stores here held block 0's next memory wait)
    if (r + 1 == a.rounds && it + 1 < a.iters && blk == 0) {
      for (int e = tid; e < 2 * H; e += NT) st_wt(&st->best_u[0][0] + e, bu[e]);
      if (tid == 0) {
        st_wt(&st->best_j, bjv);
        st_wt(&st->best_it, bitv);
        st_wt(&st->best_s, bsv);
      }
    }
  }
}

size_t nlp_lds_bytes(int H, int samples, int elite, bool ltraj) {
  return nlp_traj_off(H, samples / 64, elite) + (ltraj ? 48 * 64 * (size_t)H : 0);
}
bool nlp_ltraj_fits(int H, int samples, int elite) {
  return H <= kNlpStageH && nlp_lds_bytes(H, samples, elite, true) <= 160 * 1024;
}

hipError_t launch_nlp(const NlpLaunch& a, const NlpInline& pk, hipStream_t s) {
  const size_t lds = std::max<size_t>(nlp_lds_bytes(a.H, a.samples, a.elite, a.ltraj != 0), 82 * 1024);
  const dim3 grid(a.samples / 64);      // the sample blocks (each completes every round)
  if (a.H <= kNlpStageH) {
    allow_lds(nlp_kernel<true, 2 * kBlock>);
    hipLaunchKernelGGL((nlp_kernel<true, 2 * kBlock>), grid, dim3(2 * kBlock), lds, s, a, pk);
  } else {
    allow_lds(nlp_kernel<false, kBlock>);
    hipLaunchKernelGGL((nlp_kernel<false, kBlock>), grid, dim3(kBlock), lds, s, a, pk);
  }
  return hipGetLastError();
}

}  // namespace llampc
