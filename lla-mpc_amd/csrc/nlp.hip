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
//                   round): it polls every block's list, merges them pairwise up a tree — the
//                   lower len of two sorted lists is min(a_i, b_(len-1-i)), bitonic, then one
//                   half-cleaner network in registers per level — to the E best overall in order,
//                   reads the E elite sequences and sets the next mean / std as their mean /
//                   standard deviation (NumPy's axis-0 order): every block computes the same
//                   values in the same order, so all hold the same next distribution.  Block 0
//                   keeps the state (the best sequence so far) and writes the result.  The
//                   lists and the sequences are double-buffered by round parity: a block can be
//                   a round ahead of another, never two.  The next round's Philox variates (they
//                   do not depend on the mean / std) are drawn by the helper waves during the
//                   rollouts.  (A bitonic sort of all samples in LDS took 36 us of the 62 us
//                   round: 55 barrier-separated passes.)
#include "plan_dev.hpp"
#include "nlp.hpp"

namespace llampc {

#ifdef LLAMPC_STAMPS
// Diagnostic build only: s_memrealtime per block and phase of the last launch
// (tools/diag/nlp_phases.py): sample blocks 0 round start, 10 mean / std in, 1 samples formed,
// 2 rate-clipped, 9 staged, 3 rolled out, 11 next variates drawn; the completion block 7 round
// start, 4 lists in, 5 merged, 6 elite loaded, 8 next mean / std published.
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
// registers: their LDS reads issue together.  (Forming the samples inside this pass too, on
// its two waves instead of the block's four, measured 3.8 us against 1.8 + 1.7 us split.)
__device__ __forceinline__ void nlp_rate_chain(double* u, int H, double up, double lo, double hi) {
#pragma clang fp contract(off)
  if (!(lo <= hi)) return;
  double prev = up;
  for (int k0 = 0; k0 < H; k0 += 8) {
    const int n = H - k0;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i < n ? u[2 * (k0 + i)] : 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const double a = prev + lo, b = prev + hi;
      const double c = np_clip(v[i], a, b);
      prev = i < n ? c : prev;
      v[i] = c;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < n) u[2 * (k0 + i)] = v[i];
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

// lane ^ J's value: DPP quad_perm for J = 1, 2 (a VALU move), ds_swizzle's bit mode for J < 32
// (no address operand), ds_bpermute for J = 32 — ds_bpermute on every step made the block
// sort and the merge tree LDS-latency chains
template <int J>
__device__ __forceinline__ uint32_t nlp_xor32(uint32_t v) {
  static_assert(J >= 1 && J <= 32 && (J & (J - 1)) == 0, "a power of two below the wave size");
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (J < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (J << 10));
  else return (uint32_t)__shfl_xor((int)v, J, 64);
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
__device__ __forceinline__ void nlp_trajectory(const NlpLaunch& a, double* ub, bool better, double bj, int bit) {
  const int tid = threadIdx.x, H = a.H;
  const NlpState* st = a.st;
  NlpResult* res = a.res;
  __syncthreads();                      // the elite rows are read; best_u is final
  double* sx = ub + 2 * (size_t)H;      // after the sequence: xref [H+1][2], x0 [6]
  double* x0 = sx + 2 * (size_t)(H + 1);
  for (int e = tid; e < 2 * H; e += (int)blockDim.x) {
    const double v = better ? ub[e] : ld_wt(&st->best_u[0][0] + e);   // an earlier round's completion
    ub[e] = v;
    (&res->best_u[0][0])[e] = v;
  }
  if (tid == 0) {
    res->best_j = bj;
    res->best_it = bit;
  }
  for (int e = tid; e <= H; e += (int)blockDim.x) {
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

// The completion's LDS (every block): the lists' keys kA | kB and indices iA | iB ([nl * len] each,
// the merge tree's two buffers), then the elite sequences [E][H][2].
struct NlpCompLds {
  uint64_t *kA, *kB;
  uint32_t *iA, *iB;
  double* eu;
};
__device__ __forceinline__ NlpCompLds nlp_comp_lds(unsigned char* base, int nl, int len) {
  NlpCompLds L;
  L.kA = reinterpret_cast<uint64_t*>(base);
  L.kB = L.kA + (size_t)nl * len;
  L.iA = reinterpret_cast<uint32_t*>(L.kB + (size_t)nl * len);
  L.iB = L.iA + (size_t)nl * len;
  L.eu = reinterpret_cast<double*>(base + 24 * (size_t)nl * len);
  return L;
}
// its bytes: the lists, the elite rows, and the trajectory's reference and x0 after them
__host__ __device__ __forceinline__ size_t nlp_comp_bytes(int H, int nl, int elite) {
  return 24 * (size_t)nl * nlp_list_len(elite) + 16 * (size_t)elite * H + 16 * (size_t)(H + 1) + 48;
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
                                             int& bitv, double* ms, bool last_of_launch) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, H = a.H, E = a.elite;
  const int len = nlp_list_len(E);
  const bool b0 = blockIdx.x == 0;
  NlpState* st = a.st;
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
  const int bit0 = bitv;
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
    if (b0 && better) st_wt(&st->best_u[k][j], eu[2 * k + j]);
    msn[im] = m;                        // this block's copy (ms is read again only after a barrier)
    msn[is] = sd;
  }
  // the result (the last round): best objective and round, before this round's update
  const double bj = better ? c0 : bj0;
  const int bit = better ? it : bit0;
  bjv = bj;
  bitv = bit;
  if (b0 && tid == 0 && better) {
    st_wt(&st->best_j, c0);
    st_wt(&st->best_it, it);
  }
  NLP_STAMP(8);
  if (b0 && it == a.iters - 1) nlp_trajectory(a, eu, better, bj, bit);
  __syncthreads();                      // ms (the next round's) and the LDS lists (the next poll)
}

}  // namespace

// ST: the candidates' per-step input terms staged in LDS once per block (pwm, delta, sin /
// cos delta, the input-rate cost term, feasibility: the plan kernel's staged Euler layout,
// [k][c][kStageW]), so the rollout loop reads them instead of forming them per step; when
// 64 x H x 64 B fit beside the rest (H <= kNlpStageH).
constexpr int kNlpStageH = 28;

// The round's Philox variates z of this block's samples into Ul (value (s H + k) 2 + j; the
// pair (s H + k) shares one call): independent of the round's mean / std, so a block draws the
// next round's while the completion block works.
__device__ __forceinline__ void nlp_draw(const NlpLaunch& a, int blk, int it, double* Ul, int t0, int stride) {
  constexpr int kPerBlock = 64;
  const int H = a.H;
  for (int e = t0; e < kPerBlock * H; e += stride) {
    const int rr = e / H, k = e - rr * H, s = blk * kPerBlock + rr;
    double z0, z1;
    nlp_z2((uint32_t)(s * H + k), a.call, a.seed, (uint32_t)(it + 1), z0, z1);
    Ul[2 * e] = z0;
    Ul[2 * e + 1] = z1;
  }
}

// The sample block's LDS after the scratch: xref [H+1][2] | Ul [64][H][2] | x0 [6] | keys [64] |
// mean / std [2][H][2] | ST: the staged terms [H][64][kStageW] — the completion's region
// (nlp_comp_bytes) reuses them once the rollouts are done — else the completion's region.
__host__ __device__ __forceinline__ size_t nlp_su_off(int H) {
  return kScratchBytes + 16 * (size_t)(H + 1) + 16 * 64 * (size_t)H + 48 + 8 * 64 + 32 * (size_t)H;
}

// NT threads: the rollouts take the first 256 (a quad per sample); the other waves share the
// blocks' per-round loops (bounds, staging, the completion) and draw the next round's variates
// while the rollouts run (ST), two waves per SIMD
template <bool ST, int NT>
__global__ __launch_bounds__(NT) void nlp_kernel(NlpLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* rflag = reinterpret_cast<int*>(smem + kFlagOff);   // a bounded wait's block verdict
  const int tid = threadIdx.x, H = a.H, blk = (int)blockIdx.x;
  const int nl = (int)gridDim.x;        // every block samples, every block completes every round
  constexpr int LPM = 4, kPerBlock = 64;             // 64 samples per block, a quad each
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);            // xref [H+1][2]
  double* Ul = sx + 2 * (H + 1);                                            // [64][H][2]
  double* x0 = Ul + 2 * (size_t)kPerBlock * H;                              // [6]
  uint64_t* ks = reinterpret_cast<uint64_t*>(x0 + 6);                       // [64] the samples' keys
  double* ms = reinterpret_cast<double*>(ks + 64);                          // the round's mean, std [2][H][2]
  double* su = reinterpret_cast<double*>(smem + nlp_su_off(H));             // ST: [H][64][kStageW]
  unsigned char* cbase = smem + nlp_su_off(H);                              // the completion's region
  NlpState* st = a.st;
  const int len = nlp_list_len(a.elite), nbl = nl * len;
  for (int e = tid; e <= H; e += NT) {   // the solve's inputs (this block's LDS only)
    sx[2 * e] = a.xref[e];
    sx[2 * e + 1] = a.xref[(H + 1) + e];
  }
  if (tid < 6) x0[tid] = a.x0[tid];
  nlp_draw(a, blk, a.it, Ul, tid, NT);      // the first round's variates
  // the best so far as the launch starts (host-staged, or an earlier launch's rounds)
  double bjv = ld_wt(&st->best_j);
  int bitv = ld_wt(&st->best_it);
  for (int r = 0; r < a.rounds; ++r) {
    const int it = a.it + r;
    const uint32_t sq = nlp_seq(a.host_seq, it);
    NLP_STAMP(0);
    // the round's mean / std: the host-staged state (round 0), this block's completion of the
    // previous round (in ms already), or — a launch's first round after round 0 — the previous
    // launch's block 0's tagged halves
    if (it == 0) {
      for (int e = tid; e < 4 * H; e += NT)
        ms[e] = ld_wt(e < 2 * H ? &st->mean[0][0] + e : &st->std_[0][0] + (e - 2 * H));
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
    for (int e = tid; e < kPerBlock * H; e += NT) {
      const int rr = e / H, k = e - rr * H, s = blk * kPerBlock + rr;
      Ul[2 * e] = nlp_raw_z(a, ms, it, s, k, 0, Ul[2 * e]);
      Ul[2 * e + 1] = nlp_raw_z(a, ms, it, s, k, 1, Ul[2 * e + 1]);
    }
    __syncthreads();
    NLP_STAMP(1);
    if (tid < 2 * kPerBlock) {
      const int rr = tid >> 1, j = tid & 1;
      nlp_rate_chain(Ul + 2 * (size_t)rr * H + j, H, j ? a.up1 : a.up0, j ? a.rlo1 : a.rlo0, j ? a.rhi1 : a.rhi0);
    }
    __syncthreads();
    NLP_STAMP(2);
    // the rate-clipped sequences for every block's elite read (each wave drains these stores
    // before its list is published, below)
    double* cand = nlp_cand(a, it);
    for (int e = tid; e < kPerBlock * H * 2; e += NT) st_wt(&cand[(size_t)blk * kPerBlock * 2 * H + e], Ul[e]);
    const fm::FmK K = fm::FmK::load();
    if constexpr (ST) {
      const CostK& q0 = a.la.cost;
      // consecutive threads take consecutive candidates of one step: their 64-B records are
      // adjacent in LDS (one step per thread-row was a 4 KB stride: every write one bank)
      for (int f = tid; f < kPerBlock * H; f += NT) {
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
    } else if (ST && r + 1 < a.rounds) {
      // the helper waves: the next round's variates (Ul is dead: staged above, stored to cand)
      nlp_draw(a, blk, it + 1, Ul, tid - kPerBlock * LPM, NT - kPerBlock * LPM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's candidate stores (above)
    __syncthreads();
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
    // unstaged (H > kNlpStageH): the rollouts read Ul, so the next round's variates now
    if (!ST && r + 1 < a.rounds) nlp_draw(a, blk, it + 1, Ul, tid, NT);
    NLP_STAMP(11);
    // the round's completion, in every block
    const NlpCompLds L = nlp_comp_lds(cbase, nl, len);
    NLP_STAMP(7);
    if (!nlp_poll_lists(a, L, nl, it, sq, rflag)) return;
    NLP_STAMP(4);
    nlp_complete(a, cbase, it, nl, bjv, bitv, ms, r + 1 == a.rounds);
  }
}

size_t nlp_lds_bytes(int H, int samples, int elite) {
  const size_t su = H <= kNlpStageH ? 8 * kStageW * 64 * (size_t)H : 0;
  return nlp_su_off(H) + std::max(su, nlp_comp_bytes(H, samples / 64, elite));
}

hipError_t launch_nlp(const NlpLaunch& a, hipStream_t s) {
  const size_t lds = std::max<size_t>(nlp_lds_bytes(a.H, a.samples, a.elite), 82 * 1024);
  const dim3 grid(a.samples / 64);      // the sample blocks (each completes every round)
  if (a.H <= kNlpStageH) {
    allow_lds(nlp_kernel<true, 2 * kBlock>);
    hipLaunchKernelGGL((nlp_kernel<true, 2 * kBlock>), grid, dim3(2 * kBlock), lds, s, a);
  } else {
    allow_lds(nlp_kernel<false, kBlock>);
    hipLaunchKernelGGL((nlp_kernel<false, kBlock>), grid, dim3(kBlock), lds, s, a);
  }
  return hipGetLastError();
}

}  // namespace llampc
