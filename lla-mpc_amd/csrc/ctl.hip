// ctl.hip — the controller tick: one launch per LLA-MPC control step (ctl.hpp has the map to
// the reference).  Roles by block index (look-back blocks first in dispatch order):
//
//   look-back blocks [0, nb_lb)   the plan launch's look-back (lookback_block: RK4 step of
//                                 every model from the state's (x_{t-1}, u_{t-1}), error, ring,
//                                 window mean, wave/block top-K lists); the last one (ticket)
//                                 merges them (lb_final<SEL>), PUBLISHES the selection
//                                 (top-K + argmin, tagged words) and completes the tick
//                                 (ctl_complete).  Without a look-back (ticks 0, 1) block 0
//                                 only completes.
//   look-ahead blocks [nb_lb, ..) each: the raceline tables to LDS; the projection of x_t and
//                                 ConstantSpeed with mu-hat (one lane walks, planner.py:
//                                 24-65); the C candidates (Philox, every lane); then it WAITS
//                                 for the selection (or, while the window fills, takes the
//                                 nominal model) and rolls out its slots' models x C candidates
//                                 (the plan kernel's fused RK4 rollout, candidates read from
//                                 LDS) and publishes each slot's best candidate.
//
// Waiting: a look-ahead block waits only for the look-back ticket winner, a block of LOWER
// index; workgroups are dispatched in index order (per XCD), so that block has been dispatched
// and never waits on a look-ahead block before it publishes (the selection comes before its
// own poll).  The completion waits only for look-ahead blocks, which then never wait again.
// Every wait has a bound (status LLAMPC_STATUS_POLL_TIMEOUT, never expected).
#include "plan_dev.hpp"
#include "ctl.hpp"

namespace llampc {

// LDS layout of the controller launch (byte offsets; 16-B aligned regions).  Look-ahead
// blocks: xref [H+1][2] | U [C][H][2] | knots [n + pad] | the two speed profiles bracketing mu
// interleaved per segment [n-1][2][4] (a, b, c, d of lo, then of hi: one segment's values are
// four 16-B reads) | with s4: sin / cos delta [C][H][2], then per candidate the summed
// input-rate cost and its feasibility flag [C][2] (staged during the walk) | misc.
// The completing block: lb_final's region from kScratchBytes (then the candidates [C][H][2]),
// its own area at poll_off (CtlPollLds).
struct CtlLds {
  size_t sx, ul, kn, spd, s4, misc, end;
};
__host__ __device__ __forceinline__ size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ __forceinline__ CtlLds ctl_lds(int H, int C, int n, bool s4 = false) {
  CtlLds L;
  size_t o = kScratchBytes;
  L.sx = o;
  o = align16(o + 16 * (size_t)(H + 1));
  L.ul = o;
  o = align16(o + 16 * (size_t)C * H);
  L.kn = o;
  o = align16(o + 8 * (size_t)(n + kKnotPad));
  L.spd = o;
  o = align16(o + 64 * (size_t)(n - 1));
  L.s4 = o;
  if (s4) o = align16(o + 16 * (size_t)C * H + 16 * (size_t)C);
  L.misc = o;
  L.end = o + 1024;
  return L;
}
// A spec block (ctl_spec): xref [H+1][2] (from the walker) | U [C][H][2] | the staged terms
// (s4) | the deferred positions [C][2][H] (X, Y of each candidate per step) | the quads' unused
// lanes' sink | misc (x_t, the doorbell's verdict, the model).
struct SpecLds {
  size_t sx, ul, s4, pos, junk, misc, end;
};
__host__ __device__ __forceinline__ SpecLds spec_lds(int H, int C) {
  SpecLds L;
  size_t o = kScratchBytes;
  L.sx = o;
  o = align16(o + 16 * (size_t)(H + 1));
  L.ul = o;
  o = align16(o + 16 * (size_t)C * H);
  L.s4 = o;
  o = align16(o + 16 * (size_t)C * H + 16 * (size_t)C);
  L.pos = o;
  o = align16(o + 16 * (size_t)C * H);
  L.junk = o;
  o += 8 * 64;
  L.misc = o;
  L.end = o + 256;
  return L;
}
constexpr size_t kCtlPollBytes = 4096;   // ctl_complete's area (layout there)
// ctl_complete's record words (one 8-byte word per lane of wave 0)
static_assert(offsetof(llampc_plan_out, window_full) == 4 && offsetof(llampc_plan_out, K) == 8 &&
                  offsetof(llampc_plan_out, sel_owned) == 12 && offsetof(llampc_plan_out, lb_best) == 16 &&
                  offsetof(llampc_plan_out, lb_best_val) == 24 && offsetof(llampc_plan_out, sel_model) == 32 &&
                  offsetof(llampc_plan_out, sel_cand) == 40 && offsetof(llampc_plan_out, n_nonfinite) == 44 &&
                  offsetof(llampc_plan_out, sel_cost) == 48 && offsetof(llampc_plan_out, la_best_model) == 56 &&
                  offsetof(llampc_plan_out, la_best_cand) == 64 && offsetof(llampc_plan_out, status) == 68 &&
                  offsetof(llampc_plan_out, la_best_cost) == 72 && offsetof(llampc_plan_out, topk) == 80,
              "llampc_plan_out header words");
static_assert(offsetof(llampc_ctl_out, tick) == sizeof(llampc_plan_out) &&
                  offsetof(llampc_ctl_out, projidx) == offsetof(llampc_ctl_out, tick) + 8 &&
                  offsetof(llampc_ctl_out, warm) == offsetof(llampc_ctl_out, tick) + 12 &&
                  offsetof(llampc_ctl_out, mu_used) == offsetof(llampc_ctl_out, tick) + 16 &&
                  offsetof(llampc_ctl_out, scale_used) == offsetof(llampc_ctl_out, tick) + 24 &&
                  offsetof(llampc_ctl_out, mu_pred) == offsetof(llampc_ctl_out, tick) + 32 &&
                  offsetof(llampc_ctl_out, dr_mean) == offsetof(llampc_ctl_out, tick) + 40 &&
                  offsetof(llampc_ctl_out, df_mean) == offsetof(llampc_ctl_out, tick) + 48,
              "llampc_ctl_out words");

#ifdef LLAMPC_STAMPS
// Diagnostic build only: s_memrealtime (100 MHz) per block and phase of the last launch
// (tools/diag/ctl_phases.py).  Look-ahead blocks: 0 entry, 1 staged, 10 walk done, 2 walk
// barrier, 3 selection, 4 rolled out, 5 published; look-back blocks: 0 entry, 6 scored,
// 7 lb_final done (ticket winner), 8 slots polled, 12 top-K / sequence stores issued, 13 the
// record words computed, 11 record stores issued, 9 record written; look-ahead prologue: 14 the
// mu bracket known, 15 the tables' LDS stores issued; 16 an armed launch's doorbell seen; the
// walk (cs_walk_wave): 17 its loop entered, 18 its loop done (then x/y).
static __device__ unsigned long long g_ctl_ph[64][24];
#define CTL_STAMP(blk, slot)                                                                   \
  do {                                                                                         \
    if (threadIdx.x == 0 && (blk) < 64) g_ctl_ph[blk][slot] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
extern "C" int llampc_debug_ctl_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ctl_ph), sizeof(g_ctl_ph)) == hipSuccess ? 0 : -2;
}
#else
#define CTL_STAMP(blk, slot) \
  do {                       \
  } while (0)
#endif

namespace {

// x_t[i] of the kernel argument by constant indices (a dynamic index into the argument's array
// makes the compiler copy the whole argument to scratch)
__device__ __forceinline__ double ctl_xt(const CtlLaunch& c, int i) {
  double v = c.x_t[0];
#pragma unroll
  for (int j = 1; j < 6; ++j) v = i == j ? c.x_t[j] : v;
  return v;
}

__device__ __forceinline__ bool ctl_late(uint64_t t0, uint32_t poll) {
  return __builtin_amdgcn_s_memrealtime() - t0 > ((uint64_t)poll << 16);
}

// An armed launch's doorbell (CtlLaunch.door): thread 0 of block 0 polls the pinned host copy
// (system-scope loads, all 13 words a round), every other block the device copy block 0 makes:
// its STATUS word alone, and once that carries door_seq the 12 x_t halves (block 0 drains their
// stores before it stores the status); every word's tag is checked.  One word per round on the
// device side: 13 words a round from 64 blocks made the relay 2.9 us instead of 1.1
// (tools/diag/doorbell_lat.hip, mode 3).  Returns, block-uniform after
// the barrier: kCtlDoorFire (x_t in xl), kCtlDoorCancel, kCtlDoorExpired.
__device__ __forceinline__ int ctl_door(const CtlLaunch& c, double* xl, int* res) {
  if (threadIdx.x == 0) {
    const bool host = blockIdx.x == 0;
    auto ld = [&](int q) {
      return host ? __hip_atomic_load(&c.door[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : ld_wt(&c.door_dev[q]);
    };
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t w[kCtlDoorWords];
    int r;
    for (;;) {
      // block 0 reads every word each round (the PCIe reads overlap; a second round trip for
      // the x_t halves after the status would add ~1 us), the others the status word first
      if (host) {
#pragma unroll
        for (int q = 0; q < kCtlDoorWords - 1; ++q) w[q] = ld(q);
      }
      const uint64_t sw = ld(kCtlDoorWords - 1);
      if (tag_ok(sw, c.door_seq)) {
        w[kCtlDoorWords - 1] = sw;
        r = (int)(uint32_t)sw;
        if (r != (int)kCtlDoorFire) break;
        if (!host) {
#pragma unroll
          for (int q = 0; q < kCtlDoorWords - 1; ++q) w[q] = ld(q);
        }
        int all = 1;
#pragma unroll
        for (int q = 0; q < kCtlDoorWords - 1; ++q) all &= (int)tag_ok(w[q], c.door_seq);
        if (all) break;
      }
      // block 0 gives up at the bound; the others wait twice as long for its verdict
      if (ctl_late(t0, host ? c.door_bound : 2 * c.door_bound)) {
        r = (int)kCtlDoorExpired;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (host) {                         // the verdict for the other blocks: x_t, drained, then the status
      if (r == (int)kCtlDoorFire) {
        st_wt(&c.door_dev[kCtlTimeWord], (uint64_t)__builtin_amdgcn_s_memrealtime());
#pragma unroll
        for (int q = 0; q < kCtlDoorWords - 1; ++q) st_wt(&c.door_dev[q], w[q]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      st_wt(&c.door_dev[kCtlDoorWords - 1], r == (int)kCtlDoorExpired ? tag_word(c.door_seq, kCtlDoorExpired)
                                                                       : w[kCtlDoorWords - 1]);
    }
    if (r == (int)kCtlDoorFire) {
#pragma unroll
      for (int j = 0; j < 6; ++j) xl[j] = __longlong_as_double((long long)join_words(w[2 * j], w[2 * j + 1]));
    }
    *res = r;
  }
  CTL_STAMP(blockIdx.x, 16);
  __syncthreads();
  return *res;
}

// ---- the speculative look-ahead (CtlLaunch.n_spec; ctl.hpp) --------------------------------
// The n_spec best of the look-back blocks' sorted lists: a tree merge in LDS (the cross-shard
// merge's), published as tagged words (local model index; kNoLocal: none).
// Polls this rank's mailbox words own[g stride + w] (w < nw, every g != rank) until each carries
// the tag seq — every thread issues all of its loads of a round before checking any (one memory
// round trip per round; a load under a per-word condition waits its own) — into rec32[g nw + w].
// Gives up after `bound` s_memrealtime ticks; returns this thread's late flag.
template <int kPer>
__device__ __forceinline__ int ctl_poll_words(const uint64_t* own, size_t stride, int G, int nw, int rank,
                                              uint32_t seq, uint64_t bound, uint32_t* rec32) {
  const int tid = threadIdx.x, total = G * nw;
  uint64_t need = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int e = tid + j * kBlock;
    if (e < total && e / nw != rank) need |= 1ull << j;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (need) {
    uint64_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int e = ((need >> j) & 1) ? tid + j * kBlock : rank * nw;   // idle: own slot (never read back)
      const int g = e / nw, w = e - g * nw;
      v[j] = __hip_atomic_load(own + (size_t)g * stride + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      if (((need >> j) & 1) && tag_ok(v[j], seq)) {
        rec32[tid + j * kBlock] = (uint32_t)v[j];
        need &= ~(1ull << j);
      }
    }
    if (!need) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > bound) return 1;
    __builtin_amdgcn_s_sleep(1);
  }
  return 0;
}

// The sharded controller's speculative list (peer transport, armed ticks): this shard's n_spec
// best by the window mean without x_t (value, GLOBAL index) as 4 n_spec tagged words pushed into
// every peer's mailbox slot at px_spec_off (after the selection record's words; the same tick
// number: the exchange of this tick, only earlier), the peers' lists polled, and the n_spec best
// over the ranks published — global indices, which the spec blocks roll out from the replicated
// global table.  All before the doorbell.  A peer whose list does not arrive within
// px_spec_wait (a rank that launched this tick instead of arming it has none) leaves this rank
// with its own list: the speculation only decides which models are rolled out early, never a
// result, so the ranks' records stay equal whatever their lists.
__device__ __forceinline__ void ctl_spec_exchange(const CtlLaunch& c, unsigned char* base, const Ent* top) {
  const int tid = threadIdx.x, G = c.px_G, rank = c.px_rank, M = c.n_spec, nw = 4 * M;
  uint32_t* rec32 = reinterpret_cast<uint32_t*>(base);                          // [G][nw]
  Ent* g0 = reinterpret_cast<Ent*>(base + align16(4 * (size_t)G * nw));
  Ent* g1 = g0 + (size_t)G * M;
  const int64_t goff = c.fin.goff;
  const size_t slot0 = (size_t)(c.px_seq & 1) * G * kRecWords;
  const size_t mine = slot0 + (size_t)rank * kRecWords + c.px_spec_off;
  for (int p = tid; p < G * nw; p += kBlock) {
    const int g = p / nw, w = p - g * nw;
    const Ent& x = top[w >> 2];
    const uint64_t q = (w & 2) ? (uint64_t)(x.i == kNoIndex ? (int64_t)-1 : goff + x.i) : (uint64_t)__double_as_longlong(x.v);
    const uint32_t word = (w & 1) ? (uint32_t)q : (uint32_t)(q >> 32);
    if (g == rank) rec32[(size_t)rank * nw + w] = word;
    else __hip_atomic_store(c.px_box[g] + mine + w, tag_word(c.px_seq, word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  constexpr int kPer = (kCtlPxMax * 4 * kCtlSpecMax + kBlock - 1) / kBlock;
  const int late = __syncthreads_or(
      ctl_poll_words<kPer>(c.px_box[rank] + slot0 + c.px_spec_off, kRecWords, G, nw, rank, c.px_seq, c.px_spec_wait, rec32));
  const int Gm = late ? 1 : G;
  for (int e = tid; e < Gm * M; e += kBlock) {
    const int g = late ? rank : e / M, j = e - (late ? 0 : g) * M;
    const uint32_t* r = rec32 + (size_t)g * nw + 4 * j;
    const int64_t id = (int64_t)join_words(r[2], r[3]);
    g0[e] = Ent{__longlong_as_double((long long)join_words(r[0], r[1])), id < 0 ? kNoIndex : id};
  }
  __syncthreads();
  const Ent* gtop = tree_merge(g0, g1, Gm, M);
  if (tid < M) {
    const int64_t i = gtop[tid].i;
    st_wt(&c.spec_tag[tid], tag_word(c.seq, i == kNoIndex ? kNoLocal : (uint32_t)i));
  }
}

template <bool PX>
__device__ __forceinline__ void ctl_spec_merge(const CtlLaunch& c, unsigned char* smem) {
  const int L = c.nb_lb, M = c.n_spec, tid = threadIdx.x;
  Ent* b0 = reinterpret_cast<Ent*>(smem + kScratchBytes);
  Ent* b1 = b0 + (size_t)L * M;
  for (int e = tid; e < L * M; e += kBlock) b0[e] = Ent{ld_wt(&c.spec_val[e]), ld_wt(&c.spec_idx[e])};
  __syncthreads();
  const Ent* top = tree_merge(b0, b1, L, M);
  if constexpr (PX) {
    if (c.px_G) {                       // launch-uniform: the lists of every rank
      ctl_spec_exchange(c, smem + kScratchBytes + align16(2 * sizeof(Ent) * (size_t)L * M), top);
      return;
    }
  }
  if (tid < M) {
    const int64_t i = top[tid].i;
    st_wt(&c.spec_tag[tid], tag_word(c.seq, i == kNoIndex ? kNoLocal : (uint32_t)i));
  }
}

// A look-back block's part, before the doorbell: its models ranked by the window mean without
// x_t (pred; NaN last, ties to the lower index — lb_final's order), the n_spec best stored
// sorted; the last block (ticket 1, reset at once: every block has drawn) merges the lists.
template <bool PX>
__device__ __forceinline__ void ctl_spec_lists(const CtlLaunch& c, int blk, double pred, bool valid, int64_t n,
                                               unsigned char* smem, int* flag) {
  const int tid = threadIdx.x, M = c.n_spec;
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem + kScratchBytes);
  uint32_t* ids = reinterpret_cast<uint32_t*>(keys + kBlock);
  const uint64_t key = valid ? order_key(pred) : ~0ull;
  const uint32_t id = valid ? (uint32_t)n : kNoModelId + (uint32_t)tid;
  keys[tid] = key;
  ids[tid] = id;
  __syncthreads();
  int r = 0;
#pragma unroll 16
  for (int j = 0; j < kBlock; ++j) r += (int)(keys[j] < key) | ((int)(keys[j] == key) & (int)(ids[j] < id));
  if (r < M) {
    st_wt(&c.spec_val[(int64_t)blk * M + r], valid ? pred : __builtin_nan(""));
    st_wt(&c.spec_idx[(int64_t)blk * M + r], valid ? n : kNoIndex);
  }
  if (!ticket_last(&c.tickets[1], (unsigned)c.nb_lb, flag)) return;
  if (tid == 0) __hip_atomic_store(&c.tickets[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ctl_spec_merge<PX>(c, smem);
}

// The deferred tracking cost (rollout<DEFER>): the split rollout's epilogue with the reference
// known — the same terms in the same order, so J equals the undeferred rollout's bitwise.
__device__ __forceinline__ double defer_cost(const double* dpos, int dstride, const double* sx, int H, int pc,
                                             double Qd, double Pd, const DeferOut& d, bool sok, bool& bad) {
  double track = 0.0, xr0 = 0.0;
  for (int k = 0; k < H; ++k) {
    xr0 = sx[2 * (k + 1) + pc];
    const double e = dpos[k * dstride] - xr0;
    track = track + e * (Qd * e);
  }
  const double e = d.xl - xr0;
  const double jl = e * (Pd * e) + track;
  double J = (dpp_bcast<kQuad0>(jl) + dpp_bcast<kQuad1>(jl)) + d.act;
  bad = (int)bad | (int)!sok | (int)!d.dok | (int)!(fabs(J) <= __DBL_MAX__) | (int)(d.feas_s != d.feas_s);
  if (!(d.feas_s != 0.0)) J = __builtin_inf();
  return J;
}

// The raw candidates [C][H][2] (before the rate clip) by threads t0 + i stride, i >= 0: from
// this tick's variates when the previous tick's completion drew them (znoise, tagged), four
// pairs' loads in flight per thread; else one Philox call per pair here.
__device__ __forceinline__ void ctl_draw(const CtlLaunch& c, const double* prev_seq, double up0, double up1,
                                         double* U, int t0, int stride) {
  const int H = c.la.H, C = c.la.C, CH = C * H;
  const double up[2] = {up0, up1};
  const int half = (int)(c.tick & 1);
  if (c.znoise && c.ztag[half] == c.tick + 1) {                     // launch-uniform
    const double* zb = c.znoise + 2 * (size_t)CH * half;
    for (int p0 = t0; p0 < CH; p0 += 4 * stride) {
      double z[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = p0 + i * stride < CH ? p0 + i * stride : CH - 1;
        z[i][0] = zb[2 * p];
        z[i][1] = zb[2 * p + 1];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = p0 + i * stride;
        if (p < CH) {
          const int cc = p / H, k = p - cc * H;
          ctl_cand_pair_z(cc, k, H, prev_seq, up, c.nscale, c.umin, c.umax, z[i][0], z[i][1], U + 2 * (size_t)p);
        }
      }
    }
  } else {
    for (int p = t0; p < CH; p += stride) {
      const int cc = p / H, k = p - cc * H;
      ctl_cand_pair(cc, k, H, prev_seq, up, c.nscale, c.umin, c.umax, c.tick, c.seed, 0, U + 2 * (size_t)p);
    }
  }
}

// The next tick's variates into znoise half (t + 1) & 1 (the completing block's waves 1-3
// while wave 0 polls), then its tag; the next launch reads them after this one has ended.
__device__ __forceinline__ void ctl_draw_next(const CtlLaunch& c, int t0, int stride) {
  if (!c.znoise) return;
  const int H = c.la.H, CH = c.la.C * H;
  const uint64_t nt = c.tick + 1;
  double* zb = c.znoise + 2 * (size_t)CH * (int)(nt & 1);
  for (int p = t0; p < CH; p += stride) {
    double z0 = 0.0, z1 = 0.0;
    if (p >= H) ctl_z2((uint32_t)p, nt, c.seed, 0, z0, z1);           // candidate 0 has none
    *reinterpret_cast<double2*>(zb + 2 * (size_t)p) = double2{z0, z1};
  }
  if (t0 == 0) c.ztag[nt & 1] = nt + 1;
}

// ------------------------------------------------------------------------------------
// The completing block (after lb_final<true>, or alone on ticks without a look-back).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void ctl_complete(const CtlLaunch& c, unsigned char* smem, const CtlSel& cs,
                                             const double* xt) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x;
  const int H = c.la.H, C = c.la.C;
  unsigned char* pl = smem + c.poll_off;
  double* pdist = reinterpret_cast<double*>(pl);                  // [16]
  double* pcost = reinterpret_cast<double*>(pl + 128);            // [kCtlSlotsMax]
  int32_t* pcand = reinterpret_cast<int32_t*>(pl + 448);          // [kCtlSlotsMax]
  int32_t* pnf = reinterpret_cast<int32_t*>(pl + 608);            // [kCtlSlotsMax]
  double* pmu = reinterpret_cast<double*>(pl + 768);              // dr, df, mu_pred, mu_used
  int32_t* pmisc = reinterpret_cast<int32_t*>(pl + 1792);         // projidx
  double* cu = reinterpret_cast<double*>(smem + kScratchBytes);   // [C][H][2] (lb_final's region, dead)
  unsigned char* late_w = smem + kLateOff;
  CtlState* st = c.st;
  const bool warm = c.warm != 0;
  // the spec list (CtlLaunch.n_spec): a slot whose model is on it reads the spec block's words
  uint32_t* spec_ids = reinterpret_cast<uint32_t*>(pl + 3648);    // [kCtlSpecMax]
  if (tid < c.n_spec) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v = kNoLocal;
    for (;;) {
      const uint64_t w = ld_wt(&c.spec_tag[tid]);
      if (tag_ok(w, c.seq)) {
        v = (uint32_t)w;
        break;
      }
      if (ctl_late(t0, c.poll)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    spec_ids[tid] = v;
  }
  // Before the poll (the look-ahead blocks' rollouts take most of the launch) everything that
  // does not need their results: the projection, mu-hat and every candidate after its rate
  // clip (the look-ahead blocks' generator), so the chosen sequence is a copy after the poll.
  // The state is only read here; it is written after the poll, when no block reads it.
  const int p0 = st->projidx;
  const int segs = ctl_segments(p0, c.np);
  if (tid < kCtlSegs && tid < segs)                                // track.py:155-157
    pdist[tid] = ref_project_dist(xt[0], xt[1], c.pts[p0 + tid], c.pts[c.np + p0 + tid],
                                  c.pts[p0 + tid + 1], c.pts[c.np + p0 + tid + 1]);
  const double up0 = st->u_prev[0], up1 = st->u_prev[1];
  {
    const double* prev_seq = st->has_seq ? &st->useq[0][0] : nullptr;
    ctl_draw(c, prev_seq, up0, up1, cu, tid, kBlock);
  }
  __syncthreads();
  for (int t = tid; t < 2 * C; t += kBlock) {
    const int j = t & 1;
    ctl_rate_chain(cu + 2 * (size_t)(t >> 1) * H + j, H, j ? up1 : up0, j ? c.rate[1] : c.rate[0]);
  }
  if (tid == kBlock - 1) {
    pmisc[0] = segs >= 1 ? p0 + np_argmin(pdist, segs) : p0;      // planner.py:26-27
    // mu-hat (rt.py:326-344): the warm-up split with g = 9.8, else the top-K means
    const double mass = c.la.veh.mass, lf = c.la.veh.lf, lr = c.la.veh.lr;
    double dr, df;
    if (warm) {
      dr = c.mu_init * mass * 9.8 * lr / (lf + lr);
      df = c.mu_init * mass * 9.8 * lf / (lf + lr);
    } else {
      int kk = 0;
      while (kk < c.K && cs.ids[kk] != kNoLocal) ++kk;
      dr = np_pairwise_ring(cs.dr, 0, kk, LLAMPC_KMAX) / kk;
      df = np_pairwise_ring(cs.df, 0, kk, LLAMPC_KMAX) / kk;
    }
    // the histories are read and written by this block only (the look-ahead blocks read
    // mu_pred, which is written after the poll)
    const int cnt = st->hist_count;
    const int S = c.S;
    st->dr_hist[cnt % S] = dr;
    st->df_hist[cnt % S] = df;
    st->hist_count = cnt + 1;
    const int tot = cnt + 1, nl = tot < S ? tot : S, first = (tot - nl) % S;
    const double mu_old = ld_wt(&st->mu_pred);
    double mu_pred = mu_old;
    if (!warm)                                                     // rt.py:341
      mu_pred = (np_pairwise_ring(st->dr_hist, first, nl, S) / nl + np_pairwise_ring(st->df_hist, first, nl, S) / nl) /
                (9.81 * mass);
    pmu[0] = dr;
    pmu[1] = df;
    pmu[2] = mu_pred;
    pmu[3] = c.use_mu ? mu_old : c.mu_fixed;                       // the mu this tick's walk used
  }
  // the current model (this block writes it after the poll): loaded now, off the tail
  const int64_t cur_model = (tid < 64 && warm) ? st->current_model : 0;
  // x_prev: every look-back block has read it (this block holds the last ticket) and the
  // look-ahead blocks never do — stored now, so no load of x_t sits behind the record's host
  // stores after the poll
  if (tid < 6) st->x_prev[tid] = xt[tid];
  // the record's scalar kernel arguments, loaded (and kept) before the poll: the tail used
  // to wait for them one by one after it
  // (readfirstlane: launch-uniform values in SGPRs whatever the argument's copy)
  auto rfl = [](int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane(v); };
  auto rfl64 = [](int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  };
  int32_t a_wc = rfl(c.fin.window_count), a_full = rfl(c.fin.full), a_K = rfl(c.K), a_warm = rfl(c.warm),
          a_lap = rfl(c.lap_projidx);
  int64_t a_goff = rfl64(c.sel_goff), a_tick = rfl64((int64_t)c.tick);
  double a_scale = __longlong_as_double((long long)rfl64(__double_as_longlong(c.use_mu ? c.v_factor : c.scale_fixed)));
  asm volatile("" : "+s"(a_wc), "+s"(a_full), "+s"(a_K), "+s"(a_warm), "+s"(a_lap));
  asm volatile("" : "+s"(a_goff), "+s"(a_tick), "+s"(a_scale));
  // waves 1-3 draw the next tick's variates while wave 0 polls (off every critical path)
  if (tid >= 64) ctl_draw_next(c, tid - 64, kBlock - 64);
  // every slot's result (tagged words of the look-ahead blocks)
  int late = 0;
  if (tid < c.nslots) {
    uint64_t w[4];
    const uint64_t* src = c.slot_tag + 4 * (size_t)tid;
    if (c.n_spec && !warm) {
      const uint32_t id = cs.ids[tid];
      for (int p = 0; p < c.n_spec; ++p)
        if (id != kNoLocal && spec_ids[p] == id) src = c.spec_res + 4 * (size_t)p;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = ld_wt(&src[q]);
      if ((int)tag_ok(w[0], c.seq) & (int)tag_ok(w[1], c.seq) & (int)tag_ok(w[2], c.seq) & (int)tag_ok(w[3], c.seq))
        break;
      if (ctl_late(t0, c.poll)) {
        late = 1;
        break;
      }
    }
    const uint32_t nfw = (uint32_t)w[3];
    late |= (int)(nfw >> 31);
    pcost[tid] = late ? __builtin_nan("") : __longlong_as_double((long long)join_words(w[0], w[1]));
    pcand[tid] = late ? -1 : (int32_t)(uint32_t)w[2];
    pnf[tid] = late ? 0 : (int32_t)(nfw & 0x7FFFFFFFu);
  }
  const int wl = __any(late);
  if ((tid & 63) == 0) late_w[tid >> 6] = (unsigned char)wl;
  __syncthreads();
  CTL_STAMP(blockIdx.x, 8);
  // the record and the state
  const int ss = warm ? 0 : c.K;                                   // the selected model's slot
  const int scand = pcand[ss] >= 0 ? pcand[ss] : 0;
  // (assembling the record in LDS and copying it with 16-B stores made the system fence wait
  // ~2 us for the ~100 wide host stores: +1 us on the tail, profiles/r04/s4/ctl_phases_image.txt)
  llampc_ctl_out* o = c.out;
  llampc_plan_out* po = &o->plan;
  const double nan = __builtin_nan("");
  // the top-K's candidates (wave 1) and the chosen sequence (waves 2-3) while wave 0 forms the
  // record's words: every wave issues its own stores into the pinned record (one wave issuing
  // them all in turn put ~1 us before the words, profiles/r05/spec2/phases_armed.txt)
  if (tid >= 64 && tid < 64 + LLAMPC_KMAX) {
    const int k = tid - 64;
    const bool have = !warm && k < c.K;
    if (warm) {                         // no look-back selection yet (lb_final did not run)
      po->topk[k] = -1;
      po->topk_val[k] = po->topk_Df[k] = po->topk_Dr[k] = nan;
    }
    po->topk_cand[k] = have ? pcand[k] : -1;
    po->topk_cost[k] = have ? pcost[k] : nan;
  }
  if (tid >= 128 && tid < 128 + 2 * H) {   // the chosen sequence: candidate sel_cand
    const int e = tid - 128;
    const double v = cu[2 * (size_t)scand * H + e];
    (&o->u_seq[0][0])[e] = v;
    (&st->useq[0][0])[e] = v;
    if (e < 2) st->u_prev[e] = v;
  }
  CTL_STAMP(blockIdx.x, 12);
  if (tid < 64) {
    // wave 0: the look-ahead best over the rolled-out slots (flattened (model, candidate)
    // order, NaN last, ties to the lower key) as a wave pick, then the record's scalars as
    // one 8-byte word per lane — one store instruction into the pinned host record (thread 0
    // storing the ~25 fields one by one over PCIe took ~4 us, profiles/r04/ctl_record_split.txt)
    const int q = tid;
    const bool slot = q < c.nslots;
    const bool valid = slot && !warm && pcand[q] >= 0 && cs.ids[q] != kNoLocal;
    double lav = valid ? pcost[q] : nan;
    int64_t lai = valid ? (a_goff + (int64_t)cs.ids[q]) * C + pcand[q] : kNoIndex;
    wave_pick_nl64(lav, lai);
    const int nf = wave_sum(slot ? pnf[q] : 0);
    int anyl = *cs.xlate;                // the sharded exchange gave up on a peer
    for (int w = 0; w < kWaves; ++w) anyl |= late_w[w];
    const int64_t sel = warm ? cur_model : a_goff + (int64_t)cs.ids[a_K];
    const double dr = pmu[0], df = pmu[1], mu_pred = pmu[2];
    int pj = pmisc[0];
    if (pj > a_lap) pj = 0;                                        // rt.py:287-296
    int64_t lm;
    int32_t lc;
    split_key(lai == kNoIndex ? 0 : lai, C, lm, lc);
    auto pack = [](int32_t lo, int32_t hi) { return (uint64_t)(uint32_t)lo | ((uint64_t)(uint32_t)hi << 32); };
    auto bits = [](double v) { return (uint64_t)__double_as_longlong(v); };
    // llampc_plan_out words 0..9 (lb_best / lb_best_val, words 2 and 3, are lb_final's unless
    // warm), then llampc_ctl_out's words after the plan record (static_asserts below)
    // every word uniform, each lane selects its own (no per-lane branches)
    const uint64_t W[17] = {pack(a_wc, a_full),
                            pack(a_K, 1),                                  // sel_owned
                            (uint64_t)(int64_t)-1,
                            bits(nan),
                            (uint64_t)sel,
                            pack(pcand[ss], nf),
                            bits(pcost[ss]),
                            (uint64_t)(lai == kNoIndex ? (int64_t)-1 : lm),
                            pack(lai == kNoIndex ? -1 : lc, anyl ? kPollTimeoutStatus : 0),
                            bits(lai == kNoIndex ? nan : lav),
                            (uint64_t)a_tick,
                            pack(pj, a_warm),
                            bits(pmu[3]),                                  // mu_used
                            bits(a_scale),
                            bits(mu_pred),
                            bits(dr),
                            bits(df)};
    uint64_t w = W[0];
#pragma unroll
    for (int i = 1; i < 17; ++i) w = q == i ? W[i] : w;
    const bool store = q < 17 && (warm || (q != 2 && q != 3));
    uint64_t* dst = q < 10 ? reinterpret_cast<uint64_t*>(po) + q : reinterpret_cast<uint64_t*>(&o->tick) + (q - 10);
    CTL_STAMP(blockIdx.x, 13);
    if (store) *dst = w;
    if (q == 0) {
      st->mu_pred = mu_pred;
      st->projidx = pj;
      st->has_seq = 1;
      if (!warm) st->current_model = sel;
      __hip_atomic_store(&c.tickets[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  CTL_STAMP(blockIdx.x, 11);
  if (tid == 0)                        // x_t on the device -> the record's stores issued (ctl.hpp)
    __hip_atomic_store(c.host_tag + 1, (uint64_t)__builtin_amdgcn_s_memrealtime() - ld_wt(&c.door_dev[kCtlTimeWord]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();              // ~0.4 us (a plain vmcnt wait: ~0.3, ctl_record_split.txt)
  __syncthreads();
  CTL_STAMP(blockIdx.x, 9);
  if (tid == 0) __hip_atomic_store(c.host_tag, c.host_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------
// The sharded controller's exchange (ctl.hpp "sharded controller"; BASELINE config 5): run by
// the look-back ticket winner after lb_final<2> left this shard's top-K and argmin in cs.ids /
// cs.xv.  (a) The record — K + 1 entries of (window mean, global index) as 32-bit words — goes
// to LDS and, tagged with the mailbox's tick number, into slot [seq & 1][rank] of every peer's
// mailbox (system-scope stores over xGMI; the slot-reuse argument is peer_exchange_kernel's);
// (b) this rank's mailbox is polled for the G - 1 peer records (every thread issues all of its
// loads before checking any); (c) the merge: each top-K entry's rank among the G K gathered
// ones (ctl_merge_rank), the argmin over the G argmins (ctl_merge_argmin); (d) the MERGED
// selection is published for the look-ahead blocks (global indices: they roll the models out
// from the replicated global parameter table) and (e) the record's look-back fields and the
// top-K Dr / Df for mu-hat are written.  A peer that never arrives (past px_bound): this
// shard's own selection is used and the record's status says so.
// ------------------------------------------------------------------------------------
// Word w of this shard's record: entry w / 4 of lb_final<2>'s lists (cs.ids local index / cs.xv
// window mean) as value hi, lo, global index hi, lo (index -1: none).
__device__ __forceinline__ uint32_t ctl_rec_word(const CtlSel& cs, int64_t goff, int w) {
  const int e = w >> 2;
  const uint32_t l = cs.ids[e];
  const uint64_t q = (w & 2) ? (uint64_t)(l == kNoLocal ? (int64_t)-1 : goff + (int64_t)l)
                             : (uint64_t)__double_as_longlong(cs.xv[e]);
  return (w & 1) ? (uint32_t)q : (uint32_t)(q >> 32);
}

// A gather transport's first launch (px_phase 1): the look-back's ticket winner stores this
// shard's record, tagged px_seq, at px_send for the all-gather between the launches, and
// re-arms the look-back ticket (the completion does it on one-launch ticks).
__device__ __forceinline__ void ctl_px_send(const CtlLaunch& c, const CtlSel& cs) {
  __syncthreads();                                       // lb_final's wave 0 wrote cs.ids / xv
  const int nw = ctl_rec_words(c.K);
  for (int w = threadIdx.x; w < nw; w += kBlock) st_wt(&c.px_send[w], tag_word(c.px_seq, ctl_rec_word(cs, c.fin.goff, w)));
  if (threadIdx.x == 0) __hip_atomic_store(&c.tickets[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void ctl_exchange(const CtlLaunch& c, unsigned char* smem, const CtlSel& cs) {
  const int tid = threadIdx.x;
  const int G = c.px_G, rank = c.px_rank, K = c.K, nw = ctl_rec_words(K), M = G * K;
  const int64_t goff = c.fin.goff;
  unsigned char* base = smem + kScratchBytes;            // lb_final's region (dead)
  uint32_t* rec32 = reinterpret_cast<uint32_t*>(base);   // [G][nw]
  uint64_t* ekey = reinterpret_cast<uint64_t*>(base + align16(4 * (size_t)G * nw));
  uint64_t* eid = ekey + M;
  int* top = reinterpret_cast<int*>(eid + M);            // [KMAX] entry of each merged rank
  int* wlate = top + LLAMPC_KMAX;                        // [kWaves]
  const bool gath = c.px_phase == 2;                     // launch-uniform
  if (!gath) __syncthreads();                            // lb_final's wave 0 wrote cs.ids / xv
  // (a) this shard's record: to LDS and, tagged, to every peer (one (peer, word) per thread);
  // gathered: the own record from px_send (the first launch's), the peers' come from px_gath
  const size_t slot0 = gath ? 0 : (size_t)(c.px_seq & 1) * G * kRecWords;
  const size_t mine = slot0 + (size_t)rank * kRecWords;
  if (gath) {
    for (int w = tid; w < nw; w += kBlock) rec32[(size_t)rank * nw + w] = (uint32_t)ld_wt(&c.px_send[w]);
  } else {
    for (int p = tid; p < G * nw; p += kBlock) {
      const int g = p / nw, w = p - g * nw;
      const uint32_t word = ctl_rec_word(cs, goff, w);
      if (g == rank) rec32[(size_t)rank * nw + w] = word;
      else __hip_atomic_store(c.px_box[g] + mine + w, tag_word(c.px_seq, word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // (b) the peers' records from this rank's mailbox (gathered: from px_gath, stride nw)
  constexpr int kPer = (kCtlPxMax * ctl_rec_words(LLAMPC_KMAX) + kBlock - 1) / kBlock;
  const uint64_t* own = gath ? c.px_gath : c.px_box[rank] + slot0;
  const size_t stride = gath ? (size_t)nw : (size_t)kRecWords;
  int late = ctl_poll_words<kPer>(own, stride, G, nw, rank, c.px_seq, (uint64_t)c.px_bound << 16, rec32);
  const int wl = __any(late);
  if ((tid & 63) == 0) wlate[tid >> 6] = wl;
  __syncthreads();
  late = 0;
  for (int w = 0; w < kWaves; ++w) late |= wlate[w];
  auto ent_v = [&](int g, int j) {
    const uint32_t* r = rec32 + (size_t)g * nw + 4 * j;
    return __longlong_as_double((long long)join_words(r[0], r[1]));
  };
  auto ent_id = [&](int g, int j) {
    const uint32_t* r = rec32 + (size_t)g * nw + 4 * j;
    return (int64_t)join_words(r[2], r[3]);
  };
  // (c) the merge (block-uniform branch): every top-K entry's merged rank
  if (!late) {
    for (int e = tid; e < M; e += kBlock) {
      const int g = e / K, j = e - g * K;
      ctl_entry_order(ent_v(g, j), ent_id(g, j), e, ekey[e], eid[e]);
    }
    __syncthreads();
    for (int e = tid; e < M; e += kBlock) {
      const int r = ctl_merge_rank([&](int j) { return ekey[j]; }, [&](int j) { return eid[j]; }, M, e);
      if (r < K) top[r] = e;
    }
  } else if (tid < K) {
    top[tid] = rank * K + tid;                           // this shard's own lists
  }
  __syncthreads();
  if (tid >= 64) return;                                 // one wave finishes (the caller re-converges)
  const int lane = tid;
  const int Gm = late ? 1 : G;                           // argmin over every shard, or this one
  double bv;
  int64_t bi;
  ctl_merge_argmin([&](int g, double& v, int64_t& id) {
                     const int gg = late ? rank : g;
                     v = ent_v(gg, K);
                     id = ent_id(gg, K);
                   },
                   Gm, c.fin.nan_first != 0, bv, bi);
  double kv = __builtin_nan("");
  int64_t kid = -1;
  if (lane < K) {
    const int e = top[lane], g = e / K, j = e - g * K;
    kv = ent_v(g, j);
    kid = ent_id(g, j);
  }
  // (d) the merged selection (global indices < 2^32 - 1: llampc_ctl_set_exchange checks)
  const uint32_t kl = kid < 0 ? kNoLocal : (uint32_t)kid;
  const uint32_t al = bi < 0 ? kNoLocal : (uint32_t)bi;
  if (lane < K) {
    cs.ids[lane] = kl;
    st_wt(&cs.tag[lane], tag_word(cs.seq, kl));
  }
  if (lane == 0) {
    cs.ids[K] = al;
    st_wt(&cs.tag[K], tag_word(cs.seq, al));
    *cs.xlate = late;
  }
  // (e) the record's look-back half (pinned host memory, sc1 like lb_final's) and mu-hat's Dr / Df
  const double* gp = c.la.params;                        // the replicated global table [6][n]
  const int64_t gn = c.la.n;
  llampc_plan_out* o = &c.out->plan;
  const double nan = __builtin_nan("");
  if (lane < LLAMPC_KMAX) {
    const bool have = lane < K && kid >= 0;
    const double df = have ? gp[2 * gn + kid] : nan, dr = have ? gp[5 * gn + kid] : nan;
    st_wt(&o->topk[lane], have ? kid : (int64_t)-1);
    st_wt(&o->topk_val[lane], have ? kv : nan);
    st_wt(&o->topk_Df[lane], df);
    st_wt(&o->topk_Dr[lane], dr);
    if (lane < K) {
      cs.dr[lane] = dr;
      cs.df[lane] = df;
    }
  }
  if (lane == 0) {
    st_wt(&o->lb_best, bi);
    st_wt(&o->lb_best_val, bi < 0 ? nan : bv);
  }
}

// ------------------------------------------------------------------------------------
// The device ConstantSpeed (planner.py:12-67), shared by the controller's look-ahead blocks
// and llampc_ctl_reference: tables -> LDS, the projection, one lane's walk.
// ------------------------------------------------------------------------------------
// knots (+inf pad, RaceRef::step) and the two speed profiles bracketing mu, interleaved per
// segment [n-1][2][4] (consecutive threads write consecutive LDS words; a wave's loads touch 8
// rows x 8 consecutive segments).  The x/y rows stay in global memory: the walk records each
// step's (segment, dx) and x/y are evaluated once after it, in parallel.
__device__ __forceinline__ void cs_stage(const RacelineK& rl, const MuBracket& br, double* kn, double* spd) {
  const int nseg = rl.n - 1;
  const double* slo = rl.speed + (size_t)br.lo * 4 * nseg;
  const double* shi = rl.speed + (size_t)br.hi * 4 * nseg;
  copy_lds<4>(kn, rl.n, [&](int e) { return rl.knots[e]; });
  copy_lds<24>(spd, 8 * nseg, [&](int e) {
    const int sg = e >> 3, q = e & 3;
    return ((e >> 2) & 1 ? shi : slo)[(size_t)q * nseg + sg];
  });
  if ((int)threadIdx.x < kKnotPad) kn[rl.n + threadIdx.x] = __builtin_inf();
}

// project_fast of (px, py) on points[:, p0 : p0 + 10] (track.py:147-160): threads < segs
// write their segment's distance; returns the segment count
__device__ __forceinline__ int cs_project(const double* pts, int np_, int p0, double px, double py, double* dist) {
  const int segs = ctl_segments(p0, np_);
  const int tid = threadIdx.x;
  if (tid < kCtlSegs && tid < segs)
    dist[tid] = ref_project_dist(px, py, pts[p0 + tid], pts[np_ + p0 + tid], pts[p0 + tid + 1], pts[np_ + p0 + tid + 1]);
  return segs;
}

// x / den rounded as the IEEE division, by den's correctly rounded reciprocal rden = 1 / den:
// q0 = x rden, then one FMA residual step (Markstein; checked against x / den on 10^8 pairs
// of normal operands) — 3 dependent instructions instead of the division's ~10
__device__ __forceinline__ double div_by(double x, double den, double rden) {
  const double q0 = x * rden;
  const double e = __builtin_fma(-q0, den, x);
  return __builtin_fma(e, rden, q0);
}

// One speed profile's cubic at dx from its interleaved coefficients (spline_at's expression,
// so the same roundings): two 16-B LDS reads.
__device__ __forceinline__ double spline4(const double* c, double dx) {
  const double2 ab = *reinterpret_cast<const double2*>(c);
  const double2 cd = *reinterpret_cast<const double2*>(c + 2);
  const double dx2 = dx * dx;
  return ab.x + ab.y * dx + cd.x * dx2 + cd.y * (dx2 * dx);
}

// ConstantSpeed's walk (planner.py:24-65) by ONE WAVE (all 64 lanes call it, uniform control
// flow): projidx = p0 + argmin (:26-27), the start arc length from the prefix table (:29-36),
// then H <= 64 steps of :40-62 into sx [H+1][2]; returns projidx and, in lane 0, vr (:63-64).
// RaceRef::step's walk over a window of 64 consecutive segments held in registers — lane j
// segment w0 + j: its knot (+inf past the last) and the two speed cubics' coefficients — so a
// step reads no memory: every lane evaluates its segment's v at t, the count of knots <= t over
// the kWalkAhead lanes past the current segment (a ballot: RaceRef::step's advance) picks the
// lane whose v holds, and readlane takes v, the knot and dx from it.  The chain of a step is
// the cubic and one division chain.  The window moves (64 lanes' LDS reads) when the
// candidates would leave it — about once per walk; x/y are not on the chain: lane k keeps step
// k's (segment, dx) and evaluates :43 after the walk.  (Before: each step read its candidate
// segments from LDS — one LDS round trip on the chain, ~0.3 us a step; the serial walker
// ~0.7 us.)  v = (v_lo wa) / den + (v_hi wb) / den (:58-60), the divisions by div_by, the cubic
// spline_at's expression (spline4's): the same roundings as before.
constexpr int kWalkAhead = 16;
__device__ __forceinline__ double cubic4(double a, double b, double c, double d, double dx) {
  const double dx2 = dx * dx;
  return a + b * dx + c * dx2 + d * (dx2 * dx);
}
__device__ __forceinline__ int cs_walk_wave(const RacelineK& rl, const MuBracket& br, const double* kn,
                                            const double* spd, const double* prefix, const double* dist, int segs,
                                            int p0, double px, double py, double v0, double scale, double Ts, int H,
                                            double* sx, double* vr) {
  const int lane = (int)threadIdx.x & 63;
  const int m = rl.n - 1;
  const int pj = segs >= 1 ? p0 + np_argmin(dist, segs) : p0;
  const double L = kn[m];
  double s = prefix[pj];
  double v = fmax(v0, 0.01);                                        // planner.py:34
  // the start segment: bisect-right on the knots clamped to [0, m - 1] = the count of
  // knots[i] <= s over i in [1, m - 1] (ascending knots)
  int cnt = 0;
  for (int i = 1 + lane; i <= m - 1; i += 64) cnt += (int)(kn[i] <= s);
  int seg = wave_sum(cnt);
  double kseg = kn[seg];
  // a single profile (mu outside the table) has wa = 1, wb = 0, den = 1: v = v_lo exactly
  // (both rows hold it), so no branch keeps the second cubic's reads behind the first
  const double wa = br.wa, wb = br.wb, den = br.den, rden = 1.0 / den;
  // the register window: lane j <- segment w0 + j (cubics of min(w0 + j, m - 1), as before)
  int w0 = 0;
  double wk, c0, c1, c2, c3, c4, c5, c6, c7;
  auto load_win = [&](int base) {
    w0 = base;
    const int sj = base + lane;
    wk = sj <= m ? kn[sj] : __builtin_inf();
    const int sl = sj < m - 1 ? sj : m - 1;
    const double2* c = reinterpret_cast<const double2*>(spd + 8 * (size_t)sl);
    const double2 q0 = c[0], q1 = c[1], q2 = c[2], q3 = c[3];
    c0 = q0.x;
    c1 = q0.y;
    c2 = q1.x;
    c3 = q1.y;
    c4 = q2.x;
    c5 = q2.y;
    c6 = q3.x;
    c7 = q3.y;
  };
  load_win(seg);
  CTL_STAMP(blockIdx.x, 17);
  int myseg = 0;                                                    // lane k: step k's segment, dx
  double mydx = 0.0, v1 = 0.0;
  for (int k = 0; k < H; ++k) {
    double t = s + scale * v * Ts;                                  // :41
    if (!(t >= 0.0 && t < L)) {                                     // :42 Python float %
      double r = fmod(t, L);
      if (r != 0.0 && r < 0.0) r += L;
      t = (r == 0.0) ? 0.0 : r;
    }
    s = t;
    if (t < kseg) {                                                 // wrapped past the lap end
      seg = 0;
      kseg = kn[0];
    }
    int rel = seg - w0;
    if (rel < 0 || rel + kWalkAhead > 63) {                         // wave-uniform: move the window
      load_win(seg);
      rel = 0;
    }
    double dl = t - wk;
    const double vb = cubic4(c0, c1, c2, c3, dl);
    const double va = cubic4(c4, c5, c6, c7, dl);
    double vl = div_by(vb * wa, den, rden) + div_by(va * wb, den, rden);
    const int adv = __popcll(__ballot(lane > rel && lane <= rel + kWalkAhead && wk <= t));
    double dx;
    if (__builtin_expect(adv < kWalkAhead, 1)) {                    // wave-uniform
      const int ch = rel + adv;
      v = readlane_d(vl, ch);
      kseg = readlane_d(wk, ch);
      dx = readlane_d(dl, ch);
      seg += adv;
    } else {                                                        // past the candidates: serial
      int sg = seg + kWalkAhead;
      while (sg < m - 1 && kn[sg + 1] <= t) ++sg;
      kseg = kn[sg];
      dx = t - kseg;
      const double* c = spd + 8 * (size_t)sg;
      const double b = spline4(c, dx);
      const double a = spline4(c + 4, dx);
      v = div_by(b * wa, den, rden) + div_by(a * wb, den, rden);
      seg = sg;
    }
    if (lane == k) {
      myseg = seg;
      mydx = dx;
    }
    if (k == 0) v1 = v;
  }
  CTL_STAMP(blockIdx.x, 18);
  if (lane == 0) {
    sx[0] = px;                                                     // planner.py:33
    sx[1] = py;
    *vr = v1 * scale;
  }
  if (lane < H) {                                                   // :43 calc_position
    sx[2 * (lane + 1)] = spline_at(rl.xy, m, myseg, mydx);
    sx[2 * (lane + 1) + 1] = spline_at(rl.xy + 4 * (size_t)m, m, myseg, mydx);
  }
  return pj;
}

// ------------------------------------------------------------------------------------
// A look-ahead block: the tick's reference and candidates (redundantly per block: they only
// read the state and the tables), then its slots' rollouts.
// ------------------------------------------------------------------------------------
// Waves 1-3 of a look-ahead block while wave 0 walks: an arrival count in LDS joins them (a
// block barrier would wait for the walk).  Every wave's LDS stores are complete before it
// arrives; the count only grows within a launch (targets 3, 6).
__device__ __forceinline__ void ctl_group_sync(int* arrived, int target) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(arrived, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(arrived, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
  }
}

// The staged look-ahead inputs (s4; waves 1-3, t in [0, 192), after the rate clip): sin / cos
// delta of every (candidate, step) — make_input_fast's values — and per candidate the
// rollout's input-rate cost sum (act_term over k in order from 0, nmpc.py:65-68, 111) and
// its feasibility (1 / 0, nmpc.py:102-105; NaN: a steering outside sincos_fast's domain, so
// the rollout re-runs in the general evaluation).  The same arithmetic as the unstaged step.
__device__ __forceinline__ void ctl_stage(const CtlLaunch& c, const double* Ul, double* s4, int t, double up0,
                                          double up1) {
  const int H = c.la.H, C = c.la.C;
  constexpr int kThreads = kBlock - 64;
  const int ns = C < kThreads / 2 ? C : kThreads / 2;                 // threads summing per candidate
  if (t < ns) {
    const CostK q = c.la.cost;          // a copy: a reference into the kernel argument made
                                        // the compiler copy the whole argument to scratch
    for (int cc = t; cc < C; cc += ns) {
      const double* u = Ul + 2 * (size_t)cc * H;
      double act = 0.0, p0 = up0, p1 = up1;
      bool feas = true, bad = false;
      for (int k = 0; k < H; ++k) {
        const double ua = u[2 * k], ud = u[2 * k + 1];
        const double d0 = ua - p0, d1 = ud - p1;
        if (q.enforce) feas = (int)feas & (int)input_feasible(q, ua, ud, d0, d1);
        act = act + act_term(q, d0, d1);
        bad = (int)bad | (int)!fm::sincos_fast_ok(ud);
        p0 = ua;
        p1 = ud;
      }
      *reinterpret_cast<double2*>(s4 + 2 * (size_t)C * H + 2 * cc) =
          double2{act, bad ? __builtin_nan("") : (feas ? 1.0 : 0.0)};
    }
  } else {
    const fm::FmK K = fm::FmK::load();
    for (int f = t - ns; f < C * H; f += kThreads - ns) {
      double sd, cd;
      fm::sincos_fast(Ul[2 * f + 1], &sd, &cd, K);
      *reinterpret_cast<double2*>(s4 + 2 * (size_t)f) = double2{sd, cd};
    }
  }
}

template <int LPM>
__device__ __forceinline__ void ctl_lookahead(const CtlLaunch& c, int blk, unsigned char* smem, const Scratch& sc) {
  const int tid = threadIdx.x;
  const int H = c.la.H, C = c.la.C;
  const RacelineK rl = c.la.rl;
  const CtlLds L = ctl_lds(H, C, rl.n, c.s4 != 0);
  double* sx = reinterpret_cast<double*>(smem + L.sx);
  double* Ul = reinterpret_cast<double*>(smem + L.ul);
  double* kn = reinterpret_cast<double*>(smem + L.kn);
  double* spd = reinterpret_cast<double*>(smem + L.spd);
  double* dist = reinterpret_cast<double*>(smem + L.misc);              // [16]
  uint32_t* slot_id = reinterpret_cast<uint32_t*>(smem + L.misc + 128);   // [mpb] (<= 64)
  int32_t* sel_late = reinterpret_cast<int32_t*>(smem + L.misc + 384);    // [mpb]
  double* x0 = reinterpret_cast<double*>(smem + L.misc + 640);            // [6] x_t (no kernarg address taken)
  int* arrived = reinterpret_cast<int*>(smem + L.misc + 688);              // waves 1-3 (ctl_group_sync)
  double* s4 = reinterpret_cast<double*>(smem + L.s4);                      // s4: the staged inputs
  int* door_res = reinterpret_cast<int*>(smem + L.misc + 720);
  CTL_STAMP(blockIdx.x, 0);
  const bool armed = c.door != nullptr;
  if (!armed && tid < 6) x0[tid] = ctl_xt(c, tid);
  if (tid == 0) *arrived = 0;
  const CtlState* st = c.st;
  const double* prev_seq = st->has_seq ? &st->useq[0][0] : nullptr;
  // rt.py:278-282: projidx and the mu bracket (mu-hat or the fixed mu) come from the host's
  // copy of the state (CtlLaunch.p0_walk / br_walk): the tables' loads follow the kernel
  // arguments directly (profiles/r04/s4/ctl_phases_prologue.txt: 2.5 us to the bracket before).
  // An armed launch reads the state itself: the previous tick ended before it started, and
  // the loads sit before the doorbell.
  // (values, not pointers, are selected — the empty asm keeps the compiler from loading through a
  // select of the state's and the kernel argument's addresses, which copies the whole argument
  // to scratch)
  int p0 = c.p0_walk;
  double mu_k = c.mu_fixed;
  asm volatile("" : "+s"(p0));
  asm volatile("" : "+v"(mu_k));
  if (armed) {
    p0 = st->projidx;
    if (c.use_mu) mu_k = st->mu_pred;
  }
  const double scale = c.use_mu ? c.v_factor : c.scale_fixed;
  const MuBracket br = armed ? mu_bracket(rl.mus, rl.M, mu_k) : c.br_walk;
  CTL_STAMP(blockIdx.x, 14);
  // waves 1-3: this tick's candidate variates (the previous tick's completion drew them) are
  // loaded now, their latency under the tables' (used only when their tag matches: ctl_draw)
  constexpr int kZPre = 16;
  const int CH = C * H;
  const bool zfit = c.znoise != nullptr && CH <= kZPre * (kBlock - 64);
  double zr[kZPre][2];
  if (tid >= 64 && zfit) {
    const double* zb = c.znoise + 2 * (size_t)CH * (int)(c.tick & 1);
#pragma unroll
    for (int i = 0; i < kZPre; ++i) {
      const int p = tid - 64 + i * (kBlock - 64);
      const int pc = p < CH ? p : CH - 1;
      zr[i][0] = zb[2 * pc];
      zr[i][1] = zb[2 * pc + 1];
    }
  }
  // (a) tables: knots, x/y rows, the two speed profiles bracketing mu (cs_stage); (b)
  //     project_fast of x_t on raceline[:, p0 : p0 + 10] (track.py:147-160)
  cs_stage(rl, br, kn, spd);
  CTL_STAMP(blockIdx.x, 15);
  double px = 0.0, py = 0.0, pv = 0.0;
  if (armed) {                          // x_t: the doorbell (x0 in LDS after its barrier)
    if (ctl_door(c, x0, door_res) != (int)kCtlDoorFire) return;
    px = x0[0];
    py = x0[1];
    pv = x0[3];
  } else {
    px = c.x_t[0];
    py = c.x_t[1];
    pv = c.x_t[3];
    asm volatile("" : "+v"(px), "+v"(py), "+v"(pv));
  }
  const int segs = cs_project(c.pts, c.np, p0, px, py, dist);
  __syncthreads();
  CTL_STAMP(blockIdx.x, 1);
  // (c) wave 0 walks ConstantSpeed from the projection (planner.py:24-65) while waves 1-3
  //     draw the candidates before the rate clip, every (c, k, j)
  const double up0 = st->u_prev[0], up1 = st->u_prev[1];
  if (tid < 64) {
    double vr;
    (void)cs_walk_wave(rl, br, kn, spd, c.prefix, dist, segs, p0, px, py, pv, scale, c.la.Ts, H, sx, &vr);
    CTL_STAMP(blockIdx.x, 10);
  } else {
    if (zfit && c.ztag[(int)(c.tick & 1)] == c.tick + 1) {          // launch-uniform
      const double up[2] = {up0, up1};
#pragma unroll
      for (int i = 0; i < kZPre; ++i) {
        const int p = tid - 64 + i * (kBlock - 64);
        if (p < CH) {
          const int cc = p / H, k = p - cc * H;
          ctl_cand_pair_z(cc, k, H, prev_seq, up, c.nscale, c.umin, c.umax, zr[i][0], zr[i][1], Ul + 2 * (size_t)p);
        }
      }
    } else {
      ctl_draw(c, prev_seq, up0, up1, Ul, tid - 64, kBlock - 64);
    }
    if (c.s4) {                         // block-uniform: still during the walk, clip and stage
      ctl_group_sync(arrived, kWaves - 1);
      for (int t = tid - 64; t < 2 * C; t += kBlock - 64) {
        const int j = t & 1;
        ctl_rate_chain(Ul + 2 * (size_t)(t >> 1) * H + j, H, j ? up1 : up0, j ? c.rate[1] : c.rate[0]);
      }
      ctl_group_sync(arrived, 2 * (kWaves - 1));
      ctl_stage(c, Ul, s4, tid - 64, up0, up1);
    }
  }
  __syncthreads();
  CTL_STAMP(blockIdx.x, 2);
  // speculative look-ahead (c.n_spec): the first block publishes the reference for the spec
  // blocks' deferred costs, and wave 1 of every block loads the spec list (its models' results
  // come from the spec blocks)
  uint32_t* spec_ids = reinterpret_cast<uint32_t*>(smem + L.misc + 768);   // [kCtlSpecMax]
  if (c.n_spec) {
    if (blk == 0 && tid < 2 * (H + 1)) {
      const uint64_t v = (uint64_t)__double_as_longlong(sx[tid]);
      st_wt(&c.xref_tag[2 * tid], tag_word(c.seq, (uint32_t)(v >> 32)));
      st_wt(&c.xref_tag[2 * tid + 1], tag_word(c.seq, (uint32_t)v));
    }
    if (tid >= 64 && tid < 64 + c.n_spec) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t v = kNoLocal;
      for (;;) {
        const uint64_t w = ld_wt(&c.spec_tag[tid - 64]);
        if (tag_ok(w, c.seq)) {
          v = (uint32_t)w;
          break;
        }
        if (ctl_late(t0, c.poll)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      spec_ids[tid - 64] = v;
    }
  }
  // (d) waves 1-3 clip the candidates' rates; meanwhile (e) wave 0 takes this block's slots:
  //     the selection (tagged words of the look-back ticket winner), or the nominal model
  //     while the window fills
  const int mpb = c.mpb;
  if (!c.s4 && tid >= 64) {
    for (int t = tid - 64; t < 2 * C; t += kBlock - 64) {
      const int j = t & 1;
      ctl_rate_chain(Ul + 2 * (size_t)(t >> 1) * H + j, H, j ? up1 : up0, j ? c.rate[1] : c.rate[0]);
    }
  }
  if (tid < mpb) {                      // wave 0 (mpb <= 64): this block's slots
    const int slot = blk * mpb + tid;
    uint32_t id = kNoLocal;
    int late = 0;
    if (slot < c.nslots) {
      if (c.warm) {
        id = 0;
      } else {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const uint64_t w = ld_wt(&c.sel_tag[slot]);
          if (tag_ok(w, c.seq)) {
            id = (uint32_t)w;
            break;
          }
          if (ctl_late(t0, c.poll)) {
            late = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    slot_id[tid] = id;
    sel_late[tid] = late;
  }
  __syncthreads();
  if (c.n_spec) {                       // launch-uniform: a slot whose model a spec block rolls out: bit 1
    if (tid < 64) {
      const int lane = tid;
      for (int q = 0; q < mpb; ++q) {
        const uint32_t sid = slot_id[q];
        const bool hit = __ballot(lane < c.n_spec && sid != kNoLocal && spec_ids[lane] == sid) != 0;
        if (lane == 0 && hit) sel_late[q] |= 2;
      }
    }
    __syncthreads();
  }
  CTL_STAMP(blockIdx.x, 3);
  if (c.dbg && blk == 0) {              // tests: this tick's reference and candidates
    for (int e = tid; e < 2 * (H + 1); e += kBlock) {
      const int row = e / (H + 1), k = e - row * (H + 1);
      c.dbg[e] = sx[2 * k + row];
    }
    for (int e = tid; e < 2 * C * H; e += kBlock) c.dbg[2 * (H + 1) + e] = Ul[e];
  }
  // (f) rollouts: lane layout of the plan kernel's look-ahead (G candidate lanes per model,
  //     LPM lanes per rollout)
  const int G = c.G, cpl = c.cpl;
  const int sub = tid % LPM, cl = tid / LPM, g = cl & (G - 1), si = cl / G;
  const int slot = blk * mpb + si;
  const uint32_t id = si < mpb ? slot_id[si] : kNoLocal;
  const bool spec_hit = si < mpb && (sel_late[si] & 2);
  const bool live = slot < c.nslots && id != kNoLocal && !spec_hit;
  Tire t{};
  if (live) {
    if (c.warm) {
      t.Bf = c.nominal[0];
      t.Cf = c.nominal[1];
      t.Df = c.nominal[2];
      t.Br = c.nominal[3];
      t.Cr = c.nominal[4];
      t.Dr = c.nominal[5];
    } else {
      t = load_tire(c.la.params, c.la.n, id);
    }
  }
  CostK q = c.la.cost;
  VehK veh = c.la.veh;
  double Ts = c.la.Ts;
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
  pin_vgpr(veh.lf);
  pin_vgpr(veh.lr);
  pin_vgpr(veh.mass);
  pin_vgpr(veh.inv_mass);
  pin_vgpr(veh.inv_Iz);
  pin_vgpr(veh.Cm1);
  pin_vgpr(veh.Cm2);
  pin_vgpr(veh.Cr0);
  pin_vgpr(veh.Cr2);
  pin_vgpr(Ts);
  double bv = __builtin_nan("");
  int64_t bc = kNoIndex;
  int nf = 0;
  constexpr bool kSplit = (LPM == 4);
  const bool diagQP = c.la.cost.Q[1] == 0.0 && c.la.cost.Q[2] == 0.0 && c.la.cost.P[1] == 0.0 && c.la.cost.P[2] == 0.0;
  if (live) {
    constexpr bool kScaled = scaled_yaw(LPM);
    StageK sk = make_stage<LPM>(veh, t, sub, Ts);
    if (kScaled) sk.ch[0].lw = sk.ch[0].lw / Ts;
    if (kScaled && LPM == 1) sk.ch[1].lw = sk.ch[1].lw / Ts;
    if (kScaled && LPM == 4 && sub >= 2) {   // lanes 2/3: zero-operand chains (plan kernel)
      sk.ch[0].lw = 0.0;
      sk.ch[0].sg = 0.0;
      sk.ch[0].B = 0.0;
      sk.ch[0].nsB = 0.0;
    }
    const FusedK fq = make_fused(veh, sk, Ts, kScaled);
    const fm::FmK K = fm::FmK::load<kLeanLA>();
    for (int j = 0; j < cpl; ++j) {
      const int cc = g + j * G;
      if (cc >= C) break;
      bool bad = false;
      double J;
      if (c.s4) {                       // block-uniform: the staged input terms
        if (kSplit && diagQP)
          J = rollout<0, false, LPM, 0, true, kSplit, true, false, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts,
                                                                        up0, up1, K, fq, bad, nullptr, s4);
        else
          J = rollout<0, false, LPM, 0, true, false, true, false, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts,
                                                                       up0, up1, K, fq, bad, nullptr, s4);
      } else if (kSplit && diagQP) {
        J = rollout<0, false, LPM, 0, true, kSplit, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts, up0, up1, K,
                                                         fq, bad);
      } else {
        J = rollout<0, false, LPM, 0, true, false, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts, up0, up1, K,
                                                        fq, bad);
      }
      if (LPM == 2) {
        const int bi = bad;
        bad = __builtin_amdgcn_mov_dpp(bi, kPair0, 0xF, 0xF, false) | __builtin_amdgcn_mov_dpp(bi, kPair1, 0xF, 0xF, false);
      } else if (LPM == 4) {
        int bi = bad;
        bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
        bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
        bad = bi;
      }
      if (__builtin_expect(__any(bad), 0)) {
        bool unused = false;
        if (bad)
          J = rollout<0, false, LPM, 0, false, false, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts, up0, up1, K,
                                                           fq, unused);
      }
      if (sub == 0) nf += !isfinite(J);
      if (less_nan_last(J, cc, bv, bc)) {
        bv = J;
        bc = cc;
      }
    }
  }
  CTL_STAMP(blockIdx.x, 4);
  // (g) per-slot argmin over its candidates and non-finite count: xor shuffles inside a wave,
  //     then across the slot's waves in LDS (a slot of 2 or 4 waves: G LPM in {128, 256})
  const int span = G * LPM;
  for (int off = (span < 64 ? span : 64) >> 1; off >= LPM; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int64_t oc = __shfl_xor(bc, off, 64);
    nf += __shfl_xor(nf, off, 64);
    if (less_nan_last(ov, oc, bv, bc)) {
      bv = ov;
      bc = oc;
    }
  }
  if (span > 64) {                      // block-uniform
    if ((tid & 63) == 0) {
      sc.sv[tid >> 6] = bv;
      sc.si[tid >> 6] = bc;
      sc.sn[tid >> 6] = nf;
    }
    __syncthreads();
    const int w0 = (tid / span) * (span / 64);
    bv = sc.sv[w0];
    bc = sc.si[w0];
    nf = sc.sn[w0];
    for (int k = 1; k < span / 64; ++k) {
      nf += sc.sn[w0 + k];
      if (less_nan_last(sc.sv[w0 + k], sc.si[w0 + k], bv, bc)) {
        bv = sc.sv[w0 + k];
        bc = sc.si[w0 + k];
      }
    }
  }
  // (h) publish: cost (hi, lo), candidate, non-finite count | late << 31 (tagged words)
  if (g == 0 && sub == 0 && si < mpb && slot < c.nslots && !spec_hit) {
    const uint64_t vb = (uint64_t)__double_as_longlong(bv);
    const uint32_t nfw = (uint32_t)nf | ((uint32_t)(sel_late[si] & 1) << 31);
    uint64_t* w = c.slot_tag + 4 * (size_t)slot;
    st_wt(&w[0], tag_word(c.seq, (uint32_t)(vb >> 32)));
    st_wt(&w[1], tag_word(c.seq, (uint32_t)vb));
    st_wt(&w[2], tag_word(c.seq, (uint32_t)(int32_t)bc));
    st_wt(&w[3], tag_word(c.seq, nfw));
  }
  CTL_STAMP(blockIdx.x, 5);
}

// A spec block: model spec_tag[j] x the C candidates from the doorbell on (ctl.hpp
// CtlLaunch.n_spec).  Before the doorbell: the candidates (the look-ahead blocks' generator, so
// the same sequences), the rate clip, the staged terms, the model.  Then the rollouts with the
// tracking cost deferred (rollout<DEFER>), the reference from the first look-ahead block's walk
// (xref_tag), defer_cost, and the block's best candidate as ctl_lookahead publishes a slot.
// LPM 4 with diagonal Q / P only (the host enables spec blocks for that layout).
template <int LPM>
__device__ __forceinline__ void ctl_spec(const CtlLaunch& c, int j, unsigned char* smem, const Scratch& sc) {
  if constexpr (LPM != 4) {
    return;
  } else {
    const int tid = threadIdx.x;
    const int H = c.la.H, C = c.la.C;
    const SpecLds S = spec_lds(H, C);
    double* sx = reinterpret_cast<double*>(smem + S.sx);
    double* Ul = reinterpret_cast<double*>(smem + S.ul);
    double* s4 = reinterpret_cast<double*>(smem + S.s4);
    double* pos = reinterpret_cast<double*>(smem + S.pos);
    double* junk = reinterpret_cast<double*>(smem + S.junk);
    double* x0 = reinterpret_cast<double*>(smem + S.misc);            // [6]
    int* door_res = reinterpret_cast<int*>(smem + S.misc + 64);
    uint32_t* sid = reinterpret_cast<uint32_t*>(smem + S.misc + 80);
    const CtlState* st = c.st;
    const double* prev_seq = st->has_seq ? &st->useq[0][0] : nullptr;
    const double up0 = st->u_prev[0], up1 = st->u_prev[1];
    ctl_draw(c, prev_seq, up0, up1, Ul, tid, kBlock);
    __syncthreads();
    for (int t = tid; t < 2 * C; t += kBlock) {
      const int jj = t & 1;
      ctl_rate_chain(Ul + 2 * (size_t)(t >> 1) * H + jj, H, jj ? up1 : up0, jj ? c.rate[1] : c.rate[0]);
    }
    __syncthreads();
    if (tid >= 64) ctl_stage(c, Ul, s4, tid - 64, up0, up1);      // waves 1-3, as the look-ahead blocks
    if (tid == 0) {                     // the model (the spec merge publishes before the doorbell)
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t id = kNoLocal;
      for (;;) {
        const uint64_t w = ld_wt(&c.spec_tag[j]);
        if (tag_ok(w, c.seq)) {
          id = (uint32_t)w;
          break;
        }
        if (ctl_late(t0, 2 * c.door_bound)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      *sid = id;
    }
    __syncthreads();
    const uint32_t id = *sid;
    if (id == kNoLocal) return;         // block-uniform: fewer models than spec blocks
    const Tire t = load_tire(c.la.params, c.la.n, id);
    if (ctl_door(c, x0, door_res) != (int)kCtlDoorFire) return;
    CTL_STAMP(blockIdx.x, 19);
    const int G = c.G, cpl = c.cpl;
    const int sub = tid % LPM, cl = tid / LPM, g = cl & (G - 1);
    CostK q = c.la.cost;
    VehK veh = c.la.veh;
    double Ts = c.la.Ts;
    for (int m = 0; m < 4; ++m) {
      pin_vgpr(q.Q[m]);
      pin_vgpr(q.R[m]);
      pin_vgpr(q.P[m]);
    }
    pin_vgpr(veh.lf);
    pin_vgpr(veh.lr);
    pin_vgpr(veh.mass);
    pin_vgpr(veh.inv_mass);
    pin_vgpr(veh.inv_Iz);
    pin_vgpr(veh.Cm1);
    pin_vgpr(veh.Cm2);
    pin_vgpr(veh.Cr0);
    pin_vgpr(veh.Cr2);
    pin_vgpr(Ts);
    constexpr bool kScaled = scaled_yaw(LPM);
    StageK sk = make_stage<LPM>(veh, t, sub, Ts);
    if (kScaled) sk.ch[0].lw = sk.ch[0].lw / Ts;
    if (kScaled && sub >= 2) {          // lanes 2/3: zero-operand chains (plan kernel)
      sk.ch[0].lw = 0.0;
      sk.ch[0].sg = 0.0;
      sk.ch[0].B = 0.0;
      sk.ch[0].nsB = 0.0;
    }
    const FusedK fq = make_fused(veh, sk, Ts, kScaled);
    const fm::FmK K = fm::FmK::load<kLeanLA>();
    const double Qd = sk.pc ? q.Q[3] : q.Q[0], Pd = sk.pc ? q.P[3] : q.P[0];
    // cpl == 1 with G == C (the host's layout for spec blocks): candidate g in quad g
    const int cc = g;
    double* dp = sub < 2 ? pos + (size_t)(2 * cc + sub) * H : junk + (tid & 63);
    const int ds = sub < 2 ? 1 : 0;
    bool bad = false;
    DeferOut d{};
    (void)cpl;
    (void)rollout<0, false, LPM, 0, true, true, true, false, true, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts,
                                                                         up0, up1, K, fq, bad, nullptr, s4, dp, ds,
                                                                         &d);
    CTL_STAMP(blockIdx.x, 20);
    // the reference: the walker's tagged halves (its walk ended long before these rollouts)
    {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (int e = tid; e < 2 * (H + 1); e += kBlock) {
        uint64_t hi, lo;
        for (;;) {
          hi = ld_wt(&c.xref_tag[2 * e]);
          lo = ld_wt(&c.xref_tag[2 * e + 1]);
          if ((int)tag_ok(hi, c.seq) & (int)tag_ok(lo, c.seq)) break;
          if (ctl_late(t0, c.poll)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        sx[e] = __longlong_as_double((long long)join_words(hi, lo));
      }
    }
    __syncthreads();
    double J = defer_cost(dp, ds, sx, H, sk.pc, Qd, Pd, d, sk.sok, bad);
    {
      int bi = bad;
      bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
      bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
      bad = bi;
    }
    if (__builtin_expect(__any(bad), 0)) {
      bool unused = false;
      if (bad)
        J = rollout<0, false, LPM, 0, false, false, true>(c.la, cc, 0, x0, sx, Ul, veh, t, sk, q, Ts, up0, up1, K, fq,
                                                         unused);
    }
    double bv = __builtin_nan("");
    int64_t bc = kNoIndex;
    int nf = 0;
    if (sub == 0) nf += !isfinite(J);
    if (less_nan_last(J, cc, bv, bc)) {
      bv = J;
      bc = cc;
    }
    // the block's argmin over its C candidates and non-finite count (ctl_lookahead's (g))
    const int span = G * LPM;
    for (int off = (span < 64 ? span : 64) >> 1; off >= LPM; off >>= 1) {
      const double ov = __shfl_xor(bv, off, 64);
      const int64_t oc = __shfl_xor(bc, off, 64);
      nf += __shfl_xor(nf, off, 64);
      if (less_nan_last(ov, oc, bv, bc)) {
        bv = ov;
        bc = oc;
      }
    }
    if (span > 64) {                    // block-uniform
      if ((tid & 63) == 0) {
        sc.sv[tid >> 6] = bv;
        sc.si[tid >> 6] = bc;
        sc.sn[tid >> 6] = nf;
      }
      __syncthreads();
      const int w0 = (tid / span) * (span / 64);
      bv = sc.sv[w0];
      bc = sc.si[w0];
      nf = sc.sn[w0];
      for (int k = 1; k < span / 64; ++k) {
        nf += sc.sn[w0 + k];
        if (less_nan_last(sc.sv[w0 + k], sc.si[w0 + k], bv, bc)) {
          bv = sc.sv[w0 + k];
          bc = sc.si[w0 + k];
        }
      }
    }
    if (tid == 0) {
      const uint64_t vb = (uint64_t)__double_as_longlong(bv);
      uint64_t* w = c.spec_res + 4 * (size_t)j;
      st_wt(&w[0], tag_word(c.seq, (uint32_t)(vb >> 32)));
      st_wt(&w[1], tag_word(c.seq, (uint32_t)vb));
      st_wt(&w[2], tag_word(c.seq, (uint32_t)(int32_t)bc));
      st_wt(&w[3], tag_word(c.seq, (uint32_t)nf));
    }
    CTL_STAMP(blockIdx.x, 21);
  }
}

}  // namespace

// PX: the sharded controller (ctl_exchange after the shard's lb_final) — its own
// instantiation, so the unsharded tick's code is unchanged
template <int LPM, bool PX>
__global__ __launch_bounds__(kBlock) void ctl_kernel(CtlLaunch arg) {
  // the argument read in place from the kernarg segment (it is the launch's first and only
  // explicit argument): referencing the by-value parameter itself made the compiler copy all
  // 1.4 KB of it to scratch once the kernel grew
  (void)arg;
  const CtlLaunch& c = *(const CtlLaunch*)__builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Scratch sc(smem);
  int* flag = reinterpret_cast<int*>(smem + kFlagOff);
  const int blk = (int)blockIdx.x;
  // x_t in the argument: the device time starts here (a gathered tick's: at its first launch)
  if (blk == 0 && threadIdx.x == 0 && !c.door && !(PX && c.px_phase == 2))
    st_wt(&c.door_dev[kCtlTimeWord], (uint64_t)__builtin_amdgcn_s_memrealtime());
  if (blk >= c.nb_lb + c.nb_la) {       // spec blocks (CtlLaunch.n_spec), last in the grid
    ctl_spec<LPM>(c, blk - c.nb_lb - c.nb_la, smem, sc);
    return;
  }
  if (blk >= c.nb_lb) {
    ctl_lookahead<LPM>(c, blk - c.nb_lb, smem, sc);
    return;
  }
  unsigned char* pl = smem + c.poll_off;
  CtlSel cs{c.sel_tag, c.seq, reinterpret_cast<uint32_t*>(pl + 2048), reinterpret_cast<double*>(pl + 2304),
            reinterpret_cast<double*>(pl + 2624), reinterpret_cast<double*>(pl + 3200),
            reinterpret_cast<int32_t*>(pl + 3520)};
  if (threadIdx.x == 0) *cs.xlate = 0;
  // x_t through LDS (pointing into the kernel argument itself would make the compiler copy the
  // whole argument to scratch): the kernel argument, or an armed launch's doorbell — after the
  // look-back's step, which needs only the state (lookback_block<ARMED>)
  double* xl = reinterpret_cast<double*>(pl + 3072);
  auto door = [&](double pred, bool pvalid, int64_t pn) -> const double* {
    // the speculative look-ahead's ranking first: it needs only the window (before x_t)
    if (c.n_spec) ctl_spec_lists<PX>(c, blk, pred, pvalid, pn, smem, flag);
    if (c.door) {
      const int r = ctl_door(c, xl, reinterpret_cast<int*>(pl + 3584));
      if (r != (int)kCtlDoorFire) {     // cancelled or expired: nothing touched
        if (r == (int)kCtlDoorExpired && blk == 0 && threadIdx.x == 0)
          __hip_atomic_store(c.host_tag, c.host_seq | kCtlTagExpired, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return nullptr;
      }
    } else {
      if (threadIdx.x < 6) xl[threadIdx.x] = ctl_xt(c, (int)threadIdx.x);
      __syncthreads();
    }
    return xl;
  };
  if (PX && c.px_phase == 2) {         // a gathered tick's second launch: block 0 merges, completes
    if (!door(0.0, false, 0)) return;
    ctl_exchange(c, smem, cs);
    __threadfence_system();             // the record's look-back half (pinned host memory)
    __syncthreads();
  } else if (c.do_lb) {
    LookbackLaunch lb = c.lb;           // x_prev / u_prev: the state
    CTL_STAMP(blk, 0);
    if (!lookback_block<true>(lb, blk, sc, door)) return;
    CTL_STAMP(blk, 6);
    if (!ticket_last(&c.tickets[0], (unsigned)c.nb_lb, flag)) return;
    if (c.full) {
      if constexpr (PX) {
        lb_final<2>(c.fin, smem, &cs);  // this shard's lists, then the exchange and the merge
        if (c.px_phase == 1) {          // gathered: the record out, the rest in the second launch
          ctl_px_send(c, cs);
          return;
        }
        ctl_exchange(c, smem, cs);
      } else {
        lb_final<1>(c.fin, smem, &cs);
      }
      __threadfence_system();           // the record's look-back half (pinned host memory)
    }
    CTL_STAMP(blk, 7);
    __syncthreads();
  } else if (!door(0.0, false, 0)) {    // ticks without a look-back: block 0 only completes
    return;
  }
  ctl_complete(c, smem, cs, xl);
}

// llampc_ctl_reference: ConstantSpeed alone (one block), into out = xref [2][H+1], projidx,
// vr.  LDS: xref | knots | two profiles | dists (the controller's layout with C = 0).
__global__ __launch_bounds__(kBlock) void cs_kernel(CsLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const CtlLds L = ctl_lds(a.H, 0, a.rl.n);
  double* sx = reinterpret_cast<double*>(smem + L.sx);
  double* kn = reinterpret_cast<double*>(smem + L.kn);
  double* spd = reinterpret_cast<double*>(smem + L.spd);
  double* dist = reinterpret_cast<double*>(smem + L.misc);
  const MuBracket br = mu_bracket(a.rl.mus, a.rl.M, a.mu);
  cs_stage(a.rl, br, kn, spd);
  const int segs = cs_project(a.pts, a.np, a.p0, a.x0, a.y0, dist);
  __syncthreads();
  if (threadIdx.x < 64) {                // wave 0 walks (the controller tick's walker)
    double vr = 0.0;
    const int pj = cs_walk_wave(a.rl, br, kn, spd, a.prefix, dist, segs, a.p0, a.x0, a.y0, a.v0, a.scale, a.Ts,
                                a.H, sx, &vr);
    if (threadIdx.x == 0) {
      a.out[2 * (a.H + 1)] = (double)pj;
      a.out[2 * (a.H + 1) + 1] = vr;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * (a.H + 1); e += kBlock) {
    const int row = e / (a.H + 1), k = e - row * (a.H + 1);
    a.out[e] = sx[2 * k + row];
  }
}

hipError_t launch_constant_speed(const CsLaunch& a, hipStream_t s) {
  const CtlLds L = ctl_lds(a.H, 0, a.rl.n);
  allow_lds(cs_kernel);
  hipLaunchKernelGGL(cs_kernel, dim3(1), dim3(kBlock), L.end, s, a);
  return hipGetLastError();
}

size_t ctl_lds_bytes(int H, int C, int n, int nb_lb, int K, size_t* poll_off, bool s4, int px_G, int n_spec) {
  const CtlLds L = ctl_lds(H, C, n, s4);
  const size_t M = (size_t)nb_lb * K, Lb = nb_lb;    // lb_final's region (launch_plan's formula)
  const size_t lbf = kScratchBytes + 8 * (3 * M + Lb) + sizeof(Ent) * Lb * kWaves + 4 * (3 * M + Lb + LLAMPC_KMAX + 2) + 8 + 16;
  const size_t rank = kScratchBytes + (size_t)kWaves * kRankBytes + kBlockMergeBytes;
  const size_t px = px_G ? kScratchBytes + ctl_px_bytes(px_G, K) : 0;   // ctl_exchange's region
  // the speculative look-ahead: a spec block's layout, the look-back blocks' ranking and the
  // spec merge's two list buffers
  // (sharded: then the ranks' lists, ctl_spec_exchange)
  const size_t spec_px = px_G ? align16(2 * sizeof(Ent) * Lb * n_spec) + align16(16 * (size_t)px_G * n_spec) +
                                    2 * sizeof(Ent) * (size_t)px_G * n_spec
                              : 0;
  const size_t spec = n_spec ? std::max(spec_lds(H, C).end,
                                        kScratchBytes + std::max<size_t>(std::max<size_t>(12 * kBlock, 2 * sizeof(Ent) * Lb * n_spec),
                                                                         spec_px))
                             : 0;
  size_t off = std::max(std::max(std::max(L.end, px), std::max(lbf, rank)), spec);
  off = align16(off);
  *poll_off = off;
  return off + kCtlPollBytes;
}

template <bool PX>
static void launch_ctl_px(const CtlLaunch& c, int lpm, size_t lds, hipStream_t s) {
  const dim3 grid(c.nb_lb + c.nb_la + c.n_spec), block(kBlock);
  if (lpm == 4) {
    allow_lds(ctl_kernel<4, PX>);
    hipLaunchKernelGGL((ctl_kernel<4, PX>), grid, block, lds, s, c);
  } else if (lpm == 2) {
    allow_lds(ctl_kernel<2, PX>);
    hipLaunchKernelGGL((ctl_kernel<2, PX>), grid, block, lds, s, c);
  } else {
    allow_lds(ctl_kernel<1, PX>);
    hipLaunchKernelGGL((ctl_kernel<1, PX>), grid, block, lds, s, c);
  }
}

hipError_t launch_ctl(const CtlLaunch& c, int lpm, size_t lds, hipStream_t s) {
  if (c.px_G) launch_ctl_px<true>(c, lpm, lds, s);
  else launch_ctl_px<false>(c, lpm, lds, s);
  return hipGetLastError();
}

}  // namespace llampc
