// plan_dev.hpp — device code of the plan launch (look-back, look-ahead, completion,
// cross-shard merge helpers) shared by the kernel translation units.  The plan-kernel
// instantiations are spread over plan_*.hip (one TU per integrator / lanes-per-rollout
// group, compiled in parallel); kernels.hip holds the dispatcher and the other kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include <algorithm>

#include "kernels.hpp"
#include "raceline.hpp"
#include "merge.hpp"

namespace llampc {

#ifdef LLAMPC_STAMPS
// Diagnostic build only (-DLLAMPC_STAMPS, libllampc_hip_stamps.so): tid-0 stamps of
// s_memtime (shader clock) and s_memrealtime (100 MHz) at phase boundaries of the select
// kernel; never compiled into the product library.
static __device__ unsigned long long g_stamps[64][8][2];
static __device__ unsigned int g_stamp_launch;
static __device__ unsigned long long g_la_stamps[8][8][2];   // first 8 look-ahead blocks, last launch
static __device__ unsigned long long g_lb_stamps[8][8][2];   // first 8 look-back blocks, last launch
#define LB_STAMP(blk, slot)                                                              \
  do {                                                                                   \
    if (threadIdx.x == 0 && (blk) < 8) {                                                 \
      g_lb_stamps[blk][slot][0] = __builtin_amdgcn_s_memtime();                          \
      g_lb_stamps[blk][slot][1] = __builtin_amdgcn_s_memrealtime();                      \
    }                                                                                    \
  } while (0)
static __device__ unsigned long long g_la_all[1024][4][2];    // every look-ahead block, last launch
static __device__ unsigned long long g_la_wave[1024][4];      // rollout end of every look-ahead wave
static __device__ double g_rl_dbg[8];                          // raceline window decision (block 0)
static __device__ unsigned long long g_rl_ph[1024][4];         // raceline prologue phases per block
#define RL_STAMP(blk, slot)                                                              \
  do {                                                                                   \
    if (threadIdx.x == 0 && (blk) < 1024) g_rl_ph[blk][slot] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define LA_STAMP(blk, slot)                                                              \
  do {                                                                                   \
    if (threadIdx.x == 0) {                                                              \
      const unsigned long long c_ = __builtin_amdgcn_s_memtime();                        \
      const unsigned long long r_ = __builtin_amdgcn_s_memrealtime();                    \
      if ((blk) < 8) {                                                                   \
        g_la_stamps[blk][slot][0] = c_;                                                  \
        g_la_stamps[blk][slot][1] = r_;                                                  \
      }                                                                                  \
      if ((blk) < 1024) {                                                                \
        g_la_all[blk][slot][0] = c_;                                                     \
        g_la_all[blk][slot][1] = r_;                                                     \
      }                                                                                  \
    }                                                                                    \
  } while (0)
// per rollout step (FAST rollouts, thread 0 of every block < 1024): s_memtime before step k
// (k < 24) and at the loop's end (slot 24) — the first step's cold code fetch against the rest
static __device__ unsigned long long g_la_step[1024][25];
#define STEP_STAMP(k)                                                                    \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (k) <= 24)                              \
      g_la_step[blockIdx.x][k] = __builtin_amdgcn_s_memtime();                           \
  } while (0)
#define STAMP(slot)                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0) {                                                              \
      const unsigned l = g_stamp_launch & 63;                                            \
      g_stamps[l][slot][0] = __builtin_amdgcn_s_memtime();                               \
      g_stamps[l][slot][1] = __builtin_amdgcn_s_memrealtime();                           \
    }                                                                                    \
  } while (0)
// work-queue layout: per wave, per unit j < 16, (s_memtime, s_memrealtime) at [0] the unit
// taken, [1] its Pacejka row loaded, [2] rolled out, [3] done (the tagged stores issued)
static __device__ unsigned long long g_wq_unit[256][8][16][4][2];
#define WQ_STAMP(blk, j, slot)                                                           \
  do {                                                                                   \
    if ((threadIdx.x & 63) == 0 && (blk) < 256 && (j) < 16) {                            \
      g_wq_unit[blk][threadIdx.x >> 6][j][slot][0] = __builtin_amdgcn_s_memtime();       \
      g_wq_unit[blk][threadIdx.x >> 6][j][slot][1] = __builtin_amdgcn_s_memrealtime();   \
    }                                                                                    \
  } while (0)
#else
#define STEP_STAMP(k) \
  do {                \
  } while (0)
#define WQ_STAMP(blk, j, slot) \
  do {                         \
  } while (0)
#define STAMP(slot) \
  do {              \
  } while (0)
#define LA_STAMP(blk, slot) \
  do {                      \
  } while (0)
#define RL_STAMP(blk, slot) \
  do {                      \
  } while (0)
#define LB_STAMP(blk, slot) \
  do {                      \
  } while (0)
#endif

namespace {

template <int NAN_FIRST>
__device__ __forceinline__ bool kless(double av, int64_t ai, double bv, int64_t bi) {
  return NAN_FIRST ? less_nan_first(av, ai, bv, bi) : less_nan_last(av, ai, bv, bi);
}

// Cross-lane moves within rows of 16 lanes (DPP; a disabled source lane returns the lane's
// own value).  xor 1 / xor 2 = quad_perm [1,0,3,2] / [2,3,0,1]; rotate by 4 / 8 in a row.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppRor4 = 0x124, kDppRor8 = 0x128;
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  return __hiloint2double(dpp_i<CTRL>(__double2hiint(v)), dpp_i<CTRL>(__double2loint(v)));
}
template <int CTRL>
__device__ __forceinline__ int64_t dpp_l(int64_t v) {
  const uint64_t u = (uint64_t)v;
  const uint64_t lo = (uint32_t)dpp_i<CTRL>((int)(uint32_t)u), hi = (uint32_t)dpp_i<CTRL>((int)(u >> 32));
  return (int64_t)(lo | (hi << 32));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ int64_t readlane_l(int64_t v, int l) {
  const uint64_t u = (uint64_t)v;
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(u >> 32), l);
  return (int64_t)(lo | (hi << 32));
}

template <int NAN_FIRST, int CTRL>
__device__ __forceinline__ void min_step(double& v, int64_t& i) {
  const double ov = dpp_d<CTRL>(v);
  const int64_t oi = dpp_l<CTRL>(i);
  if (kless<NAN_FIRST>(ov, oi, v, i)) {
    v = ov;
    i = oi;
  }
}

// Wave-wide min of (v, i) under kless<NAN_FIRST>, the result in every lane.  ALL 64 lanes
// must be active (converged code).  DPP butterfly inside each row of 16 lanes, then the four
// row results combined from readlanes — no LDS round trips (the __shfl_xor form cost ~4k
// cycles per block reduction, SQ stamps).
template <int NAN_FIRST>
__device__ __forceinline__ void wave_min(double& v, int64_t& i) {
  min_step<NAN_FIRST, kDppXor1>(v, i);
  min_step<NAN_FIRST, kDppXor2>(v, i);
  min_step<NAN_FIRST, kDppRor4>(v, i);
  min_step<NAN_FIRST, kDppRor8>(v, i);
  double bv = readlane_d(v, 0);
  int64_t bi = readlane_l(i, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const double rv = readlane_d(v, r);
    const int64_t ri = readlane_l(i, r);
    if (kless<NAN_FIRST>(rv, ri, bv, bi)) {
      bv = rv;
      bi = ri;
    }
  }
  v = bv;
  i = bi;
}

// Branch-free ordered picks over a wave (all 64 lanes active).  A lane's candidate is
// (v, li) with li a local model index (order = global index order); a lane without one holds
// li = kNoLocal (and v = NaN, or +inf under NaN-first).  The value min runs on v_min_f64
// (IEEE minNum: NaN only when every lane is NaN), the tie-break on u32 mins — no compare of
// (value, index) pairs and no divergent branch.
constexpr uint32_t kNoLocal = 0xFFFFFFFFu;
__device__ __forceinline__ double wave_min_f64(double v) {
  v = fmin(v, dpp_d<kDppXor1>(v));
  v = fmin(v, dpp_d<kDppXor2>(v));
  v = fmin(v, dpp_d<kDppRor4>(v));
  v = fmin(v, dpp_d<kDppRor8>(v));
  return fmin(fmin(readlane_d(v, 0), readlane_d(v, 16)), fmin(readlane_d(v, 32), readlane_d(v, 48)));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  x = min(x, (uint32_t)dpp_i<kDppXor1>((int)x));
  x = min(x, (uint32_t)dpp_i<kDppXor2>((int)x));
  x = min(x, (uint32_t)dpp_i<kDppRor4>((int)x));
  x = min(x, (uint32_t)dpp_i<kDppRor8>((int)x));
  const uint32_t a = min((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16));
  const uint32_t b = min((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48));
  return min(a, b);
}
// NaN-last order (argsort): the smallest value, ties (and all-NaN) -> the lowest li.
__device__ __forceinline__ void wave_pick_nl(double& v, uint32_t& li) {
  const double m = wave_min_f64(v);
  const int c = (int)(li != kNoLocal) & ((int)(v == m) | ((int)(m != m) & (int)(v != v)));
  li = wave_min_u32(c ? li : kNoLocal);
  v = m;
}
// NaN-first order (np.argmin): the lowest li holding NaN if there is one.
__device__ __forceinline__ void wave_pick_nf(double& v, uint32_t& li) {
  const int isn = (int)(li != kNoLocal) & (int)(v != v);
  if (__any(isn)) {                     // wave-uniform
    li = wave_min_u32(isn ? li : kNoLocal);
    v = __builtin_nan("");
  } else {
    wave_pick_nl(v, li);
  }
}

// As wave_pick_nl with an int64 key (kNoIndex = none): u32 mins over the key's high word,
// then over the low word of the lanes holding that high word.
__device__ __forceinline__ void wave_pick_nl64(double& v, int64_t& key) {
  const double m = wave_min_f64(v);
  const int c = (int)(key != kNoIndex) & ((int)(v == m) | ((int)(m != m) & (int)(v != v)));
  const uint32_t hi = (uint32_t)((uint64_t)key >> 32), lo = (uint32_t)key;
  const uint32_t mh = wave_min_u32(c ? hi : kNoLocal);
  const uint32_t ml = wave_min_u32((c & (int)(hi == mh)) ? lo : kNoLocal);
  key = (mh == kNoLocal && ml == kNoLocal) ? kNoIndex : (int64_t)(((uint64_t)mh << 32) | ml);
  v = m;
}

// Cross-workgroup hand-offs inside the plan launch use write-through (sc1) stores and sc1
// loads with a relaxed agent-scope ticket (MI355X_MICROARCH.md, "Valid forms", first table
// row: every handed-off byte stored sc1 by a wave that drains vmcnt(0) before its block's
// barrier and the one-lane ticket add; the last adder's block loads them sc1; one workgroup
// per CU, guaranteed by the launch's LDS request).  No buffer_wbl2 / buffer_inv.
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T ld_wt(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// key = m C + c (0 <= c < C, 0 <= key < 2^63) split without the 64-bit integer division's
// ~150-instruction software sequence (the controller record's look-ahead best): the fp64
// quotient of the key is within 2^11 of m (the key's rounding), that of the exact remainder
// within 1, and one fix-up step makes the split exact.
__device__ __forceinline__ void split_key(int64_t key, int32_t C, int64_t& m, int32_t& c) {
  const double dc = (double)C;
  int64_t q = (int64_t)((double)key / dc);
  q += (int64_t)((double)(key - q * C) / dc);
  int64_t r = key - q * C;
  if (r < 0) {
    q -= 1;
    r += C;
  } else if (r >= C) {
    q += 1;
    r -= C;
  }
  m = q;
  c = (int32_t)r;
}

// Tagged 64-bit words of the polled completion: launch tag in the high half, payload low.
__device__ __forceinline__ uint64_t tag_word(uint32_t seq, uint32_t payload) {
  return ((uint64_t)seq << 32) | payload;
}
__device__ __forceinline__ bool tag_ok(uint64_t w, uint32_t seq) { return (uint32_t)(w >> 32) == seq; }
__device__ __forceinline__ uint64_t join_words(uint64_t hi, uint64_t lo) {
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ int wave_sum(int x) {
  x += dpp_i<kDppXor1>(x);
  x += dpp_i<kDppXor2>(x);
  x += dpp_i<kDppRor4>(x);
  x += dpp_i<kDppRor8>(x);
  return __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) +
         __builtin_amdgcn_readlane(x, 32) + __builtin_amdgcn_readlane(x, 48);
}


// Keep a wave-uniform value in a VGPR: the rollout loop needs ~25 uniform vehicle/cost
// constants; left in SGPRs they overflow the 102-SGPR budget together with the
// polynomial constants and get spilled to VGPR lanes (v_readlane reloads in the loop).
__device__ __forceinline__ void pin_vgpr(double& x) { asm volatile("" : "+v"(x)); }


__device__ __forceinline__ Tire load_tire(const double* p, int64_t ld, int64_t i) {
  Tire t;
  t.Bf = p[i];
  t.Cf = p[ld + i];
  t.Df = p[2 * ld + i];
  t.Br = p[3 * ld + i];
  t.Cr = p[4 * ld + i];
  t.Dr = p[5 * ld + i];
  return t;
}

// np.mean(window, axis=1) for one model (rt.py:358): NumPy's pairwise order (8 partial sums)
// over the ring read oldest -> newest, then / W; W <= LLAMPC_WMAX (one pairwise block).
// Split around the newest value (the ring slot this tick writes): every older
// value is loaded and summed BEFORE the look-back's RK4 step — the loads' latency under the
// step instead of after it — in that exact order, so finishing with the newest error
// (win_finish) gives the mean's bits in that order.  Oldest -> newest is i = 0 .. W-1, the newest i = W-1:
//   W < 8 or W % 8 != 0: the newest is the sequential tail's last add:  s = pre + e
//   W % 8 == 0 (W >= 8):  it is r[7]'s last term (W = 8: r[7] itself), so
//                          s = A + (B + (r6 + r7)),  A = (r0 + r1) + (r2 + r3),  B = r4 + r5
struct WinPre {
  double a, b, c, d;                    // pre | A, B, r6, r7 without the newest
};
__device__ __forceinline__ WinPre win_pre(const double* ring, int64_t ld, int64_t n, int o, int W) {
  auto at = [&](int i) {
    int s = o + i;
    if (s >= W) s -= W;
    return ring[(int64_t)s * ld + n];
  };
  WinPre p{0.0, 0.0, 0.0, 0.0};
  if (W < 8) {
    for (int i = 0; i < W - 1; ++i) p.a += at(i);
    return p;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = j < W - 1 ? at(j) : 0.0;
  int i = 8;
  const int full = W - (W % 8);
  for (; i < full; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + j < W - 1) r[j] += at(i + j);
  }
  if (W % 8 == 0) {
    p.a = (r[0] + r[1]) + (r[2] + r[3]);
    p.b = r[4] + r[5];
    p.c = r[6];
    p.d = r[7];                         // W = 8: unused (r[7] is the newest itself)
    return p;
  }
  double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < W - 1; ++i) s += at(i);
  p.a = s;
  return p;
}
__device__ __forceinline__ double win_finish(const WinPre& p, double e, int W) {
  double s;
  if (W >= 8 && W % 8 == 0) {
    const double r7 = W == 8 ? e : p.d + e;
    s = p.a + (p.b + (p.c + r7));
  } else {
    s = p.a + e;
  }
  return s / W;
}

}  // namespace

// ------------------------------------------------------------------------------------
// Look-back body (one block = 256 models, lane per model)
// ------------------------------------------------------------------------------------
// Dynamic LDS carve shared by every role (16-B aligned offsets, cdna_hip_programming.md
// G17): [0,64) sv[2][4] double | [64,128) si[2][4] int64 | [128,160) sn[8] int32 (the
// 8-wave work-queue block's la_publish uses all 8) | [160,164) the ticket flag (kFlagOff) |
// [168,176) the poller's per-wave late flags (kLateOff) | pad to 192 | role-specific region
// from 192.
constexpr int kScratchBytes = 192;
constexpr int kFlagOff = 160;
constexpr int kLateOff = 168;
constexpr int kStageW = 8;              // doubles per staged (step, candidate) input
constexpr int kRankBytes = 64 * 8 + 64 * 4 + 256;   // wave_topk_rank: keys + ids per wave (+pad)
constexpr int kWaves = kBlock / 64;     // look-back lists per block (one per wave)
constexpr int kListsPerLane = 8;        // lb_final: lists per lane of the merging wave

struct Scratch {
  double* sv;
  int64_t* si;
  int32_t* sn;
  __device__ explicit Scratch(unsigned char* smem)
      : sv(reinterpret_cast<double*>(smem)),
        si(reinterpret_cast<int64_t*>(smem + 64)),
        sn(reinterpret_cast<int32_t*>(smem + 128)) {}
};

// Block min with ONE barrier: consecutive calls alternate between two scratch buffers, so
// a buffer is rewritten only after the next call's barrier has retired all its readers.
template <int NAN_FIRST>
__device__ __forceinline__ void block_min1(double& v, int64_t& i, const Scratch& s, int& par) {
  wave_min<NAN_FIRST>(v, i);
  double* sv = s.sv + 4 * par;
  int64_t* si = s.si + 4 * par;
  par ^= 1;
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = v;
    si[threadIdx.x >> 6] = i;
  }
  __syncthreads();
  v = sv[0];
  i = si[0];
#pragma unroll
  for (int k = 1; k < kBlock / 64; ++k) {
    if (kless<NAN_FIRST>(sv[k], si[k], v, i)) {
      v = sv[k];
      i = si[k];
    }
  }
}

// ------------------------------------------------------------------------------------
// In-launch completion tickets (wait-free): every storing wave drains its (sc1) stores, the
// block barriers, lane 0 bumps the ticket (relaxed, agent scope); the block that draws the
// last ticket continues and reads the handed-off data with sc1 loads (st_wt / ld_wt above).
// No block ever waits on another, so residency/dispatch order cannot deadlock.  Tickets are
// reset by the final block (and zeroed when a bank is created or reset).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool ticket_last(unsigned* t, unsigned expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == expected - 1;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ double sq_err4(const double* x, const double* xn) {
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double e = x[j] - xn[j];
    s += e * e;
  }
  return s;
}

// Order-preserving u64 of a window mean for the argsort order (rt.py:360): -0 -> +0 and
// every NaN -> one canonical NaN above +inf.
__device__ __forceinline__ uint64_t order_key(double w) {
  const double wc = (w != w) ? __builtin_nan("") : w + 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(wc);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// A top-K entry in LDS: its key, its local model index (ids from kNoModelId up mark lanes
// without a model: unique per slot, above every real index since n <= INT32_MAX) and value.
constexpr uint32_t kNoModelId = 0xFFFFFE00u;
struct BEnt {
  uint64_t key;
  uint32_t id;
  uint32_t pos;
  double v;
};
// (key, id, pos) order: total, so every rank below is unique.
__device__ __forceinline__ bool bless(const BEnt& a, const BEnt& b) {
  return (int)(a.key < b.key) |
         ((int)(a.key == b.key) & ((int)(a.id < b.id) | ((int)(a.id == b.id) & (int)(a.pos < b.pos))));
}
constexpr int kBlockMergeBytes = kWaves * LLAMPC_KMAX * (int)sizeof(BEnt);

// The block's sorted top-K from its waves' lists (kWaves x K entries staged in LDS by
// wave_topk_rank or the R > 1 rounds): the first kWaves*K threads rank their entry among
// them and the ones ranked below K store it in the block's list tk_val/tk_idx[blk][K] —
// one list per block for lb_final (its merge cost grows with the lists' count).
__device__ __forceinline__ void block_topk_merge(const LookbackLaunch& a, int blk, const BEnt* e) {
  const int M = kWaves * a.K;
  const int t = threadIdx.x;
  if (t < M) {
    const BEnt me = e[t];
    int rank = 0;
    for (int j = 0; j < M; ++j) rank += (int)bless(e[j], me);
    if (rank < a.K) {
      st_wt(&a.tk_val[(int64_t)blk * a.K + rank], me.v);
      st_wt(&a.tk_idx[(int64_t)blk * a.K + rank], me.id >= kNoModelId ? kNoIndex : a.goff + (int64_t)me.id);
    }
  }
}

// The sorted top-K of one wave's 64 window means (R == 1) by rank: every lane counts the
// lanes whose (value, index) key precedes its own — NaN last, ties to the lower index
// (rt.py:360 argsort order) — and the lanes ranked below K store their entry at that rank.
// Keys as order-preserving u64 (+0 for -0, one canonical NaN above +inf); lanes without a
// model take a key above every model's (kNoIndex entries at the end of a short list).
// The wave's list goes to out[rank] (LDS, block_topk_merge).
__device__ __forceinline__ void wave_topk_rank(const LookbackLaunch& a, double w, int64_t n,
                                               unsigned char* lds, BEnt* out) {
  const int lane = threadIdx.x & 63;
  uint64_t* keys = reinterpret_cast<uint64_t*>(lds + (threadIdx.x >> 6) * kRankBytes);
  uint32_t* ids = reinterpret_cast<uint32_t*>(keys + 64);
  const bool valid = n < a.n;
  const uint64_t key = valid ? order_key(w) : ~0ull;
  const uint32_t id = valid ? (uint32_t)n : kNoModelId + (uint32_t)threadIdx.x;
  keys[lane] = key;
  ids[lane] = id;
  __syncthreads();
  int rank = 0;
#pragma unroll 16
  for (int j = 0; j < 64; ++j) {
    const uint64_t kj = keys[j];
    const uint32_t ij = ids[j];
    rank += (int)(kj < key) | ((int)(kj == key) & (int)(ij < id));
  }
  if (rank < a.K) out[rank] = BEnt{key, id, 0u, valid ? w : __builtin_nan("")};
}

// ------------------------------------------------------------------------------------
// Look-back body: one block = 256*R models (R models per lane, coalesced in r).
// RK4 step from (x_{t-1}, u_{t-1}), 4-state MSE against x_t, in-place ring write, window
// mean in NumPy's pairwise order; then the block's argmin and its SORTED top-K list.
// ------------------------------------------------------------------------------------
// ARMED (the controller, ctl.hip): x_t comes from door(pred, valid, n) — the LDS copy of x_t,
// or null when the launch is cancelled (lookback_block then returns false) — and with one
// model per lane the RK4 step runs BEFORE it: the step needs only the state's (x_{t-1},
// u_{t-1}), x_t enters with the error, so an armed launch has the step done when its doorbell
// rings.  door() also gets the lane's model n (valid: n < N) and its window mean without x_t
// (pred: the W - 1 entries that stay, over W; the speculative look-ahead's ranking).
template <bool ARMED = false, typename Door = int>
__device__ __forceinline__ bool lookback_block(const LookbackLaunch& a, int blk, const Scratch& sc, Door door = 0) {
  LB_STAMP(blk, 0);
  const int64_t base = (int64_t)blk * kBlock * a.R;
  const fm::FmK K = fm::FmK::load();
  bool ubad = false;
  const Input uf = make_input_fast(a.u_prev[0], a.u_prev[1], K, ubad);
  double wm0 = 0.0;                     // R == 1 keeps the window mean in a register
  const double* x_now = a.x_now;
  double xp[4] = {0.0, 0.0, 0.0, 0.0};  // ARMED, R == 1: the step before the doorbell
  Tire tp{};
  WinPre wpp{0.0, 0.0, 0.0, 0.0};
  bool bp = false, pre = false;
  if constexpr (ARMED) {
    double pred = 0.0;
    bool pvalid = false;
    int64_t pn = 0;
    if (a.R == 1) {                     // launch-uniform
      const int64_t n = base + threadIdx.x;
      if (n < a.n) {
        pvalid = true;
        pn = n;
        double x[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) x[j] = a.x_prev[j];
        tp = load_tire(a.params, a.n, n);
        const int o = (a.slot + 1 == a.W) ? 0 : a.slot + 1;
        if (a.full) wpp = win_pre(a.ring, a.n, n, o, a.W);
        const StageK sk = make_stage<1>(a.veh, tp, 0);
        Dom dm;
        dm.init();
        step_fast<0, 1>(a.veh, tp, sk, x, uf, a.Ts, K, dm);
#pragma unroll
        for (int j = 0; j < 4; ++j) xp[j] = x[j];
        bp = (int)ubad | (int)!sk.sok | (int)!dm.ok();
        if (a.full) pred = win_finish(wpp, 0.0, a.W);
      }
      pre = true;
    }
    x_now = door(pred, pvalid, pn);
    if (!x_now) return false;
  }
  for (int r = 0; r < a.R; ++r) {
    const int64_t n = base + (int64_t)r * kBlock + threadIdx.x;
    if (n >= a.n) break;
    double x[6];
    Tire t;
    WinPre wp{0.0, 0.0, 0.0, 0.0};
    bool bad;
    if (ARMED && pre) {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = xp[j];
      t = tp;
      wp = wpp;
      bad = bp;
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j) x[j] = a.x_prev[j];
      t = load_tire(a.params, a.n, n);
      const int o = (a.slot + 1 == a.W) ? 0 : a.slot + 1;     // the window's oldest slot
      if (a.full) wp = win_pre(a.ring, a.n, n, o, a.W);      // launch-uniform; under the step
      // model.py:32-40, one RK4 step: the fast stage; a lane whose operands leave the fast
      // cores' domains redoes the step with the general functions (as the look-ahead does)
      const StageK sk = make_stage<1>(a.veh, t, 0);
      Dom dm;
      dm.init();
      step_fast<0, 1>(a.veh, t, sk, x, uf, a.Ts, K, dm);
      bad = (int)ubad | (int)!sk.sok | (int)!dm.ok();
    }
    double s = sq_err4(x, x_now);                         // rt.py:349 mean over 4 states
    // the domain once per step; a NaN operand reaches x[0..3] (the stage-4 chains feed x[3])
    bad = (int)bad | (int)!(s <= __DBL_MAX__);
    if (__builtin_expect(__any(bad), 0)) {
      if (bad) {
#pragma unroll
        for (int j = 0; j < 6; ++j) x[j] = a.x_prev[j];
        rk4_step(a.veh, t, x, make_input(a.u_prev[0], a.u_prev[1]), a.Ts);
        s = sq_err4(x, x_now);
      }
    }
    const double err = s / 4;
    if (a.err_out) a.err_out[n] = err;
    a.ring[(int64_t)a.slot * a.n + n] = err;             // rt.py:352-353 without np.roll
    if (a.full) {
      const double wm = win_finish(wp, err, a.W);          // rt.py:358
      if (a.R > 1 || a.wm_keep) a.wm_buf[n] = wm;         // launch-uniform
      if (r == 0) wm0 = wm;
    }
  }
  LB_STAMP(blk, 1);
  if (!a.full) return true;  // launch-uniform

  // per WAVE (a list): the argmin (rt.py:359 semantics) and the sorted top-K (rt.py:360
  // argsort order) of its 64*R models with branch-free wave picks — no LDS round trip, no
  // barrier (a block-wide (value, index) min per round cost ~4k cycles); lb_final merges
  // the kWaves lists of every block.  Local index n < 2^32 (bank size check in the C-ABI).
  const int lane = threadIdx.x & 63;
  const int64_t list = (int64_t)blk * kWaves + (threadIdx.x >> 6);
  double v = a.nan_first ? __builtin_inf() : __builtin_nan("");
  uint32_t li = kNoLocal;
  for (int r = 0; r < a.R; ++r) {
    const int64_t n = base + (int64_t)r * kBlock + threadIdx.x;
    if (n >= a.n) break;
    const double w = (a.R == 1) ? wm0 : a.wm_buf[n];
    const bool t = a.nan_first ? less_bf<1>(w, (uint32_t)n, v, li) : less_bf<0>(w, (uint32_t)n, v, li);
    v = t ? w : v;
    li = t ? (uint32_t)n : li;
  }
  if (a.nan_first) wave_pick_nf(v, li);
  else wave_pick_nl(v, li);
  if (lane == 0) {
    st_wt(&a.am_val[list], v);
    st_wt(&a.am_idx[list], li == kNoLocal ? kNoIndex : a.goff + li);
  }
  LB_STAMP(blk, 2);
  unsigned char* rank_lds = reinterpret_cast<unsigned char*>(sc.sv) + kScratchBytes;
  BEnt* wl = reinterpret_cast<BEnt*>(rank_lds + kWaves * kRankBytes);   // [kWaves][K]
  BEnt* mine = wl + (threadIdx.x >> 6) * a.K;
  if (a.R == 1) {                       // launch-uniform
    wave_topk_rank(a, wm0, base + threadIdx.x, rank_lds, mine);
    __syncthreads();
    block_topk_merge(a, blk, wl);
    LB_STAMP(blk, 3);
    return true;
  }
  // R > 1: K rounds of "next key after the previous pick" (NaN last, ties -> lower index)
  double lv = 0.0;
  uint32_t ll = kNoLocal;
  for (int k = 0; k < a.K; ++k) {
    double cv = __builtin_nan("");
    uint32_t cl = kNoLocal;
    for (int r = 0; r < a.R; ++r) {
      const int64_t n = base + (int64_t)r * kBlock + threadIdx.x;
      if (n >= a.n) break;
      const double w = (a.R == 1) ? wm0 : a.wm_buf[n];
      const uint32_t ln = (uint32_t)n;
      const bool t = (int)(k == 0 || less_bf<0>(lv, ll, w, ln)) & (int)less_bf<0>(w, ln, cv, cl);
      cv = t ? w : cv;
      cl = t ? ln : cl;
    }
    wave_pick_nl(cv, cl);
    if (lane == 0) {
      const bool none = cl == kNoLocal;
      mine[k] = BEnt{none ? ~0ull : order_key(cv), none ? kNoModelId + (uint32_t)((threadIdx.x >> 6) * a.K + k) : cl,
                     0u, none ? __builtin_nan("") : cv};
    }
    lv = cv;
    ll = cl;
  }
  __syncthreads();
  block_topk_merge(a, blk, wl);
  LB_STAMP(blk, 3);
  return true;
}

// Input-rate term du' R du of one step (nmpc.py:65-68, 111) and the bounds / rate
// feasibility of one input (nmpc.py:102-105; branch-free: |d| <= dmax is false for NaN like
// the two one-sided tests; dmax < 0 disables).
__device__ __forceinline__ double act_term(const CostK& q, double d0, double d1) {
  return d0 * (q.R[0] * d0 + q.R[1] * d1) + d1 * (q.R[2] * d0 + q.R[3] * d1);
}
__device__ __forceinline__ bool input_feasible(const CostK& q, double ua, double ud, double d0,
                                               double d1) {
  return (int)(ua <= q.umax[0]) & (int)(ua >= q.umin[0]) & (int)(ud <= q.umax[1]) &
         (int)(ud >= q.umin[1]) & ((int)(q.dmax[0] < 0) | (int)(fabs(d0) <= q.dmax[0])) &
         ((int)(q.dmax[1] < 0) | (int)(fabs(d1) <= q.dmax[1]));
}

// One (model, candidate) rollout over H steps and its NLP objective (nmpc.py:44-111).
// FAST: the branch-free stage (dyn.hpp step_fast); `bad` |= any operand of this lane outside
// the fast cores' domains.  !FAST: the general evaluation (rk4_step / euler / rk6 with the
// general transcendentals) — the re-run of bad lanes, so every lane's result depends on its
// own operands only.  Returns J (+inf when infeasible).
// SPLIT (fused RK4 at LPM = 4, diagonal Q and P): each lane of the quad integrates one
// position component (dyn.hpp k_fused) and accumulates its tracking term; the quad's J is
// (J_X + J_Y) + act by two DPP broadcasts at the end.
// ULDS (the controller tick, ctl.hip): the raw candidates U [C][H][2] are at `su` (LDS)
// instead of a.U; only with STAGE = false.  S4 (with ULDS, FAST): the steering's sin / cos
// per (candidate, step) at s4 [C][H][2], then per candidate the input-rate cost sum and the
// feasibility (1 / 0; NaN: a steering outside sincos_fast's domain, so the rollout re-runs in
// the general evaluation) at s4 + 2CH [C][2] (LDS; ctl.hip ctl_stage) — the step reads two
// values instead of forming them, with the same values and roundings.
// DEFER (with SPLIT and S4: the controller's speculative look-ahead, ctl.hip ctl_spec): the
// reference is not known yet — the lane stores its position component after step k at
// dpos[k dstride] instead of accumulating the tracking term, and returns its last position,
// the summed input-rate cost, the feasibility and the domain flag in *dout (J: defer_cost,
// the same terms in the same order once the reference is known).
struct DeferOut {
  double xl, act, feas_s;
  bool dok;
};
// SW: doubles per staged record (the plan kernel's kStageW; the NLP kernel's compact 6: the
// Euler record's input-rate term and feasibility then at 4 and 5 instead of 6 and 7).
template <int INTEG, bool STAGE, int LPM, int XM, bool FAST, bool SPLIT = false, bool ULDS = false, bool TRAJ = false,
          bool S4 = false, bool DEFER = false, int SW = kStageW>
__device__ __forceinline__ double rollout(const LookaheadLaunch& a, int c, int64_t n,
                                          const double* x0, const double* sx, const double* su, const VehK& veh,
                                          const Tire& t, const StageK& sk, const CostK& q,
                                          double Ts, double up0, double up1, const fm::FmK& K,
                                          const FusedK& fq, bool& bad, double* traj = nullptr,
                                          const double* s4 = nullptr, double* dpos = nullptr, int dstride = 0,
                                          DeferOut* dout = nullptr) {
  static_assert(!DEFER || (SPLIT && S4), "deferred tracking cost: the controller's split, staged rollout");
  static_assert(!TRAJ || (INTEG != 0 && !SPLIT), "trajectory output: unscaled, unsplit state");
  static_assert(!S4 || (ULDS && FAST && !STAGE), "staged sincos / cost terms: the controller's fast rollout");
  static_assert(!SPLIT || (FAST && INTEG == 0 && LPM == 4), "position split: fused RK4 quads only");
  static_assert(!ULDS || !STAGE, "candidates in LDS: unstaged rollout");
  const int H = a.H, C = a.C;
  const double* Ub = ULDS ? su : a.U;
  double x[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) x[m] = x0[m];
  if (SPLIT) x[0] = sk.pc ? x0[1] : x0[0];
  if (FAST && INTEG == 0 && scaled_yaw(LPM)) {   // the scaled yaw and yaw rate (make_fused)
    x[2] = x0[2] * K.two_pi;
    x[5] = x0[5] * Ts;
  }
  const double Qd = sk.pc ? q.Q[3] : q.Q[0], Pd = sk.pc ? q.P[3] : q.P[0];   // SPLIT only
  double track = 0.0, act = 0.0;
  double p0 = up0, p1 = up1;
  bool feas = true;
  double feas_s = 1.0;
  double xr0 = 0.0, xr1 = 0.0;
  const double* xpm = XM ? a.xref_pm + n * 2 * H : nullptr;   // this model's reference
  Dom dm;                               // FAST: the operands' running extremes
  dm.init();
  for (int k = 0; k < H; ++k) {
    if (FAST) STEP_STAMP(k < 24 ? k : 24);
    double ua, ud;
    Input u;
    FusedIn fi{};
    if (STAGE) {                        // staged per block (lookahead_block), layouts there
      static_assert(SW == kStageW || (SW == 6 && INTEG != 0), "the compact record: NLP-Euler only");
      constexpr int kAct = SW == kStageW ? 6 : 4, kFeas = kAct + 1;
      const double* o = su + SW * (k * C + c);
      if (INTEG == 0 && FAST) {         // the fused stages' input terms
        fi = FusedIn{o[0], o[1], o[2], o[3], o[4]};
        ua = 0.0;
        ud = o[5];
      } else if (INTEG == 0) {          // the general re-run: the candidate from U itself
        ua = Ub[2 * ((int64_t)c * H + k)];
        ud = Ub[2 * ((int64_t)c * H + k) + 1];
        u = make_input(ua, ud);
      } else {                          // sincos(delta) staged with the fast/general rule
        ua = o[0];
        ud = o[1];
        u.a = ua;
        u.d = ud;
        u.sd = o[2];
        u.cd = o[3];
      }
      act = act + o[kAct];              // the candidate's input-rate term and feasibility
      feas_s = feas_s * o[kFeas];
    } else {
      ua = Ub[2 * ((int64_t)c * H + k)];
      ud = Ub[2 * ((int64_t)c * H + k) + 1];
      if (S4) {
        const double2 sc2 = *reinterpret_cast<const double2*>(s4 + 2 * ((int64_t)c * H + k));
        u.a = ua;
        u.d = ud;
        u.sd = sc2.x;
        u.cd = sc2.y;
      } else if (FAST) {
        u = make_input_fast(ua, ud, K, bad);
      } else {
        u = make_input(ua, ud);
      }
    }
    const double d0 = ua - p0, d1 = ud - p1;          // nmpc.py:65-68
    if (!STAGE && !S4 && q.enforce) feas = (int)feas & (int)input_feasible(q, ua, ud, d0, d1);
    if (FAST && INTEG == 0 && STAGE) step_fused<LPM, SPLIT>(sk, fq, x, fi, ud, K, dm);
    else if (FAST && INTEG == 0) step_fused<LPM, SPLIT>(sk, fq, x, u, K, dm);
    else if (FAST) step_fast<INTEG, LPM>(veh, t, sk, x, u, Ts, K, dm);
    else step<INTEG>(veh, t, x, u, Ts);
    if (DEFER) {                        // the position component, for defer_cost
      dpos[k * dstride] = x[0];
    } else if (SPLIT) {                 // this lane's component of the reference and term
      xr0 = XM ? xpm[2 * k + sk.pc] : sx[2 * (k + 1) + sk.pc];
      const double e = x[0] - xr0;
      track = track + e * (Qd * e);
    } else if (XM) {
      xr0 = xpm[2 * k];
      xr1 = xpm[2 * k + 1];
    } else {
      xr0 = sx[2 * (k + 1)];
      xr1 = sx[2 * (k + 1) + 1];
    }
    if (!SPLIT) {
      const double e0 = x[0] - xr0, e1 = x[1] - xr1;
      track = track + (e0 * (q.Q[0] * e0 + q.Q[1] * e1) + e1 * (q.Q[2] * e0 + q.Q[3] * e1));
    }
    if (!STAGE && !S4) act = act + act_term(q, d0, d1);
    p0 = ua;
    p1 = ud;
    if (TRAJ && traj != nullptr) {      // the state after step k (every lane of a quad holds it;
#pragma unroll                          // the caller passes traj to one lane): three 16-B stores
      for (int m = 0; m < 6; m += 2) *reinterpret_cast<double2*>(traj + 6 * (k + 1) + m) = double2{x[m], x[m + 1]};
    }
  }
  if (S4) {                             // the candidate's summed input-rate cost, feasibility
    const double2 af = *reinterpret_cast<const double2*>(s4 + 2 * (int64_t)C * H + 2 * c);
    act = af.x;
    feas_s = af.y;
  }
  if constexpr (DEFER) {
    (void)track;
    (void)Qd;
    (void)Pd;
    *dout = DeferOut{x[0], act, feas_s, dm.ok()};
    return 0.0;
  }
  double J;
  if (SPLIT) {                                                    // nmpc.py:48, :111
    const double e = x[0] - xr0;
    const double jl = e * (Pd * e) + track;                       // this component's part
    J = (dpp_bcast<kQuad0>(jl) + dpp_bcast<kQuad1>(jl)) + act;    // X (lane 0) + Y (lane 1)
  } else {
    const double e0 = x[0] - xr0, e1 = x[1] - xr1;                 // nmpc.py:48 (xref_H)
    const double term = e0 * (q.P[0] * e0 + q.P[1] * e1) + e1 * (q.P[2] * e0 + q.P[3] * e1);
    J = (term + track) + act;                                     // nmpc.py:111
  }
  // the domain, once per rollout: a NaN operand reaches x[0..1] (every chain output feeds
  // the later stages' positions, the last stage's feeds vx, vy, omega only through a NaN
  // state that the position update already carries), so a non-finite J is re-run too
  if (FAST) {
    const bool dok = dm.ok();
    bad = (int)bad | (int)!sk.sok | (int)!dok | (int)!(fabs(J) <= __DBL_MAX__);
    if (S4) bad = (int)bad | (int)(feas_s != feas_s);   // a steering outside sincos_fast's domain
  }
  if (STAGE || S4) feas = feas_s != 0.0;
  if (!feas) J = __builtin_inf();
  return J;
}

// Global -> LDS copy of `count` doubles with B loads in flight per thread: a plain strided
// loop waits one memory round trip per element — ~25 per thread for the ETHZ spline table
// (50 KB per block), which made the raceline prologue ~25 us.  src(e) gives element e; it
// is called for e = threadIdx.x + j kBlock in order, j < B per batch, past count too (with
// e clamped to count - 1: unguarded loads, no branch per element; those are not stored).
template <int B = 16, typename Src>
__device__ __forceinline__ void copy_lds(double* dst, int count, Src src) {
  for (int base = threadIdx.x; base < count; base += B * kBlock) {
    double v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = base + j * kBlock;
      v[j] = src(e < count ? e : count - 1);
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int e = base + j * kBlock;
      if (e < count) dst[e] = v[j];
    }
  }
}

// ------------------------------------------------------------------------------------
// Look-ahead body.  Lane layout inside a block: sub = lane % LPM (LPM = 2: the lane pair
// of one rollout, front/rear chain), cl = lane / LPM; G candidate-lanes per model (power of two); a model's
// candidates c = g + j*G, j < cpl, run sequentially in its G*LPM lanes.
//   LDS from kScratchBytes: xref as [k][2]; U as [k][c][kStageW] (RK4: F0, F1, h/m sin,
//   h/m cos, h lf/Iz cos, delta; else pwm, delta, sin, cos; then
//   input-rate cost term, feasibility) when staged.
// ------------------------------------------------------------------------------------
// The block's partial of the look-ahead argmin over (model, candidate) in flattened order
// (goff+n)*C + c — (v, key) per lane (kNoIndex: none) and the lanes' non-finite counts:
// branch-free wave picks, one LDS exchange, thread 0 publishes (tagged words or plain).
template <int NW = kWaves>
__device__ __forceinline__ void la_publish(const LookaheadLaunch& a, int blk, const Scratch& sc, int par,
                                           double v, int64_t key, int nf) {
  // NW = 8 (the work-queue block) uses both halves of sv / si (par = 0 there) and sn[4..8)
  static_assert(NW == kWaves || NW == 8, "4- or 8-wave blocks");
  wave_pick_nl64(v, key);
  const int nfw = wave_sum(nf);
  double* sv = sc.sv + 4 * par;         // the buffer a span > 64 exchange did not use
  int64_t* si = sc.si + 4 * par;
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = v;
    si[threadIdx.x >> 6] = key;
    sc.sn[threadIdx.x >> 6] = nfw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int nfs = sc.sn[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const bool t = (int)(si[w] != kNoIndex) & (int)less_bf<0>(sv[w], si[w], v, key);
      v = t ? sv[w] : v;
      key = t ? si[w] : key;
      nfs += sc.sn[w];
    }
    if (a.poll) {
      uint64_t* r = a.blk_tag + 5 * (int64_t)blk;
      const uint64_t vb = (uint64_t)__double_as_longlong(v), kb = (uint64_t)key;
      st_wt(&r[0], tag_word(a.seq, (uint32_t)(vb >> 32)));
      st_wt(&r[1], tag_word(a.seq, (uint32_t)vb));
      st_wt(&r[2], tag_word(a.seq, (uint32_t)(kb >> 32)));
      st_wt(&r[3], tag_word(a.seq, (uint32_t)kb));
      st_wt(&r[4], tag_word(a.seq, (uint32_t)nfs));
    } else {
      st_wt(&a.pv[blk], v);
      st_wt(&a.pidx[blk], key);
      st_wt(&a.pnf[blk], nfs);
    }
  }
}

// WQ (the throughput regime, launch_plan): a persistent layout — the grid holds one look-ahead
// block per CU and each wave takes units of 64 / G models (one model at G = 64) from the
// bank's work counter, so the staging prologue runs once per CU instead of once per 4 models
// and no CU waits for a new block between units (v29 stamps at C = 64: prologue 3.4 us and
// reduction 2 us of each 45 us block).
template <int INTEG, bool STAGE, int LPM, int XM, int WQ = 0>
__device__ __forceinline__ void lookahead_block(const LookaheadLaunch& a, int blk, int G, int cpl,
                                                unsigned char* smem, const Scratch& sc) {
  LA_STAMP(blk, 0);
  constexpr int BT = wq_threads(WQ);   // threads of this block
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);
  double* su = sx + 2 * (a.H + 1);
  const int H = a.H, C = a.C;
  // this lane's model: its Pacejka row and the start state are loaded first, so they are in
  // flight while the block stages the shared inputs (one HBM round trip, not two)
  const int sub = threadIdx.x % LPM;
  const int cl = threadIdx.x / LPM;
  const int g = cl & (G - 1);
  const int64_t n = (int64_t)blk * (kBlock / (G * LPM)) + cl / G;
  const bool live = n < a.n;
  // XM: threads [0, mpb) walk the raceline; the U staging below runs on the threads after
  // them, so the two overlap (the walk is one lane's serial chain, latency-bound)
  const int mpb = kBlock / (G * LPM);
  const int soff = (XM && mpb < kBlock) ? mpb : 0;
  Tire t{};
  if (!WQ && live) t = load_tire(a.params, a.n, n);
  double x0[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) x0[m] = a.x0[m];
  // XM = 1 (per-model raceline reference): knots [n] and the x/y spline rows [2][4][n-1]
  // after the (optional) U staging; a.xref holds the shared start {s0, v0, scale}
  double* rl_knots = su + (STAGE ? kStageW * C * H : 0);
  double* rl_xy = rl_knots + a.rl.n + kKnotPad;
  if (XM) {
    const int nk = a.rl.n, nseg = a.rl.n - 1, nxy = 8 * nseg;
    const double* gk = a.rl.knots;                          // knots | xy contiguous
    const double* gmu = a.rl.mus;
    double* rl_mus = rl_xy + nxy;                           // [M], then the speed window
    // knots, the +inf pad (RaceRef::step), xy and mus in one batch (one memory round trip
    // per thread at the ETHZ size)
    copy_lds<4>(rl_knots, nk, [&](int e) { return gk[e]; });
    copy_lds<24>(rl_xy, nxy + a.rl.M, [&](int e) {
      const double* p = e < nxy ? gk + nk + e : gmu + (e - nxy);
      return *p;
    });
    if ((int)threadIdx.x < kKnotPad) rl_knots[nk + threadIdx.x] = __builtin_inf();
    // the window end: s0 plus the largest advance of H walker steps (one lap at most)
    const double s0 = a.xref[0];
    const double L = gk[nseg];
    const double adv = window_adv(a.xref[1], a.xref[2], a.Ts, H, a.rl.vmax);
    const bool bounded = adv < L && s0 >= 0.0 && s0 < L;
    double te = s0 + adv;
    if (te >= L) te -= L;
    __syncthreads();
    RL_STAMP(blk, 0);
    // bisect-right of s0 and te on the knots (RaceRef::init's: the largest i in [1, n-2]
    // with knots[i] <= s, else 0) as one parallel pass: with the knots ascending, exactly
    // one segment i has (i == 0 or knots[i] <= s) and (i == n-2 or not knots[i+1] <= s),
    // and it writes i.  XM leaves sx (the shared xref stage) unused: two ints there.
    int* rl_sel = reinterpret_cast<int*>(sx);
    for (int i = threadIdx.x; i < nseg; i += kBlock) {
      const double ki = rl_knots[i], kn = rl_knots[i + 1];
      const bool last = i == nseg - 1;
      if ((i == 0 || ki <= s0) && (last || !(kn <= s0))) rl_sel[0] = i;
      if ((i == 0 || ki <= te) && (last || !(kn <= te))) rl_sel[1] = i;
    }
    __syncthreads();
    // the speed profiles' window (raceline.hpp SpeedWin): from the start segment to the
    // window end; block-uniform
    SpeedWin sw{nullptr, 0, 0};
    const int seg0 = rl_sel[0];
    {
      const int lo = seg0, l2 = rl_sel[1];
      const double need = bounded ? (double)(l2 >= lo ? l2 - lo : l2 + nseg - lo) + 2.0 : 1e300;
#ifdef LLAMPC_STAMPS
      if (blk == 0 && threadIdx.x == 0) {
        g_rl_dbg[0] = need;
        g_rl_dbg[1] = a.rl.wcap;
        g_rl_dbg[2] = adv;
        g_rl_dbg[3] = a.xref[0];
        g_rl_dbg[4] = L;
        g_rl_dbg[5] = a.rl.vmax;
      }
#endif
      if (need <= (double)a.rl.wcap) {
        double* wl = rl_mus + ((a.rl.M + 1) & ~1);          // 16-B aligned
        sw.w = wl;
        sw.seg0 = lo;
        sw.W = (int)need;
        const int W = sw.W, tot = a.rl.M * 4 * W;
        const double* gsp = a.rl.speed;
        // element e = row W + j; copy_lds asks for e = threadIdx.x + i kBlock in order, so
        // (row, j) steps by kBlock without a division per element
        int row = (int)threadIdx.x / W, j = (int)threadIdx.x - row * W;
        const int drow = kBlock / W, dj = kBlock - drow * W, rows = a.rl.M * 4;
        copy_lds<24>(wl, tot, [&](int) {          // (row, j) past the end: clamped rows
          int sg = lo + j;
          if (sg >= nseg) sg -= nseg;
          const double v = gsp[(size_t)(row < rows ? row : rows - 1) * nseg + sg];
          row += drow;
          j += dj;
          if (j >= W) {
            j -= W;
            ++row;
          }
          return v;
        });
        __syncthreads();
      }
    }
    RL_STAMP(blk, 1);
    // one thread per model of this block walks ConstantSpeed into xref_pm[m][H][2]
    const int64_t m = (int64_t)blk * mpb + threadIdx.x;
    if ((int)threadIdx.x < mpb && m < a.n) {
      const double mu = (a.params[2 * a.n + m] + a.params[5 * a.n + m]) / (9.81 * a.veh.mass);
      // the table descriptor in registers: the walk's global stores cannot alias it
      const RacelineK rl = a.rl;
      RaceRef rr;
      rr.init(rl, rl_knots, rl_mus, mu, a.xref[0], a.xref[1], a.xref[2], a.Ts, seg0);
      double2* out = reinterpret_cast<double2*>(a.xref_pm + m * 2 * H);
      for (int k = 0; k < H; ++k) {
        double xr, yr;
        rr.step(rl, rl_knots, rl_xy, sw, xr, yr);
        out[k] = make_double2(xr, yr);
      }
    }
    RL_STAMP(blk, 2);
    __threadfence_block();
    RL_STAMP(blk, 3);
  } else {
    for (int e = threadIdx.x; e <= H; e += BT) {
      sx[2 * e] = a.xref[e];
      sx[2 * e + 1] = a.xref[(H + 1) + e];
    }
  }
  // Shared xref: ONE FmK for the staging below and the rollouts (the staging uses its sincos
  // constants, the same in the lean and precise sets) instead of materialising the ~50
  // constants twice on the prologue's critical path; the raceline variant keeps two loads
  // (holding them across its prologue spilled, round 1).
  fm::FmK K0;
  if constexpr (!XM) K0 = fm::FmK::load<kLeanLA && INTEG == 0>();
  if (STAGE) {
    // [k][c] -> (pwm, delta, sin delta, cos delta): the steering's sincos depends only on the
    // shared candidates, so it is formed once per block here (same evaluation as
    // make_input_fast: the fast core on its domain, the general function off it).  RK4
    // stages the fused stages' input terms instead: (F0, F1, h/m sin d, h/m cos d,
    // h lf/Iz cos d, delta) — dyn.hpp fused_in, with the shared constants of make_fused.
    const fm::FmK K = [&] {
      if constexpr (XM) return fm::FmK::load();
      else return K0;
    }();
    const FusedK fq0 = make_fused(a.veh, make_stage<1>(a.veh, Tire{}, 0), a.Ts, scaled_yaw(LPM));
    for (int e = (int)threadIdx.x - soff; e < C * H; e += BT - soff) {
      if (e < 0) break;
      const int c = e / H, k = e - c * H;
      const double dl = a.U[2 * e + 1];
      double sd, cd;
      if (fm::sincos_fast_ok(dl)) fm::sincos_fast(dl, &sd, &cd, K);
      else LL_SINCOS(dl, &sd, &cd);
      double* o = su + kStageW * (k * C + c);
      const double ua = a.U[2 * e];
      const double p0 = k ? a.U[2 * e - 2] : a.uprev[0], p1 = k ? a.U[2 * e - 1] : a.uprev[1];
      const double d0 = ua - p0, d1 = dl - p1;
      if (INTEG == 0) {
        const FusedIn fi = fused_in(fq0, Input{ua, dl, sd, cd});
        o[0] = fi.F0;
        o[1] = fi.F1;
        o[2] = fi.hmsd;
        o[3] = fi.hmcd;
        o[4] = fi.c5a;
        o[5] = dl;
      } else {
        o[0] = ua;
        o[1] = dl;
        o[2] = sd;
        o[3] = cd;
      }
      o[6] = act_term(a.cost, d0, d1);
      o[7] = (!a.cost.enforce || input_feasible(a.cost, ua, dl, d0, d1)) ? 1.0 : 0.0;
    }
  }
  __syncthreads();

  CostK q = a.cost;
  VehK veh = a.veh;
  double Ts = a.Ts;
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
  const double up0 = a.uprev[0], up1 = a.uprev[1];

  double bv = __builtin_nan("");
  int64_t bc = kNoIndex;
  int nf = 0;
  LA_STAMP(blk, 1);
  // position split of the quad (fused RK4, LPM = 4) when Q and P are diagonal (rt.py:60-62:
  // Q = diag(1, 1), P = 0): tested on the unpinned kernel-argument copy, so the branch is
  // scalar
  constexpr bool kSplit = (INTEG == 0 && LPM == 4);
  const bool diagQP = a.cost.Q[1] == 0.0 && a.cost.Q[2] == 0.0 && a.cost.P[1] == 0.0 && a.cost.P[2] == 0.0;
  if constexpr (WQ) {
    static_assert(LPM == 1 && XM == 0, "work queue: LPM 1, shared xref");
    // Unit u = models [u mpw, (u + 1) mpw) of one wave.  Lane 0 takes unit numbers from the
    // bank's counter (relaxed agent-scope add; 0 at the launch's start: the block completing
    // the record resets it in final_write, after every look-ahead block has published, i.e.
    // after every take of the launch); the next take is issued before the current unit's
    // rollouts and read after them, so its latency is hidden.  The counter only grows within
    // a launch, so u >= 0 and every model index is checked against n.
    const int mpw = 64 / G;
    const int64_t units = (a.n + mpw - 1) / mpw;
    const int lm = (int)(threadIdx.x & 63) / G;
    // The take must stay in flight across the rollouts.  In v30 every unit waited for its
    // round trip (ISA: s_waitcnt vmcnt(0) right after the atomic): the atomic optimizer
    // rewrites an atomic on a uniform address into one lane's atomic plus a
    // readfirstlane/prefix epilogue that uses the result at once.  So the address carries an
    // opaque zero VGPR offset (not uniform to the compiler: no optimizer rewrite).  And with
    // the row loads and the atomic both pending, the waitcnt pass cannot count them apart
    // (a returning atomic and loads are different event kinds: it waits for vmcnt(0), i.e.
    // for the atomic too, at the first use of the row); so the offset of each take is a zero
    // that depends on the unit's Pacejka row (an asm reading the six values): the row is
    // waited for first, then the atomic goes out and nothing waits for it until take().
    uint32_t zoff;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zoff));
    auto issue = [&](uint32_t off) -> uint64_t {
      uint64_t v = 0;
      if ((threadIdx.x & 63) == 0)
        v = __hip_atomic_fetch_add(a.wq + off, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return v;
    };
    auto take = [&](uint64_t v) -> int64_t {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 0);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 0);
      return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    double vacc = __builtin_nan("");
    int64_t kacc = kNoIndex;
    int nfacc = 0;
    const fm::FmK K = K0;
#ifdef LLAMPC_STAMPS
    int ju = 0;                                             // this wave's unit count
#endif
    for (int64_t u = take(issue(zoff)); u < units;) {      // wave-uniform
      WQ_STAMP(blk, ju, 0);
      const int64_t nm = u * mpw + lm;
      const bool lv = nm < a.n;
      Tire tm{};
      if (lv) tm = load_tire(a.params, a.n, nm);
      uint32_t dep;
      asm volatile("v_mov_b32 %0, 0" : "=v"(dep) : "v"(tm.Bf), "v"(tm.Cf), "v"(tm.Df), "v"(tm.Br), "v"(tm.Cr), "v"(tm.Dr));
      WQ_STAMP(blk, ju, 1);
      const uint64_t nxt = issue(dep);
      double mv = __builtin_nan("");
      int64_t mc = kNoIndex;
      if (lv) {
        constexpr bool kScaled = (INTEG == 0 && scaled_yaw(1));
        StageK sk = make_stage<1>(veh, tm, 0, INTEG == 0 ? Ts : 1.0);
        if (kScaled) {                  // the chains' lw / h turns W back into omega
          sk.ch[0].lw = sk.ch[0].lw / Ts;
          sk.ch[1].lw = sk.ch[1].lw / Ts;
        }
        const FusedK fq = make_fused(veh, sk, Ts, kScaled);
        for (int j = 0; j < cpl; ++j) {
          const int c = g + j * G;
          if (c >= C) break;
          bool bad = false;
          double J = rollout<INTEG, STAGE, 1, 0, true>(a, c, nm, x0, sx, su, veh, tm, sk, q, Ts, up0, up1, K, fq, bad);
          if (__builtin_expect(__any(bad), 0)) {
            bool unused = false;
            if (bad) J = rollout<INTEG, STAGE, 1, 0, false>(a, c, nm, x0, sx, su, veh, tm, sk, q, Ts, up0, up1, K, fq, unused);
          }
          if (a.cost_out) a.cost_out[nm * C + c] = J;
          nfacc += !isfinite(J);
          if (less_nan_last(J, c, mv, mc)) {
            mv = J;
            mc = c;
          }
        }
      }
      for (int off = G >> 1; off >= 1; off >>= 1) {        // the model's argmin over its lanes
        const double ov = __shfl_xor(mv, off, 64);
        const int64_t oc = __shfl_xor(mc, off, 64);
        if (less_nan_last(ov, oc, mv, mc)) {
          mv = ov;
          mc = oc;
        }
      }
      WQ_STAMP(blk, ju, 2);
      const int64_t un = take(nxt);                         // before the unit's stores
      if (lv && g == 0) {
        if (a.poll) {
          st_wt(&a.la_tag[nm], tag_word(a.seq, (uint32_t)(__double_as_longlong(mv) >> 32)));
          st_wt(&a.la_tag[a.n + nm], tag_word(a.seq, (uint32_t)__double_as_longlong(mv)));
          st_wt(&a.la_tag[2 * a.n + nm], tag_word(a.seq, (uint32_t)(int32_t)mc));
        } else {
          st_wt(&a.best_cand[nm], (int32_t)mc);
          st_wt(&a.best_cost[nm], mv);
        }
        if (mc != kNoIndex) {
          const int64_t key = (a.goff + nm) * C + mc;
          if (less_bf<0>(mv, key, vacc, kacc)) {
            vacc = mv;
            kacc = key;
          }
        }
      }
      WQ_STAMP(blk, ju, 3);
#ifdef LLAMPC_STAMPS
      ++ju;
#endif
      u = un;
    }
    LA_STAMP(blk, 2);
    la_publish<BT / 64>(a, blk, sc, 0, vacc, kacc, nfacc);
    LA_STAMP(blk, 3);
    return;
  }
  if (live) {
    // LPM = 2: lane 0 of the pair evaluates the front chain, lane 1 the rear (dyn.hpp)
    // fused RK4 quads carry W = h omega and Psi = (2/pi) psi (make_fused): the chains'
    // lw / h turns W back into omega
    constexpr bool kScaled = (INTEG == 0 && scaled_yaw(LPM));
    StageK sk = make_stage<LPM>(veh, t, sub, INTEG == 0 ? Ts : 1.0);
    if (kScaled) sk.ch[0].lw = sk.ch[0].lw / Ts;
    if (kScaled && LPM == 1) sk.ch[1].lw = sk.ch[1].lw / Ts;
    if (kScaled && LPM == 4 && sub >= 2) {
      // lanes 2/3 run their (discarded) chain on zero operands — yy = z = 0, no extra
      // instruction: fewer toggling bits, a higher clock (A/B 28.86 -> 28.61 us/tick).
      // (Freezing the unused yaw of lanes 0/1 as well, by per-lane RK4 weights 0: 28.98.)
      sk.ch[0].lw = 0.0;
      sk.ch[0].sg = 0.0;
      sk.ch[0].B = 0.0;
      sk.ch[0].nsB = 0.0;
    }
    const FusedK fq = make_fused(veh, sk, Ts, kScaled);
    const fm::FmK K = [&] {
      if constexpr (XM) return fm::FmK::load<kLeanLA && INTEG == 0>();
      else return K0;
    }();
    for (int j = 0; j < cpl; ++j) {
      const int c = g + j * G;
      if (c >= C) break;
      bool bad = false;
      double J;
      if (kSplit && diagQP)             // launch-uniform (kernel arguments)
        J = rollout<INTEG, STAGE, LPM, XM, true, kSplit>(a, c, n, x0, sx, su, veh, t, sk, q, Ts, up0, up1, K, fq, bad);
      else
        J = rollout<INTEG, STAGE, LPM, XM, true>(a, c, n, x0, sx, su, veh, t, sk, q, Ts, up0, up1, K, fq, bad);
      if (LPM == 2) {                   // the pair shares one rollout: re-run both or neither
        const int bi = bad;
        bad = __builtin_amdgcn_mov_dpp(bi, kPair0, 0xF, 0xF, false) |
              __builtin_amdgcn_mov_dpp(bi, kPair1, 0xF, 0xF, false);
      } else if (LPM == 4) {            // the quad shares one rollout
        int bi = bad;
        bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX1, 0xF, 0xF, false);
        bi |= __builtin_amdgcn_mov_dpp(bi, kQuadX2, 0xF, 0xF, false);
        bad = bi;
      }
      if (__builtin_expect(__any(bad), 0)) {
        bool unused = false;
        if (bad) J = rollout<INTEG, STAGE, LPM, XM, false>(a, c, n, x0, sx, su, veh, t, sk, q, Ts, up0, up1, K, fq, unused);
      }
      if (sub == 0) {
        if (a.cost_out) a.cost_out[n * C + c] = J;
        nf += !isfinite(J);
      }
      if (less_nan_last(J, c, bv, bc)) {
        bv = J;
        bc = c;
      }
    }
  }
  LA_STAMP(blk, 2);
#ifdef LLAMPC_STAMPS
  if ((threadIdx.x & 63) == 0 && blk < 1024) g_la_wave[blk][threadIdx.x >> 6] = __builtin_amdgcn_s_memrealtime();
#endif
  // per-model argmin over its candidates: xor-shuffles across the model's lanes inside a
  // wave, then (a model spanning 2 or 4 waves: G*LPM in {128, 256}) across its waves in LDS
  const int span = G * LPM;
  for (int off = (span < 64 ? span : 64) >> 1; off >= LPM; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int64_t oc = __shfl_xor(bc, off, 64);
    if (less_nan_last(ov, oc, bv, bc)) {
      bv = ov;
      bc = oc;
    }
  }
  int par = 0;
  if (span > 64) {                                  // block-uniform
    double* sv = sc.sv + 4 * par;
    int64_t* si = sc.si + 4 * par;
    par ^= 1;
    if ((threadIdx.x & 63) == 0) {
      sv[threadIdx.x >> 6] = bv;
      si[threadIdx.x >> 6] = bc;
    }
    __syncthreads();
    const int w0 = (int)(threadIdx.x / span) * (span / 64);
    bv = sv[w0];
    bc = si[w0];
    for (int k = 1; k < span / 64; ++k) {
      if (less_nan_last(sv[w0 + k], si[w0 + k], bv, bc)) {
        bv = sv[w0 + k];
        bc = si[w0 + k];
      }
    }
  }
  if (live && g == 0 && sub == 0) {
    if (a.poll) {                       // tagged words only (SoA: coalesced rows); C = 1: the
      // candidate is 0, so only the cost's two words (final_poll)
      st_wt(&a.la_tag[n], tag_word(a.seq, (uint32_t)(__double_as_longlong(bv) >> 32)));
      st_wt(&a.la_tag[a.n + n], tag_word(a.seq, (uint32_t)__double_as_longlong(bv)));
      st_wt(&a.la_tag[2 * a.n + n], tag_word(a.seq, (uint32_t)(int32_t)bc));
    } else {
      st_wt(&a.best_cand[n], (int32_t)bc);
      st_wt(&a.best_cost[n], bv);
    }
  }
  // per-block argmin over (model, candidate) in flattened order (goff+n)*C + c
  const int64_t key = (live && bc != kNoIndex && g == 0 && sub == 0) ? (a.goff + n) * C + bc : kNoIndex;
  la_publish(a, blk, sc, par, (key == kNoIndex) ? __builtin_nan("") : bv, key, nf);
  LA_STAMP(blk, 3);
}

struct Ent {
  double v;
  int64_t i;
};

__device__ __forceinline__ bool ent_less(const Ent& x, const Ent& y) {
  return less_nan_last(x.v, x.i, y.v, y.i);
}

// Element k (0-based) of merge(A, B), |A| = |B| = K, both sorted with sentinel padding:
// co-rank binary search (merge path), ~log2(K) dependent LDS reads.  E has fields v, i.
template <typename E>
__device__ __forceinline__ E merge_path_at(const E* A, const E* B, int K, int k) {
  int lo = 0, hi = k;                       // i = elements taken from A before output k
  while (lo < hi) {
    const int i = (lo + hi) >> 1;
    if (less_nan_last(A[i].v, A[i].i, B[k - i - 1].v, B[k - i - 1].i)) lo = i + 1;
    else hi = i;
  }
  const int i = lo, j = k - lo;
  return (less_nan_last(A[i].v, A[i].i, B[j].v, B[j].i)) ? A[i] : B[j];
}

// Tree-merge L sorted K-lists in LDS (the cross-shard merge_kernel) (buf0 holds them; buf1
// same size); every output element of a level is computed by its own thread.  Returns the
// buffer holding the merged list (first K entries).
template <typename E>
__device__ __forceinline__ E* tree_merge(E* buf0, E* buf1, int L, int K) {
  E* src = buf0;
  E* dst = buf1;
  while (L > 1) {
    const int P = (L + 1) >> 1;
    for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
      const int p = t / K, k = t - p * K;
      const E* A = src + (size_t)(2 * p) * K;
      dst[t] = (2 * p + 1 < L) ? merge_path_at(A, A + K, K, k) : A[k];
    }
    __syncthreads();
    E* tmp = src;
    src = dst;
    dst = tmp;
    L = P;
  }
  return src;
}

// ------------------------------------------------------------------------------------
// Completion stages run by ticket winners inside the plan launch.
// lb_final  (last look-back block): argmin over the blocks' argmins; tree merge of the
//           blocks' sorted top-K lists in LDS; writes the look-back fields of the record.
//           It runs while look-ahead blocks are still rolling out, off the critical path.
// final     (last block overall): look-ahead best over the block partials, the selected
//           model's choice, each top-K model's best candidate; completes the record.
// ------------------------------------------------------------------------------------
// The controller tick's use of lb_final (SEL = true, ctl.hip): the selection is also published
// for the look-ahead blocks waiting on it — tagged words [K + 1] (local model index of top-K
// entry k, kNoLocal = none; entry K: the argmin) — and kept in LDS for the completion.
// SEL = 2 (the sharded controller, ctl.hip ctl_exchange): nothing is published and no record
// field written — the shard's top-K and argmin (local index, value) go to ids / xv for the
// exchange, which publishes the MERGED selection.
struct CtlSel {
  uint64_t* tag;
  uint32_t seq;
  uint32_t* ids;         // LDS [K + 1]
  double* dr;            // LDS [K]: bank Dr / Df of the top-K (NaN: none)
  double* df;
  double* xv;            // LDS [K + 1]: SEL = 2, the entries' window means
  int32_t* xlate;        // LDS [1]: the exchange gave up waiting for a peer (status)
};

template <int SEL = 0>
__device__ __forceinline__ void lb_final(const FinalLaunch& f, unsigned char* smem, const CtlSel* cs = nullptr) {
  STAMP(0);
  const int tid = threadIdx.x;
  const int L = f.nb_lb;                   // one sorted K-list per look-back block
  const int La = f.nb_lb * kWaves;         // one argmin per look-back wave
  const int K = f.K, M = L * K;
  // LDS (SoA, contiguous scans): thr[2] | key[M] | val[M] | hk[L] | ck[M] | am[La] | id[M] |
  // hid[L] | cid[M] | ce[M] | top[KMAX] | cnt.  Missing entries
  // take ids above every model's, unique per position, so (key, id) is a total order.
  uint64_t* thr = reinterpret_cast<uint64_t*>(smem + kScratchBytes);   // T: key, id
  uint64_t* key = thr + 2;
  double* val = reinterpret_cast<double*>(key + M);
  uint64_t* hk = reinterpret_cast<uint64_t*>(val + M);
  uint64_t* ck = hk + L;
  Ent* am = reinterpret_cast<Ent*>(ck + M);    // the waves' argmins, same round trip
  uint32_t* id = reinterpret_cast<uint32_t*>(am + La);
  uint32_t* hid = id + M;
  uint32_t* cid = hid + L;
  int* ce = reinterpret_cast<int*>(cid + M);
  int* top = ce + M;                           // [K] entry of each output rank
  int* cnt = top + LLAMPC_KMAX;
  auto local = [&](int64_t gi) { return gi == kNoIndex ? kNoLocal : (uint32_t)(gi - f.goff); };
  for (int e = tid; e < M; e += kBlock) {
    const double v = ld_wt(&f.tk_val[e]);
    const uint32_t l = local(ld_wt(&f.tk_idx[e]));
    const uint64_t k = l == kNoLocal ? ~0ull : order_key(v);
    const uint32_t i = l == kNoLocal ? kNoModelId + (uint32_t)e : l;
    key[e] = k;
    val[e] = v;
    id[e] = i;
    if (e % K == 0) {
      hk[e / K] = k;
      hid[e / K] = i;
    }
  }
  for (int b = tid; b < La; b += kBlock) am[b] = Ent{ld_wt(&f.am_val[b]), ld_wt(&f.am_idx[b])};
  if (tid == 0) {
    *cnt = 0;
    thr[0] = ~0ull;                          // L < K: every entry is a candidate
    thr[1] = 0xFFFFFFFFull;
  }
  __syncthreads();
  STAMP(1);
  // top-K of the L sorted lists without serial rounds (a wave pick per output rank cost
  // ~1 us per rank): T = the K-th smallest list head bounds the K-th smallest entry (the K
  // smallest heads are K entries <= T), so the top-K lies in {entries <= T} — K to a few K
  // entries on real banks — and each candidate's rank among the candidates is its output
  // rank.  The scans read contiguous LDS (broadcast), unrolled so loads overlap.
  auto lt = [](uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
    return (int)(ka < kb) | ((int)(ka == kb) & (int)(ia < ib));
  };
  if (L >= K) {
    for (int h = tid; h < L; h += kBlock) {
      const uint64_t mk = hk[h];
      const uint32_t mi = hid[h];
      int r = 0;
#pragma unroll 8
      for (int j = 0; j < L; ++j) r += lt(hk[j], hid[j], mk, mi);
      if (r == K - 1) {
        thr[0] = mk;
        thr[1] = mi;
      }
    }
    __syncthreads();
  }
  STAMP(6);
  const uint64_t tk = thr[0];
  const uint32_t ti = (uint32_t)thr[1];
  for (int e = tid; e < M; e += kBlock) {
    const uint64_t k = key[e];
    const uint32_t i = id[e];
    if (!lt(tk, ti, k, i)) {
      const int slot = atomicAdd(cnt, 1);
      ck[slot] = k;
      cid[slot] = i;
      ce[slot] = e;
    }
  }
  __syncthreads();
  STAMP(7);
  const int c = *cnt;                      // >= K (the K smallest heads, or all M >= K)
  for (int q = tid; q < c; q += kBlock) {
    const uint64_t mk = ck[q];
    const uint32_t mi = cid[q];
    int r = 0;
#pragma unroll 8
    for (int j = 0; j < c; ++j) r += lt(ck[j], cid[j], mk, mi);
    if (r < K) top[r] = ce[q];
  }
  __syncthreads();
  if (tid >= 64) return;                   // one wave finishes; the caller re-converges
  const int lane = tid;
  // argmin over the waves' argmins (rt.py:359)
  double v = f.nan_first ? __builtin_inf() : __builtin_nan("");
  uint32_t li = kNoLocal;
  for (int b = lane; b < La; b += 64) {
    const double bv = am[b].v;
    const uint32_t bl = local(am[b].i);
    const bool t = (int)(bl != kNoLocal) &
                   (int)(f.nan_first ? less_bf<1>(bv, bl, v, li) : less_bf<0>(bv, bl, v, li));
    v = t ? bv : v;
    li = t ? bl : li;
  }
  if (f.nan_first) wave_pick_nf(v, li);
  else wave_pick_nl(v, li);
  double kv = __builtin_nan("");
  uint32_t kl = kNoLocal;
  if (lane < K) {
    const int e = top[lane];
    kl = id[e] >= kNoModelId ? kNoLocal : id[e];
    kv = val[e];
  }
  STAMP(2);
  if constexpr (SEL == 2) {                // the sharded controller: the shard's lists only
    if (lane < K) {
      cs->ids[lane] = kl;
      cs->xv[lane] = kv;
    }
    if (lane == 0) {
      cs->ids[K] = li;
      cs->xv[K] = v;
    }
    return;
  }
  if constexpr (SEL == 1) {                // the controller's selection first: the look-ahead
    if (lane < K) {                        // blocks wait on it (the record's stores below wait
      cs->ids[lane] = kl;                  // on the Pacejka loads of the top-K rows)
      st_wt(&cs->tag[lane], tag_word(cs->seq, kl));
    }
    if (lane == 0) {
      cs->ids[K] = li;
      st_wt(&cs->tag[K], tag_word(cs->seq, li));
    }
  }
  // Every record field is stored write-through (sc1): on the ticket path another block —
  // possibly on another XCD — completes the record, and peer_finish reads all of it back
  // with sc1 loads (MI355X_MICROARCH.md "Valid forms": sc1 stores AND sc1 loads).
  llampc_plan_out* o = f.out;
  if (lane < LLAMPC_KMAX) {
    const int k = lane;
    if (k < K && kl != kNoLocal) {
      st_wt(&o->topk[k], f.goff + (int64_t)kl);      // read by final_select
      st_wt(&o->topk_val[k], kv);
      st_wt(&o->topk_Df[k], f.params[2 * f.n + kl]);
      st_wt(&o->topk_Dr[k], f.params[5 * f.n + kl]);
    } else {
      const double nan = __builtin_nan("");
      st_wt(&o->topk[k], (int64_t)-1);
      st_wt(&o->topk_val[k], nan);
      st_wt(&o->topk_Df[k], nan);
      st_wt(&o->topk_Dr[k], nan);
    }
  }
  if (lane == 0) {
    st_wt(&o->lb_best, li == kNoLocal ? (int64_t)-1 : f.goff + (int64_t)li);
    st_wt(&o->lb_best_val, li == kNoLocal ? __builtin_nan("") : v);
  }
  if constexpr (SEL == 1) {
    if (lane < K) {
      const bool have = kl != kNoLocal;
      cs->dr[lane] = have ? f.params[5 * f.n + kl] : __builtin_nan("");
      cs->df[lane] = have ? f.params[2 * f.n + kl] : __builtin_nan("");
    }
  }
}

// Completes the record from the gathered look-ahead results (final_select / final_poll).
__device__ __forceinline__ void final_write(const FinalLaunch& f, bool lb, int64_t sel, bool owned,
                                            int32_t kcand, double kcost, int32_t scand,
                                            double scost, double lav, int64_t lai, int nf,
                                            int status = 0) {
  const int tid = threadIdx.x;
  llampc_plan_out* o = f.out;
  const double nan = __builtin_nan("");
  // sc1 stores like lb_final's: the fused peer exchange reads the whole record back sc1
  if (tid < LLAMPC_KMAX) {
    const int k = tid;
    if (!lb) {
      st_wt(&o->topk[k], (int64_t)-1);
      st_wt(&o->topk_val[k], nan);
      st_wt(&o->topk_Df[k], nan);
      st_wt(&o->topk_Dr[k], nan);
    }
    st_wt(&o->topk_cand[k], kcand);
    st_wt(&o->topk_cost[k], kcost);
  }
  if (tid == 0) {
    if (!lb) {
      st_wt(&o->lb_best, (int64_t)-1);
      st_wt(&o->lb_best_val, nan);
    }
    st_wt(&o->window_count, f.window_count);
    st_wt(&o->window_full, f.full);
    st_wt(&o->K, f.K);
    st_wt(&o->n_nonfinite, nf);
    st_wt(&o->status, status);
    st_wt(&o->sel_model, sel);
    st_wt(&o->sel_owned, (int32_t)owned);
    st_wt(&o->sel_cand, scand);
    st_wt(&o->sel_cost, scost);
    const bool la_ok = f.do_la && lai != kNoIndex;
    st_wt(&o->la_best_model, la_ok ? lai / f.C : (int64_t)-1);
    st_wt(&o->la_best_cand, la_ok ? (int32_t)(lai % f.C) : (int32_t)-1);
    st_wt(&o->la_best_cost, la_ok ? lav : nan);
    __hip_atomic_store(&f.tickets[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&f.tickets[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every look-ahead block has published (polled) or drawn its ticket (ticket path) after
    // its last work-queue take: the next launch starts from unit 0
    if (f.wq) __hip_atomic_store(f.wq, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (f.host_tag) {                     // host completion: every record store performed, then the tag
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(f.host_tag, f.host_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  STAMP(5);
#ifdef LLAMPC_STAMPS
  if (tid == 0) g_stamp_launch++;
#endif
}

__device__ __forceinline__ void final_select(const FinalLaunch& f, const Scratch& sc) {
  STAMP(3);
  const int tid = threadIdx.x;
  llampc_plan_out* o = f.out;
  const bool lb = f.do_lb && f.full;
  // Every load that does not depend on the look-ahead reduction is issued first, so the
  // tail costs two dependent round trips, not three: the look-back result lb_final left in
  // the record (top-K ids, lb_best) and then those models' best candidates.
  const int64_t idk = (lb && tid < LLAMPC_KMAX) ? ld_wt(&o->topk[tid]) : -1;
  const int64_t lbi = (tid == 0 && lb) ? ld_wt(&o->lb_best) : -1;
  const int64_t sel = lbi >= 0 ? lbi : f.current_model;
  const bool owned = sel >= f.goff && sel < f.goff + f.n;
  const bool have = lb && tid < LLAMPC_KMAX && idk >= 0 && f.do_la;
  int32_t kcand = -1, scand = -1;
  double kcost = __builtin_nan(""), scost = __builtin_nan("");
  if (have) {
    kcand = ld_wt(&f.best_cand[idk - f.goff]);
    kcost = ld_wt(&f.best_cost[idk - f.goff]);
  }
  if (tid == 0 && owned && f.do_la) {
    scand = ld_wt(&f.best_cand[sel - f.goff]);
    scost = ld_wt(&f.best_cost[sel - f.goff]);
  }
  double lav = __builtin_nan("");
  int64_t lai = kNoIndex;
  int nf = 0;
  if (f.do_la) {
    for (int b = tid; b < f.nb_la; b += kBlock) {
      nf += ld_wt(&f.pnf[b]);
      const int64_t pi = ld_wt(&f.pidx[b]);
      const double pv = ld_wt(&f.pv[b]);
      const bool t = (int)(pi != kNoIndex) & (int)less_bf<0>(pv, pi, lav, lai);
      lav = t ? pv : lav;
      lai = t ? pi : lai;
    }
    wave_pick_nl64(lav, lai);           // converged: every lane of the block is here
    nf = wave_sum(nf);
    if ((tid & 63) == 0) {
      sc.sv[4 + (tid >> 6)] = lav;
      sc.si[4 + (tid >> 6)] = lai;
      sc.sn[tid >> 6] = nf;
    }
    __syncthreads();
    lav = sc.sv[4];
    lai = sc.si[4];
    nf = sc.sn[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) {
      const bool t = (int)(sc.si[4 + w] != kNoIndex) & (int)less_bf<0>(sc.sv[4 + w], sc.si[4 + w], lav, lai);
      lav = t ? sc.sv[4 + w] : lav;
      lai = t ? sc.si[4 + w] : lai;
      nf += sc.sn[w];
    }
  }
  STAMP(4);
  final_write(f, lb, sel, owned, kcand, kcost, scand, scost, lav, lai, nf);
}

// Polled completion (f.poll): run by the look-back ticket winner after lb_final.  Each thread
// spins on its share of the tagged words — the look-ahead blocks' partials (5 words each),
// the top-K models' and the selected model's results (3 words each) — until every word it
// loads carries this launch's tag; one block barrier then joins them.  The blocks it waits
// for never wait, so it cannot deadlock; a bound (f.poll x 2^16 s_memrealtime ticks, 100 MHz,
// scaled by the host with the launch's rollout steps: poll_bound_ticks in capi.hip) ends a
// poll that could never finish (a bug) with status LLAMPC_STATUS_POLL_TIMEOUT in the record
// instead of a hang.
constexpr int kPollTimeoutStatus = LLAMPC_STATUS_POLL_TIMEOUT;
__device__ __forceinline__ void final_poll(const FinalLaunch& f, const Scratch& sc) {
  STAMP(3);
  const int tid = threadIdx.x;
  llampc_plan_out* o = f.out;
  const bool lb = f.do_lb && f.full;
  const int64_t idk = (lb && tid < LLAMPC_KMAX) ? ld_wt(&o->topk[tid]) : -1;
  const int64_t lbi = (tid == 0 && lb) ? ld_wt(&o->lb_best) : -1;
  const int64_t sel = lbi >= 0 ? lbi : f.current_model;
  const bool owned = sel >= f.goff && sel < f.goff + f.n;
  // this thread's model record: top-K entry tid, or (thread 0's second slot) the selection
  const int64_t mk = (lb && tid < LLAMPC_KMAX && idk >= 0) ? idk - f.goff : -1;
  const int64_t ms = (tid == 0 && owned) ? sel - f.goff : -1;
  const int nbt = (f.nb_la + kBlock - 1) / kBlock;        // block records per thread
  uint64_t kw[3] = {0, 0, 0}, sw[3] = {0, 0, 0};
  double lav = __builtin_nan("");
  int64_t lai = kNoIndex;
  int nf = 0;
  int status = 0;
  // every thread spins on its own words (no block barrier per round: a thread's next loads
  // issue as soon as its previous ones return); one barrier after all are current
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t bound = (uint64_t)(uint32_t)f.poll << 16;
  bool late = false;
  if (mk >= 0) {
    for (;;) {
#pragma unroll
      for (int w = 0; w < 3; ++w) kw[w] = ld_wt(&f.la_tag[w * f.n + mk]);
      if ((int)tag_ok(kw[0], f.seq) & (int)tag_ok(kw[1], f.seq) & (int)tag_ok(kw[2], f.seq)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > bound) { late = true; break; }
    }
  }
  if (ms >= 0) {
    for (;;) {
#pragma unroll
      for (int w = 0; w < 3; ++w) sw[w] = ld_wt(&f.la_tag[w * f.n + ms]);
      if ((int)tag_ok(sw[0], f.seq) & (int)tag_ok(sw[1], f.seq) & (int)tag_ok(sw[2], f.seq)) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > bound) { late = true; break; }
    }
  }
  for (int j = 0; j < nbt; ++j) {
    const int b = tid + j * kBlock;
    if (b < f.nb_la) {
      uint64_t r[5];
      for (;;) {
#pragma unroll
        for (int w = 0; w < 5; ++w) r[w] = ld_wt(&f.blk_tag[5 * (int64_t)b + w]);
        if ((int)tag_ok(r[0], f.seq) & (int)tag_ok(r[1], f.seq) & (int)tag_ok(r[2], f.seq) &
            (int)tag_ok(r[3], f.seq) & (int)tag_ok(r[4], f.seq))
          break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) { late = true; break; }
      }
      const double pv = __longlong_as_double((long long)join_words(r[0], r[1]));
      const int64_t pi = (int64_t)join_words(r[2], r[3]);
      nf += (int)(uint32_t)r[4];
      const bool t = (int)(pi != kNoIndex) & (int)less_bf<0>(pv, pi, lav, lai);
      lav = t ? pv : lav;
      lai = t ? pi : lai;
    }
  }
  // the waves' late flags travel with the block reduction's LDS exchange below (one barrier;
  // no __syncthreads_or: its static LDS would break the launches' full-LDS requests)
  unsigned char* late_w = reinterpret_cast<unsigned char*>(sc.sv) + kLateOff;
  const int wlate = __any((int)late);
  int32_t kcand = -1, scand = -1;
  double kcost = __builtin_nan(""), scost = __builtin_nan("");
  if (mk >= 0 && f.do_la) {
    kcost = __longlong_as_double((long long)join_words(kw[0], kw[1]));
    kcand = (int32_t)(uint32_t)kw[2];
  }
  if (ms >= 0 && f.do_la) {
    scost = __longlong_as_double((long long)join_words(sw[0], sw[1]));
    scand = (int32_t)(uint32_t)sw[2];
  }
  wave_pick_nl64(lav, lai);
  nf = wave_sum(nf);
  if ((tid & 63) == 0) {
    sc.sv[4 + (tid >> 6)] = lav;
    sc.si[4 + (tid >> 6)] = lai;
    sc.sn[tid >> 6] = nf;
    late_w[tid >> 6] = (unsigned char)wlate;
  }
  __syncthreads();
  lav = sc.sv[4];
  lai = sc.si[4];
  nf = sc.sn[0];
  int anyl = late_w[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) {
    const bool t = (int)(sc.si[4 + w] != kNoIndex) & (int)less_bf<0>(sc.sv[4 + w], sc.si[4 + w], lav, lai);
    lav = t ? sc.sv[4 + w] : lav;
    lai = t ? sc.si[4 + w] : lai;
    nf += sc.sn[w];
    anyl |= late_w[w];
  }
  if (anyl) status = kPollTimeoutStatus;
  STAMP(4);
  final_write(f, lb, sel, owned, kcand, kcost, scand, scost, lav, lai, nf, status);
}

// Cross-shard merge after the all-gather: one wave.  Scalars by lane-parallel reads and
// shuffles; the shards' sorted top-K lists by the LDS tree merge.  merge.hpp holds the
// same semantics as straight-line host code (llampc_merge); the tests check both agree.
// A top-K entry of the cross-shard merge with its position in the gathered lists.
struct EntS {
  double v;
  int64_t i;
  int32_t src;
  int32_t pad;
};

// The merge proper over G records already staged in LDS at `rec` (their sorted top-K lists
// are ranked in `lists`, 2 G KMAX EntS); thread 0 writes the scalars, threads < KMAX the
// top-K.  `late` (the peer exchange gave up waiting) is or-ed into the status.
__device__ __forceinline__ void merge_staged(const llampc_plan_out* rec, int32_t G, int32_t nan_first,
                                             llampc_plan_out* m, EntS* lists, int32_t late) {
  const int tid = threadIdx.x;
  const int K = rec[0].K;
  const int M = G * K;
  EntS* buf0 = lists;
  EntS* buf1 = buf0 + M;
  for (int e = tid; e < M; e += kBlock) {
    const int g = e / K, j = e - g * K;
    const int64_t id = rec[g].topk[j] < 0 ? kNoIndex : rec[g].topk[j];
    buf0[e] = EntS{id == kNoIndex ? __builtin_nan("") : rec[g].topk_val[j], id, e, 0};
  }
  // wave 0: look-back argmin over the shards' local argmins; look-ahead best; counts; owners
  // — DPP wave reductions over lanes g < G (no LDS shuffles)
  double bv = nan_first ? __builtin_inf() : __builtin_nan("");
  int64_t bi = kNoIndex;
  double av = __builtin_nan("");
  int64_t akey = kNoIndex;              // (model << 24 | candidate): la_less's order
  int nf = 0;
  uint32_t owner_lb = kNoLocal, owner_sel = kNoLocal;
  if (tid < 64) {
    const int lane = tid;
    for (int g = lane; g < G; g += 64) {
      const llampc_plan_out& p = rec[g];
      if (p.lb_best >= 0 && key_less(nan_first, p.lb_best_val, p.lb_best, bv, bi)) {
        bv = p.lb_best_val;
        bi = p.lb_best;
      }
      nf += p.n_nonfinite;
      const int64_t k2 = p.la_best_model >= 0 ? ((int64_t)p.la_best_model << 24) | (uint32_t)p.la_best_cand : kNoIndex;
      if (k2 != kNoIndex && less_nan_last(p.la_best_cost, k2, av, akey)) {
        av = p.la_best_cost;
        akey = k2;
      }
    }
    if (nan_first) wave_min<1>(bv, bi);
    else wave_min<0>(bv, bi);
    wave_min<0>(av, akey);
    nf = wave_sum(nf);
    uint32_t ol = kNoLocal, os = kNoLocal;
    for (int g = lane; g < G; g += 64) {
      if (bi != kNoIndex && rec[g].lb_best == bi) ol = min(ol, (uint32_t)g);
      if (rec[g].sel_owned) os = min(os, (uint32_t)g);
    }
    owner_lb = wave_min_u32(ol);
    owner_sel = wave_min_u32(os);
  }
  const int64_t am = akey == kNoIndex ? kNoIndex : (akey >> 24);
  const int32_t ac = akey == kNoIndex ? INT32_MAX : (int32_t)(akey & 0xFFFFFF);
  __syncthreads();
  const EntS* r = tree_merge(buf0, buf1, G, K);
  if (tid < LLAMPC_KMAX) {
    const int k = tid;
    const bool have = k < K && r[k].i != kNoIndex;
    if (have) {                          // the merged entry carries its gathered position
      const int src = r[k].src, g = src / K, j = src - g * K;
      m->topk[k] = r[k].i;
      m->topk_val[k] = r[k].v;
      m->topk_Df[k] = rec[g].topk_Df[j];
      m->topk_Dr[k] = rec[g].topk_Dr[j];
      m->topk_cand[k] = rec[g].topk_cand[j];
      m->topk_cost[k] = rec[g].topk_cost[j];
    } else {
      m->topk[k] = -1;
      m->topk_val[k] = m->topk_Df[k] = m->topk_Dr[k] = m->topk_cost[k] =
          k < K ? __builtin_nan("") : 0.0;
      m->topk_cand[k] = -1;
    }
  }
  if (tid != 0) return;
  const llampc_plan_out& p0 = rec[0];
  m->window_count = p0.window_count;
  m->window_full = p0.window_full;
  m->K = K;
  int32_t st = late ? kPollTimeoutStatus : 0;
  for (int g = 0; g < G; ++g) st |= rec[g].status;
  m->status = st;
  m->lb_best = bi == kNoIndex ? -1 : bi;
  m->lb_best_val = bi == kNoIndex ? __builtin_nan("") : bv;
  if (m->window_full && owner_lb != kNoLocal) {
    m->sel_model = bi;
    m->sel_owned = rec[owner_lb].sel_owned;
    m->sel_cand = rec[owner_lb].sel_cand;
    m->sel_cost = rec[owner_lb].sel_cost;
  } else {                               // the first shard owning sel (merge.hpp)
    m->sel_model = p0.sel_model;
    m->sel_owned = owner_sel != kNoLocal;
    m->sel_cand = owner_sel != kNoLocal ? rec[owner_sel].sel_cand : -1;
    m->sel_cost = owner_sel != kNoLocal ? rec[owner_sel].sel_cost : __builtin_nan("");
  }
  m->la_best_model = am == kNoIndex ? -1 : am;
  m->la_best_cand = am == kNoIndex ? -1 : ac;
  m->la_best_cost = av;
  m->n_nonfinite = nf;
}

// Poll this rank's mailbox slots [G][kRecWords] (tick parity already applied) for the G-1 peer
// records of tick `seq`, unpacking the payloads into rec32 (LDS).  Every round issues ALL of a
// thread's loads before it checks any (unconditional loads — a load under a per-word
// condition gets its own branch and vmcnt(0) wait, i.e. one memory round trip per word: ~11
// sequential round trips per thread at G = 8); words already valid, past the end or in this
// rank's own slot (never read back) reload a harmless address in that own slot.  Returns 1 if
// `bound` s_memrealtime ticks pass first.
// A peer exchange that gave up waiting (a missing rank): the merged record is this rank's own
// record with status LLAMPC_STATUS_POLL_TIMEOUT (the missing slots hold no record to merge).
__device__ __forceinline__ void peer_timeout_record(const uint32_t* rec32, int rank, llampc_plan_out* m) {
  const uint32_t* mine = rec32 + (size_t)rank * kRecWords;
  uint32_t* dst = reinterpret_cast<uint32_t*>(m);
  constexpr int kStatus = (int)(offsetof(llampc_plan_out, status) / 4);
  for (int w = threadIdx.x; w < kRecWords; w += kBlock)
    dst[w] = w == kStatus ? (uint32_t)LLAMPC_STATUS_POLL_TIMEOUT : mine[w];
}

template <int kPer>
__device__ __forceinline__ int poll_mailbox(const uint64_t* own, int G, int rank, uint32_t seq,
                                            uint64_t bound, uint32_t* rec32) {
  static_assert(kPer <= 64, "one need bit per word");
  const int tid = threadIdx.x;
  const int total = G * kRecWords, skip0 = rank * kRecWords, skip1 = skip0 + kRecWords;
  const int idle = skip0 + tid % kRecWords;      // this thread's harmless address
  uint64_t need = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int e = tid + j * kBlock;
    if (e < total && (e < skip0 || e >= skip1)) need |= 1ull << j;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (need) {
    uint64_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int e = ((need >> j) & 1) ? tid + j * kBlock : idle;
      v[j] = __hip_atomic_load(own + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

// Fused peer exchange, run by the block that completed this rank's record (after final_poll /
// final_select): the record's words are read back, pushed as tagged words into slot [seq & 1][rank] of every mailbox, and the
// px_G slots of this rank's mailbox are polled into LDS and merged (peer_exchange_kernel's
// protocol and merge; its comment has the slot-reuse argument).
__device__ __forceinline__ void peer_finish(const FinalLaunch& f, unsigned char* smem) {
  const int tid = threadIdx.x;
  const int G = f.px_G;
  constexpr int kW2 = kRecWords / 2;            // the record as 64-bit loads
  static_assert(kRecWords % 2 == 0, "record of whole 64-bit words");
  // The record is read back with sc1 loads after the block barrier.  This block wrote part
  // of it (final_write); on the ticket path lb_final wrote the rest in ANOTHER block, which
  // can sit on another XCD: every lb_final field is stored sc1 and every load here is sc1,
  // so the ticket hand-off is the "sc1 stores and loads both sides" form and no stale L2
  // line of last tick's record can be merged.  No agent-scope fence: on MI355X that is an
  // L2 writeback of the XCD (measured ~3 us per tick here).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const size_t slot0 = (size_t)(f.px_seq & 1) * G * kRecWords;
  const size_t mine = slot0 + (size_t)f.px_rank * kRecWords;
  const uint64_t* src = reinterpret_cast<const uint64_t*>(f.out);
  unsigned char* base = smem + 256;             // past the scratch the completion used
  uint32_t* rec32 = reinterpret_cast<uint32_t*>(base);
  uint64_t* rec_mine = reinterpret_cast<uint64_t*>(base + (size_t)f.px_rank * sizeof(llampc_plan_out));
  for (int w = tid; w < kW2; w += kBlock) {
    const uint64_t v = ld_wt(&src[w]);
    rec_mine[w] = v;                            // this rank's record: straight to LDS
    const uint64_t lo = tag_word(f.px_seq, (uint32_t)v), hi = tag_word(f.px_seq, (uint32_t)(v >> 32));
    for (int g = 0; g < G; ++g) {
      if (g == f.px_rank) continue;
      uint64_t* d = f.px_box[g] + mine + 2 * w;
      __hip_atomic_store(d, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(d + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const uint64_t* own = f.px_box[f.px_rank] + slot0;
  constexpr int kPerF = (kPeerFuseMax * kRecWords + kBlock - 1) / kBlock;
  int late = poll_mailbox<kPerF>(own, G, f.px_rank, f.px_seq, (uint64_t)f.px_bound << 16, rec32);
  EntS* lists = reinterpret_cast<EntS*>(base + (size_t)G * sizeof(llampc_plan_out));
  int* wave_late = reinterpret_cast<int*>(lists + 2 * (size_t)G * LLAMPC_KMAX);
  const int wl = __any(late);
  if ((tid & 63) == 0) wave_late[tid >> 6] = wl;
  __syncthreads();
  late = 0;
  for (int w = 0; w < kWaves; ++w) late |= wave_late[w];
  if (late) {                                   // block-uniform
    peer_timeout_record(rec32, f.px_rank, f.px_merged);
    return;
  }
  merge_staged(reinterpret_cast<const llampc_plan_out*>(base), G, f.nan_first, f.px_merged, lists, 0);
}

// ------------------------------------------------------------------------------------
// The tick: ONE launch.  Blocks [0, nb_lb) run the look-back, blocks [nb_lb, nb_lb+nb_la)
// the look-ahead (the halves are independent: x_{t-1} -> x_t vs. rollouts from x_t).
// Look-back blocks come first in dispatch order; the last of them merges the look-back
// (lb_final) while look-ahead blocks still run; the last block overall completes the
// llampc_plan_out record (final_select).
// ------------------------------------------------------------------------------------
template <int INTEG, bool STAGE, int LPM, int XM, bool PX = false, int WQ = 0>
__device__ __forceinline__ void plan_body(const LookbackLaunch& lb, const LookaheadLaunch& la,
                                          const FinalLaunch& fin, int G, int cpl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Scratch sc(smem);
  int* flag = reinterpret_cast<int*>(smem + kFlagOff);
  // WQ launches run kBlockWQ threads per block: every role but the work-queue look-ahead is
  // written for kBlock and its surplus waves leave at once (s_barrier waits for the waves
  // that have not ended)
  // block roles: look-back blocks first in the grid (dispatch order; the look-ahead blocks
  // first measured 26.82-26.92 -> 27.67-27.75 us per tick)
  const bool is_lb = (int)blockIdx.x < fin.nb_lb;
  const int lb_blk = (int)blockIdx.x, la_blk = (int)blockIdx.x - fin.nb_lb;
  if constexpr (wq_threads(WQ) > kBlock) {
    if (is_lb && threadIdx.x >= kBlock) return;
  }
  if (is_lb) {
    lookback_block(lb, lb_blk, sc);
    if (!ticket_last(&fin.tickets[0], (unsigned)fin.nb_lb, flag)) return;
    if (fin.full) {
      lb_final(fin, smem);
      // host completion: lb_final's record stores are performed before any later hand-off
      // (the final block, possibly another one, publishes the host tag after them)
      if (fin.host_tag) __threadfence_system();
    }
    if (fin.poll) {                   // the look-back winner completes the tick
      __syncthreads();
      final_poll(fin, sc);
      if constexpr (PX) peer_finish(fin, smem);
      return;
    }
  } else {
    lookahead_block<INTEG, STAGE, LPM, XM, WQ>(la, la_blk, G, cpl, smem, sc);
    if (fin.poll) return;                // published tagged records; no ticket
    if constexpr (wq_threads(WQ) > kBlock) {
      if (threadIdx.x >= kBlock) return;
    }
  }
  const unsigned expected = (unsigned)fin.nb_la + (fin.nb_lb > 0 ? 1u : 0u);
  if (!ticket_last(&fin.tickets[1], expected, flag)) return;
  final_select(fin, sc);
  if constexpr (PX) peer_finish(fin, smem);
}

// PX: the sharded tick's fused peer exchange (a separate instantiation, so the plain tick's
// code is unchanged: inlining it into every variant cost the headline tick 0.5 us)
template <int INTEG, bool STAGE, int LPM, int XM, bool PX = false, int WQ = 0>
__global__ __launch_bounds__(wq_threads(WQ)) void plan_kernel(LookbackLaunch lb, LookaheadLaunch la,
                                                      FinalLaunch fin, int G, int cpl) {
  plan_body<INTEG, STAGE, LPM, XM, PX, WQ>(lb, la, fin, G, cpl);
}

// The same tick with its inputs in the kernarg segment (InlinePack): the pointers are set to
// the pack's fields, read by flat loads like any other input (no H2D copy on the host path).
template <int LPM>
__global__ __launch_bounds__(kBlock) void plan_kernel_inl(LookbackLaunch lb, LookaheadLaunch la,
                                                          FinalLaunch fin, int G, int cpl,
                                                          InlinePack pk) {
  const double* v = pk.v;
  lb.x_prev = v;
  lb.u_prev = v + 6;
  lb.x_now = v + 8;
  la.x0 = v + 8;
  la.uprev = v + 14;
  la.xref = v + 16;
  la.U = v + 16 + 2 * (la.H + 1);
  plan_body<0, true, LPM, 0>(lb, la, fin, G, cpl);
}

constexpr size_t kOneBlockPerCuLds = 82 * 1024;

template <typename KERN>
static void allow_lds(KERN k) {
  static bool done = false;             // once per instantiation (idempotent if raced)
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)(160 * 1024));
    done = true;
  }
}

template <int INTEG, bool STAGE, int PX, int WQ>
static void launch_plan_wq(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f,
                           int G, int cpl, size_t lds, hipStream_t s) {
  allow_lds(plan_kernel<INTEG, STAGE, 1, 0, PX, WQ>);
  hipLaunchKernelGGL((plan_kernel<INTEG, STAGE, 1, 0, PX, WQ>), dim3(f.nb_lb + f.nb_la), dim3(wq_threads(WQ)),
                     lds, s, lb, la, f, G, cpl);
}

template <int INTEG, bool STAGE, int LPM>
static void launch_plan_t(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f,
                          int G, int cpl, size_t lds, hipStream_t s, int wq = 0) {
  lds = std::max(lds, kOneBlockPerCuLds);
  if constexpr (INTEG == LLAMPC_RK4 && LPM == 1) {
    if (wq) {                            // work queue: given xref only (launch_plan checks)
      if constexpr (STAGE) {
        if (wq == 2) {
          if (f.px_G) launch_plan_wq<INTEG, STAGE, 1, 2>(lb, la, f, G, cpl, lds, s);
          else launch_plan_wq<INTEG, STAGE, 0, 2>(lb, la, f, G, cpl, lds, s);
          return;
        }
      }
      if (f.px_G) launch_plan_wq<INTEG, STAGE, 1, 1>(lb, la, f, G, cpl, lds, s);
      else launch_plan_wq<INTEG, STAGE, 0, 1>(lb, la, f, G, cpl, lds, s);
      return;
    }
  }
  if constexpr (INTEG == LLAMPC_RK4) {
    if (f.px_G) {                        // given xref only (launch_plan checks)
      allow_lds(plan_kernel<INTEG, STAGE, LPM, 0, true>);
      hipLaunchKernelGGL((plan_kernel<INTEG, STAGE, LPM, 0, true>), dim3(f.nb_lb + f.nb_la), dim3(kBlock), lds,
                         s, lb, la, f, G, cpl);
      return;
    }
  }
  if (la.xref_mode == LLAMPC_XREF_RACELINE) {
    allow_lds(plan_kernel<INTEG, STAGE, LPM, 1>);
    hipLaunchKernelGGL((plan_kernel<INTEG, STAGE, LPM, 1>), dim3(f.nb_lb + f.nb_la), dim3(kBlock), lds, s,
                       lb, la, f, G, cpl);
  } else {
    allow_lds(plan_kernel<INTEG, STAGE, LPM, 0>);
    hipLaunchKernelGGL((plan_kernel<INTEG, STAGE, LPM, 0>), dim3(f.nb_lb + f.nb_la), dim3(kBlock), lds, s,
                       lb, la, f, G, cpl);
  }
}

template <int LPM>
static void launch_plan_inl(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f,
                            int G, int cpl, size_t lds, hipStream_t s, const InlinePack& pk) {
  lds = std::max(lds, kOneBlockPerCuLds);
  allow_lds(plan_kernel_inl<LPM>);
  hipLaunchKernelGGL((plan_kernel_inl<LPM>), dim3(f.nb_lb + f.nb_la), dim3(kBlock), lds, s, lb, la, f,
                     G, cpl, pk);
}

// One variant group of the plan launch: (integrator, lanes per rollout), staged or not;
// explicitly instantiated in plan_*.hip (declared extern in kernels.hpp).
template <int INTEG, int LPM>
void launch_plan_group(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f, int G,
                       int cpl, bool stage, size_t lds, hipStream_t s, int wq) {
  if (stage) launch_plan_t<INTEG, true, LPM>(lb, la, f, G, cpl, lds, s, wq);
  else launch_plan_t<INTEG, false, LPM>(lb, la, f, G, cpl, lds, s, wq);
}

template <int LPM>
void launch_plan_inline_group(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f,
                              int G, int cpl, size_t lds, hipStream_t s, const InlinePack& pk) {
  launch_plan_inl<LPM>(lb, la, f, G, cpl, lds, s, pk);
}

}  // namespace llampc
