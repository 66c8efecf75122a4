// ctl.hpp — the controller tick (llampc_ctl_*, include/llampc.h): the whole LLA-MPC control
// step of rt.py:269-366 in ONE launch on the device — reference trajectory from the raceline
// library (planner.py:12-67 with mu-hat, the projection of track.py:147-160 / projection.py:
// 11-38), candidate control sequences (counter-based sampling; the build's stand-in for the
// per-tick IPOPT solve, nmpc.py:161-203), look-back + window + selection (rt.py:347-366), the
// look-ahead of the selected model and the top-K (rt.py:300-305), the mu-hat estimator
// (rt.py:326-344) and the controller state (x_{t-1}, u_{t-1}, the chosen sequence, projidx).
//
// The pure functions here are __host__ __device__ so a host harness (tests/native) checks
// them bitwise against the NumPy restatement of the test suite (tests/test_ctl_native.py).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kernels.hpp"
#include "llampc.h"

namespace llampc {

constexpr int kCtlSlotsMax = LLAMPC_KMAX + 1;   // look-ahead models: top-K + the selection
constexpr int kCtlSMax = 64;                    // mu-hat smoothing window (rt.py:68 uses 20)
constexpr int kCtlSegs = 9;                     // project_fast over raceline[:, p:p+10]

// Device-resident controller state, written by the block that completes a tick and read by
// the next tick's blocks (stream order between the launches).
struct CtlState {
  double x_prev[6];               // x_{t-1}     (the look-back transition's start)
  double u_prev[2];               // u_{t-1}     (applied input: the chosen sequence's first)
  double useq[LLAMPC_HMAX][2];    // the last chosen sequence (the candidates' base)
  double mu_pred;                 // mu-hat (rt.py:341); NaN until the first update
  double dr_hist[kCtlSMax];       // the last S appended Dr / Df means, ring by count % S
  double df_hist[kCtlSMax];
  int64_t current_model;          // rt.py:264 / 363 (global index)
  int32_t hist_count;             // means appended so far
  int32_t projidx;                // planner state (rt.py:279, 296)
  int32_t has_seq;                // a chosen sequence exists (tick >= 1)
  int32_t pad;
};

// ---- counter-based sampling ------------------------------------------------------------
// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; the Random123 / rocRAND generator):
// 10 rounds, the key bumped after each.  Known answers checked in tests (Random123 kat).
struct Philox4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ Philox4 philox4x32_10(Philox4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = Philox4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// The candidates' noise: one Philox4x32-10 call per (candidate, step) PAIR p = c H + k,
// counter (p, tick lo, tick hi, stream), key (seed lo, seed hi); input j takes the 16-bit
// halves (j = 0 low, 1 high) of the four words: z_j = (h0 + h1 + h2 + h3 + 2) 2^-16 - 2, the
// centred 4-term Irwin-Hall variate (variance 1/3 - 1/(3 2^32); exact in fp64), as the NLP
// search's (nlp.hip nlp_z2) — half the Philox calls of one call per value.
__host__ __device__ __forceinline__ void ctl_z2(uint32_t p, uint64_t tick, uint64_t seed, uint32_t stream, double& z0,
                                                double& z1) {
  const Philox4 w = philox4x32_10(Philox4{p, (uint32_t)tick, (uint32_t)(tick >> 32), stream}, (uint32_t)seed,
                                  (uint32_t)(seed >> 32));
  const uint32_t lo = (w.x & 0xFFFFu) + (w.y & 0xFFFFu) + (w.z & 0xFFFFu) + (w.w & 0xFFFFu) + 2u;
  const uint32_t hi = (w.x >> 16) + (w.y >> 16) + (w.z >> 16) + (w.w >> 16) + 2u;
  z0 = (double)lo * 0x1p-16 - 2.0;
  z1 = (double)hi * 0x1p-16 - 2.0;
}

// np.clip for float64 (numpy clip.cpp: _NPY_MIN(_NPY_MAX(x, lo), hi), NaN passes through)
__host__ __device__ __forceinline__ double np_clip(double x, double lo, double hi) {
  const double y = (x != x) ? x : (x > lo ? x : lo);
  return (y != y) ? y : (y < hi ? y : hi);
}

// Candidate element before the rate clip: base + noise (c >= 1), then the input bounds.
// base = the previous chosen sequence shifted one step (or uprev held); noise = z nscale_j
// with nscale_j = sqrt(3) sigma_j: two roundings, reproducible in NumPy.
__host__ __device__ __forceinline__ double ctl_cand_one(int c, int k, int j, int H, const double* prev_seq, double up_j,
                                                        double ns_j, double lo_j, double hi_j, double z) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  const double base = prev_seq ? prev_seq[2 * (k + 1 < H ? k + 1 : H - 1) + j] : up_j;
  double u = base;
  if (c > 0) {
    const double noise = z * ns_j;
    u = base + noise;
  }
  return np_clip(u, lo_j, hi_j);
}
// Both inputs of candidate c at step k into u[0], u[1], given the pair's variates (z0, z1).
__host__ __device__ __forceinline__ void ctl_cand_pair_z(int c, int k, int H, const double* prev_seq, const double* up,
                                                         const double* ns, const double* lo, const double* hi,
                                                         double z0, double z1, double* u) {
  u[0] = ctl_cand_one(c, k, 0, H, prev_seq, up[0], ns[0], lo[0], hi[0], z0);
  u[1] = ctl_cand_one(c, k, 1, H, prev_seq, up[1], ns[1], lo[1], hi[1], z1);
}
// ... drawing them (one Philox call).
__host__ __device__ __forceinline__ void ctl_cand_pair(int c, int k, int H, const double* prev_seq /*[H][2] or null*/,
                                                       const double* up, const double* ns, const double* lo,
                                                       const double* hi, uint64_t tick, uint64_t seed, uint32_t stream,
                                                       double* u) {
  double z0 = 0.0, z1 = 0.0;
  if (c > 0) ctl_z2((uint32_t)(c * H + k), tick, seed, stream, z0, z1);
  ctl_cand_pair_z(c, k, H, prev_seq, up, ns, lo, hi, z0, z1, u);
}

// The rate clip of one (candidate, input) chain in order over k (controller.py
// CandidateGenerator / nmpc.py:104-105): u_k <- clip(u_k, u_{k-1} - r, u_{k-1} + r), u_{-1} =
// uprev; r = rate_max Ts (< 0: unbounded).  u points at element (c, 0, j), stride 2.
__host__ __device__ __forceinline__ void ctl_rate_chain(double* u, int H, double up, double r) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  if (!(r >= 0.0)) return;
  double prev = up;
  int k = 0;
  for (; k + 8 <= H; k += 8) {          // eight loads ahead of the dependent clips
    double v[8];
#ifdef __clang__
#pragma unroll
#endif
    for (int i = 0; i < 8; ++i) v[i] = u[2 * (k + i)];
#ifdef __clang__
#pragma unroll
#endif
    for (int i = 0; i < 8; ++i) {
      const double lo = prev - r, hi = prev + r;
      prev = np_clip(v[i], lo, hi);
      u[2 * (k + i)] = prev;
    }
  }
  for (; k < H; ++k) {
    const double lo = prev - r, hi = prev + r;
    prev = np_clip(u[2 * k], lo, hi);
    u[2 * k] = prev;
  }
}

// ---- projection (track.py:147-160, projection.py:11-38) ---------------------------------
// numpy's 2-element dot as this stack computes it (x0 y0 rounded, then fused with x1 y1;
// checked on 10^5 pairs against np.dot) and np.linalg.norm(v, 2) = sqrt(v . v).
__host__ __device__ __forceinline__ double np_dot2(double a0, double a1, double b0, double b1) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  const double p = a0 * b0;
  return fma(a1, b1, p);
}
__host__ __device__ __forceinline__ double np_norm2(double a0, double a1) { return sqrt(np_dot2(a0, a1, a0, a1)); }

// Projection(point, [x1, x2]) -> distance of the point to its projection (the foot point if
// it lies inside the segment, else the nearer vertex), in the reference's operation order.
__host__ __device__ __forceinline__ double ref_project_dist(double px, double py, double ax, double ay, double bx, double by) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  double dx = bx - ax, dy = by - ay;
  const double n1 = np_norm2(dx, dy);
  dx = dx / n1;                                    // dir1 /= norm(dir1)
  dy = dy / n1;
  const double t = np_dot2(px - ax, py - ay, dx, dy);
  const double sx = dx * t, sy = dy * t;           // x1 + dir1 * dot(x - x1, dir1)
  double qx = ax + sx, qy = ay + sy;
  const double d2x = qx - ax, d2y = qy - ay, d3x = qx - bx, d3y = qy - by;
  const double n2 = np_norm2(d2x, d2y), n3 = np_norm2(d3x, d3y);
  if (n2 > 0 && n3 > 0) {
    const double e2x = d2x / n2, e2y = d2y / n2, e3x = d3x / n3, e3y = d3y / n3;
    const bool on_line = np_norm2(e2x - e3x, e2y - e3y) > 1e-10;
    if (!on_line) {
      if (np_norm2(ax - qx, ay - qy) < np_norm2(bx - qx, by - qy)) {
        qx = ax;
        qy = ay;
      } else {
        qx = bx;
        qy = by;
      }
    }
  }
  return np_norm2(px - qx, py - qy);
}

// np.argmin over dist[0..m) (first minimum; the first NaN if there is one).
__host__ __device__ __forceinline__ int np_argmin(const double* d, int m) {
  int b = 0;
  for (int i = 1; i < m; ++i) {
    if (d[b] != d[b]) break;
    if (d[i] != d[i] || d[i] < d[b]) b = i;
  }
  return b;
}

// Segments project_fast tests from projection index p on a polyline of np points:
// raceline[:, p:p+10] holds min(10, np - p) points.
__host__ __device__ __forceinline__ int ctl_segments(int p, int np_) {
  const int pts = np_ - p < kCtlSegs + 1 ? np_ - p : kCtlSegs + 1;
  return pts - 1;
}

// numpy's pairwise sum (loops_utils.h pairwise_sum, n <= 128) of v[first..first+n) read
// through a ring of `cap` entries (np.mean(np.array(hist)[-S:]) = this / n).
__host__ __device__ __forceinline__ double np_pairwise_ring(const double* v, int first, int n, int cap) {
  auto at = [&](int i) {
    int s = first + i;
    while (s >= cap) s -= cap;
    return v[s];
  };
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += at(i);
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = at(j);
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += at(i + j);
  double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) s += at(i);
  return s;
}

// ---- the sharded controller's exchange (llampc_ctl_set_exchange; BASELINE config 5) --------
// Every rank ticks the controller on its contiguous shard of the global bank.  The look-back's
// completing block pushes ONE record per tick into every peer's mailbox: its shard's sorted
// top-K and its argmin as K + 1 entries (window mean, global model index), four 32-bit payload
// words each (value hi, lo, index hi, lo; index -1: none).  Every rank merges the G records
// the same way (below), so every rank holds the unsharded selection: the argmin (rt.py:359,
// NaN-first under NAN_FIRST) and the top-K (rt.py:360: argsort order, NaN last, ties to the
// lower global index).  Each then rolls out those K + 1 models itself from the replicated
// global parameter table, so the controller state stays identical on every rank and no second
// exchange is needed.  The host restatement (llampc_ctl_merge) runs the same functions.
__host__ __device__ constexpr int ctl_rec_words(int K) { return 4 * (K + 1); }
constexpr int kCtlPxMax = 16;               // largest world of the sharded controller (its LDS)

// argsort order key of a window mean (order_key's: -0 -> +0, every NaN one value above +inf)
__host__ __device__ __forceinline__ uint64_t ctl_okey(double w) {
  const double wc = (w != w) ? __builtin_nan("") : w + 0.0;
  const uint64_t b = __builtin_bit_cast(uint64_t, wc);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// The merge order of a top-K entry e of the G K gathered ones: (key, id) with missing entries
// after every real one, each unique by position (ids of real models are < 2^62).
__host__ __device__ __forceinline__ void ctl_entry_order(double v, int64_t gid, int e, uint64_t& key, uint64_t& id) {
  const bool none = gid < 0;
  key = none ? ~0ull : ctl_okey(v);
  id = none ? (0x7FFFFFFFFFFFFFFFull - 1024 + (uint64_t)e) : (uint64_t)gid;
}
__host__ __device__ __forceinline__ bool ctl_order_lt(uint64_t ka, uint64_t ia, uint64_t kb, uint64_t ib) {
  return (ka < kb) | ((ka == kb) & (ia < ib));
}
// The merged argmin over the G shards' argmins (entry K of each record): np.argmin's order
// (NaN-first: the lowest index holding NaN) or NaN-last; index -1 = none.  Returns the winner's
// shard (or -1).
// shard g's argmin entry comes from get(g, value, index).
template <typename Get>
__host__ __device__ __forceinline__ int ctl_merge_argmin(Get get, int G, bool nan_first, double& bv, int64_t& bi) {
  bv = nan_first ? __builtin_inf() : __builtin_nan("");
  bi = kNoIndex;
  int owner = -1;
  for (int g = 0; g < G; ++g) {
    double v;
    int64_t id;
    get(g, v, id);
    if (id < 0) continue;
    if (key_less(nan_first, v, id, bv, bi)) {
      bv = v;
      bi = id;
      owner = g;
    }
  }
  if (owner < 0) {
    bi = -1;
    bv = __builtin_nan("");
  }
  return owner;
}
// The merged top-K position of entry e among the M = G K gathered ones (order = ctl_entry_order;
// key(j) / id(j) give entry j's): its rank, < K for the entries that make the top-K.
template <typename Key, typename Id>
__host__ __device__ __forceinline__ int ctl_merge_rank(Key key, Id id, int M, int e) {
  const uint64_t k = key(e), i = id(e);
  int r = 0;
  for (int j = 0; j < M; ++j) r += (int)ctl_order_lt(key(j), id(j), k, i);
  return r;
}
// LDS bytes of the exchange (the completing block, from kScratchBytes): the G records as
// 32-bit words, the M entries' keys and ids, the output ranks, the waves' late flags.
__host__ __device__ __forceinline__ size_t ctl_px_bytes(int G, int K) {
  const size_t rec = ((size_t)4 * G * ctl_rec_words(K) + 15) & ~(size_t)15;
  return rec + 16 * (size_t)G * K + 4 * LLAMPC_KMAX + 16;
}

// The controller launch (ctl.hip ctl_kernel): every field set by the host (capi.hip
// llampc_ctl_*) except the look-back's x_now, which the kernel points at x_t.
struct CtlLaunch {
  LookbackLaunch lb;          // x_prev / u_prev -> the state (host), x_now -> x_t (kernel)
  LookaheadLaunch la;         // params, veh, cost, C, H, Ts, rl (U and xref: LDS)
  FinalLaunch fin;            // lb_final's view (out = &out->plan, nb_lb, K, lists)
  CtlState* st;
  llampc_ctl_out* out;        // device alias of the pinned host record
  uint64_t* host_tag;
  uint64_t host_seq;
  uint64_t* sel_tag;          // [kCtlSlotsMax]   selection (lb_final<true>)
  uint64_t* slot_tag;         // [kCtlSlotsMax][4] slot results: cost hi, lo, cand, nf | late << 31
  unsigned* tickets;          // [1] the look-back ticket
  double* dbg;                // null, or this tick's xref [2][H+1] then U [C][H][2]
  double* znoise;             // [2][C H][2]: the candidates' variates of tick t in half t & 1
  uint64_t* ztag;             // [2]: t + 1 once half t & 1 holds tick t's (the completing block
                              //   of tick t - 1 draws them while it polls)
  const double* pts;          // raceline points [2][np] (project_fast's polyline)
  const double* prefix;       // [np - 1] start arc length per projection index
  uint64_t tick, seed;
  double x_t[6];
  double nominal[6];          // Bf, Cf, Df, Br, Cr, Dr (the warm-up model)
  double nscale[2], rate[2];  // sqrt(3) sigma_j; rate_max_j Ts (< 0: none)
  double umin[2], umax[2];
  double mu_fixed, scale_fixed, v_factor, mu_init;
  size_t poll_off;
  uint32_t seq, poll;         // tag of this launch; poll bound (2^16 s_memrealtime units)
  int32_t np, lap_projidx;
  int32_t do_lb, warm, use_mu, full, nslots, mpb, G, cpl, S, K;
  int32_t nb_lb, nb_la;
  int32_t s4;                 // stage each (candidate, step)'s sincos / cost terms (CtlLds.s4)
  int32_t p0_walk;            // the state's projidx and the walk's mu bracket (rt.py:278-282),
  MuBracket br_walk;          //   from the host's copy of the last record: the look-ahead
                              //   prologue's table loads wait on no state or mu-table load
  // sharded (px_G > 0, llampc_ctl_set_exchange): the selection's model indices are global, the
  // look-ahead's params (la.params, la.n) the replicated global table, sel_goff = 0; else
  // sel_goff = the bank's global offset (the selection's indices are local to the bank)
  int64_t sel_goff;
  uint64_t* const* px_box;    // every rank's mailbox as mapped here (device array)
  int32_t px_G, px_rank;
  uint32_t px_seq;            // the mailbox's tick number of this exchange
  uint32_t px_bound;          // the peers' wait bound, units of 2^16 s_memrealtime ticks
  // gather transports (llampc_ctl_set_gather: RCCL or the host carries the records, no peer
  // mailbox): a full-window tick is two launches.  px_phase 1 — the look-back blocks alone; the
  // ticket winner stores this shard's record, ctl_rec_words(K) words tagged px_seq, at px_send
  // and exits.  Between the launches the G records are all-gathered into px_gath [G][nw].
  // px_phase 2 — block 0 (nb_lb = 1) reads them (ctl_exchange: the same merge, the own record
  // from px_send, the peers' from px_gath, every word's tag checked) and completes the tick;
  // the look-ahead blocks as in one launch.  px_phase 0: the peer mailbox (one launch).
  int32_t px_phase;
  uint64_t* px_send;          // [nw] (phase 1 writes, phase 2 reads)
  const uint64_t* px_gath;    // [G][nw]
  // armed ticks with the peer exchange and n_spec > 0: every rank's speculative list goes
  // through the mailbox slot too, at word px_spec_off (after the selection record), before the
  // doorbell; a peer's list that is not there after px_spec_wait s_memrealtime ticks is not
  // waited for (ctl.hip ctl_spec_exchange)
  int32_t px_spec_off;
  uint32_t px_spec_wait;
  // armed launch (door != null, llampc_ctl_set_prelaunch): enqueued behind the previous tick,
  // it runs its x_t-independent prologue and then waits for the host's doorbell: kCtlDoorWords
  // tagged words (tag door_seq) in pinned memory — x_t as 12 32-bit halves, then the status
  // (kCtlDoorFire / kCtlDoorCancel).  Block 0 alone polls the pinned words (many blocks reading
  // host memory queue behind each other on PCIe) and copies them to door_dev in device memory,
  // which the other blocks poll.  Block 0 gives up after door_bound (2^16 s_memrealtime units):
  // it then posts kCtlDoorExpired, stores host_seq | kCtlTagExpired, and every block exits
  // untouched.  projidx and the mu bracket then come from the state.
  // door_dev[kCtlTimeWord] (every launch): the s_memrealtime at which x_t reached the device
  // (armed: block 0 saw the doorbell; launched: block 0 started); the completion stores the
  // 100 MHz ticks from it to its record stores into host_tag[1], before the tag
  // (llampc_ctl_device_us)
  const uint64_t* door;
  uint64_t* door_dev;
  uint32_t door_seq, door_bound;
  // speculative look-ahead (n_spec > 0: an armed tick with a full window): before the doorbell
  // each look-back block ranks its models by their window mean without x_t — the W - 1 entries
  // that stay (win_pre) — and stores its sorted n_spec best at spec_val / spec_idx[blk]; the
  // last of them (ticket 1) merges the lists and publishes the n_spec best as tagged words
  // spec_tag[j] (local index; kNoLocal: none).  Spec block j (after the look-ahead blocks in the
  // grid) rolls model spec_tag[j] out from the doorbell on — the tracking cost deferred until
  // the reference arrives (xref_tag: the first look-ahead block's walk, tagged halves) — and
  // publishes its best candidate at spec_res[4 j] (ctl_lookahead's slot words).  A selected
  // model among them is not rolled out again: the look-ahead blocks skip it and the completion
  // reads spec_res (profiles/r05/spec_topm.json: the selection falls inside the 32 best by this
  // predictor on 86-88 % of the closed loop's ticks, the 64 best on ~90 %; 32 by default, capi.hip).
  int32_t n_spec;
  double* spec_val;           // [nb_lb][n_spec]
  int64_t* spec_idx;
  uint64_t* spec_tag;         // [kCtlSpecMax]
  uint64_t* spec_res;         // [kCtlSpecMax][4]
  uint64_t* xref_tag;         // [2 (H + 1)][2]
};
constexpr int kCtlSpecMax = 64;
constexpr int kCtlDoorWords = 13;
constexpr int kCtlTimeWord = 13;            // door_dev's x_t time (kCtlDoorWords <= it < 16)
constexpr uint32_t kCtlDoorFire = 1, kCtlDoorCancel = 2, kCtlDoorExpired = 3;
constexpr uint64_t kCtlTagExpired = 1ull << 62;

// llampc_ctl_reference's launch: ConstantSpeed alone (planner.py:12-67) on the device.
struct CsLaunch {
  RacelineK rl;
  const double* pts;          // [2][np]
  const double* prefix;       // [np - 1]
  double* out;                // [2][H+1] xref, then projidx, vr
  double x0, y0, v0, mu, scale, Ts;
  int32_t np, p0, H;
};
hipError_t launch_constant_speed(const CsLaunch& a, hipStream_t s);

// LDS bytes of the controller launch and the completing block's area offset (ctl.hip); s4:
// with the staged input terms (CtlLaunch.s4).
size_t ctl_lds_bytes(int H, int C, int n, int nb_lb, int K, size_t* poll_off, bool s4 = false, int px_G = 0,
                     int n_spec = 0);
hipError_t launch_ctl(const CtlLaunch& c, int lpm, size_t lds, hipStream_t s);

}  // namespace llampc
