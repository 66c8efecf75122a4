// kernels.hpp — internal launch interface between the C ABI (capi.hip) and the HIP
// kernels (kernels.hip).  Every pointer here is a device pointer; launches are async.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dyn.hpp"
#include "raceline.hpp"
#include "llampc.h"

namespace llampc {

constexpr int kBlock = 256;            // 4 waves of 64 lanes
// The work-queue layout's look-ahead blocks (throughput regime): 8 waves, one block per CU,
// so each SIMD interleaves two rollout waves (a lone fp64 wave issues ~4.7 cycles per
// instruction against the VALU's 4).  The other roles of that launch use 256 threads (the
// rest of their waves exit at once).
constexpr int kBlockWQ = 512;
// Work-queue layouts (plan kernel template argument WQ): 0 = none (block per models), 1 = one
// 4-wave block per CU, 2 = one 8-wave block per CU (two rollout waves per SIMD; staged launches
// only — the unstaged rollout would spill at 256 VGPRs).  launch_plan picks by the size of the
// queue (C = 64 N-sweep, profiles/r03/v31/c64_sweep.txt).
constexpr int wq_threads(int wq) { return wq == 2 ? kBlockWQ : kBlock; }

// Cost constants pre-scaled for the kernel (rate bounds multiplied by Ts).
struct CostK {
  double Q[4], R[4], P[4];
  double umin[2], umax[2];
  double dmax[2];                      // rate_max * Ts, < 0 = unbounded
  int32_t enforce;
  int32_t pad;
};

struct LookbackLaunch {
  const double* params;  int64_t n;  int64_t goff;  // params [6][n]
  VehK veh;
  const double* x_prev; const double* u_prev; const double* x_now;
  double Ts;
  double* ring;          // [W][n]
  int32_t W, slot, full, K, nan_first;
  int32_t R;             // models per lane (set by launch_plan)
  int32_t wm_keep;       // the caller reads wm_buf (else it is written only when R > 1)
  double* err_out;       // [n] or null
  double* wm_buf;        // [n] window means (when the window is full: R > 1 or wm_keep)
  double* am_val;  int64_t* am_idx;   // [blocks * kWaves] (one per look-back wave)
  double* tk_val;  int64_t* tk_idx;   // [blocks * kWaves][K]
};


struct LookaheadLaunch {
  const double* params;  int64_t n;  int64_t goff;
  VehK veh;
  const double* x0; const double* U; const double* xref; const double* uprev;
  int32_t C, H, integrator;
  double Ts;
  CostK cost;
  double* cost_out;                      // [n][C] or null
  int32_t* best_cand;  double* best_cost; // [n]
  double* pv;  int64_t* pidx;  int32_t* pnf;  // [blocks]
  int32_t xref_mode;                     // LLAMPC_XREF_*; RACELINE: xref = {s0, v0, scale}
  RacelineK rl;
  double* xref_pm;                       // RACELINE: per-model reference [n][H][2]
  // polled completion (FinalLaunch::poll): tagged records, each 64-bit word = seq << 32 |
  // 32 payload bits, so a reader validates every word it loads on its own
  uint64_t* la_tag;                      // [3][n]: best cost hi, lo, best candidate (SoA)
  uint64_t* blk_tag;                     // [blocks][5]: partial value hi, lo, key hi, lo, nf
  uint32_t seq;                          // this launch's tag (never 0)
  int32_t poll;
  // work queue (launch_plan decides: LPM 1, G <= 64, more look-ahead blocks than CUs): the
  // bank's unit counter, 0 at every launch's start (the block completing the record resets it
  // after every take of the launch, final_write)
  uint64_t* wq;
};

// What the ticket winners of the plan launch need (see plan_kernel).
struct FinalLaunch {
  llampc_plan_out* out;
  unsigned* tickets;                      // [2], zero between launches
  int32_t do_lb, do_la, full, window_count, K, nan_first, nb_lb, nb_la, C;
  int64_t current_model, n, goff;
  const double* params;
  const int32_t* best_cand; const double* best_cost;
  const double* am_val; const int64_t* am_idx; const double* tk_val; const int64_t* tk_idx;
  const double* pv; const int64_t* pidx; const int32_t* pnf;
  // poll = 1: look-ahead blocks publish tagged records and exit; the look-back ticket winner
  // (after lb_final) polls them and completes the record — no look-ahead ticket, no
  // last-block scan.  Deadlock-free: only that one block per launch waits, and only for
  // blocks that never wait.  Needs look-back blocks (do_lb) to host the poller.
  const uint64_t* la_tag; const uint64_t* blk_tag;
  uint32_t seq;
  // 0: no polling; else the poller's wait bound in units of 2^16 s_memrealtime ticks (100 MHz:
  // 655 us per unit) — one 32-bit field, as a separate 64-bit bound cost the raceline
  // variants SGPRs they spilled
  int32_t poll;
  // host completion (llampc_plan / llampc_plan_wait): `out` is then the device alias of a
  // pinned host record, and the block that completes it stores host_seq to host_tag (pinned,
  // system scope) after a system-scope fence — the host spins on that word instead of a D2H
  // copy + stream synchronisation.  Null for device-resident ticks.
  uint64_t* host_tag;
  uint64_t host_seq;
  // fused peer exchange (llampc_plan_exchange; px_G = 0: none): after the record is complete,
  // the block that completed it pushes it into every rank's mailbox (px_box: device array of
  // the px_G mailboxes as mapped here), polls this rank's, and merges into px_merged — the
  // sharded tick in one launch per rank (peer_exchange_kernel's protocol)
  uint64_t* const* px_box;
  llampc_plan_out* px_merged;
  int32_t px_G, px_rank;
  uint32_t px_seq;
  uint32_t px_bound;                      // poll bound, units of 2^16 s_memrealtime ticks
  // the work-queue unit counter (LookaheadLaunch::wq): reset to 0 by final_write, which runs
  // after every look-ahead block has published (so after every take of the launch)
  uint64_t* wq;
};

// Tick inputs in the kernarg segment (host-pointer ticks whose pack fits): x_prev[6],
// u_prev[2], x_now[6], uprev[2], xref[2][H+1], U[C][H][2] — the layout of the H2D pack.  The
// runtime copies kernargs as part of the launch, so such a tick needs no H2D copy.
constexpr int kInlineDoubles = 352;
struct InlinePack {
  double v[kInlineDoubles];
};

int lookback_blocks(int64_t n);
int lookahead_group(int32_t C);
int lookahead_lpm(int64_t n, int32_t C, int32_t integrator, int32_t share = 1);
int lookahead_blocks(int64_t n, int32_t C, int lpm);
int lookback_r(int64_t n, int32_t K);               // models per look-back lane
int lookback_blocks_r(int64_t n, int R);
size_t lookahead_lds_bytes(int32_t C, int32_t H, bool* stage_u);
size_t raceline_lds_bytes(int32_t n, int32_t M);

// The whole tick in ONE launch: look-back blocks (if lb), look-ahead blocks (if la), and
// the completion stages run by ticket winners; writes f.out.  f.nb_* / f.do_* are set here.
// pk != null: the inputs are in *pk (see InlinePack); needs a look-ahead with RK4, the
// given xref and U staged in LDS (plan_inline_ok), else hipErrorInvalidValue.
hipError_t launch_plan(const LookbackLaunch* lb, const LookaheadLaunch* la, FinalLaunch f,
                       hipStream_t s, const InlinePack* pk = nullptr, int32_t share = 1);
bool plan_inline_ok(int32_t C, int32_t H, int32_t integrator, int32_t xref_mode);
// The plan-kernel variant groups (plan_dev.hpp; one translation unit per group, plan_*.hip):
// (integrator, lanes per rollout) with the staged / unstaged inputs and, for RK4 at LPM 1, the
// work-queue layouts; the inline-pack host ticks per LPM.
template <int INTEG, int LPM>
void launch_plan_group(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f, int G,
                       int cpl, bool stage, size_t lds, hipStream_t s, int wq);
template <int LPM>
void launch_plan_inline_group(const LookbackLaunch& lb, const LookaheadLaunch& la, const FinalLaunch& f,
                              int G, int cpl, size_t lds, hipStream_t s, const InlinePack& pk);
#define LLAMPC_PLAN_GROUP_DECL(I, L)                                                               \
  extern template void launch_plan_group<I, L>(const LookbackLaunch&, const LookaheadLaunch&,      \
                                               const FinalLaunch&, int, int, bool, size_t,          \
                                               hipStream_t, int)
LLAMPC_PLAN_GROUP_DECL(0, 4);
LLAMPC_PLAN_GROUP_DECL(0, 2);
LLAMPC_PLAN_GROUP_DECL(0, 1);
LLAMPC_PLAN_GROUP_DECL(1, 4);
LLAMPC_PLAN_GROUP_DECL(1, 2);
LLAMPC_PLAN_GROUP_DECL(1, 1);
LLAMPC_PLAN_GROUP_DECL(2, 1);
extern template void launch_plan_inline_group<4>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                                 int, int, size_t, hipStream_t, const InlinePack&);
extern template void launch_plan_inline_group<2>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                                 int, int, size_t, hipStream_t, const InlinePack&);
extern template void launch_plan_inline_group<1>(const LookbackLaunch&, const LookaheadLaunch&, const FinalLaunch&,
                                                 int, int, size_t, hipStream_t, const InlinePack&);
hipError_t launch_merge(const llampc_plan_out* parts, int32_t G, int32_t nan_first,
                        llampc_plan_out* merged, hipStream_t s);
// Peer exchange of the sharded tick (peer_exchange_kernel): mailbox g is [2][G][kRecWords]
// tagged 64-bit words in rank g's device memory, mapped into this process.
constexpr int kPeerMax = 32;
constexpr int kRecWords = (int)(sizeof(llampc_plan_out) / 4);
struct PeerLaunch {
  const llampc_plan_out* local;          // this rank's record (written by its plan launch)
  uint64_t* box[kPeerMax];               // every rank's mailbox as mapped here (box[rank]: own)
  llampc_plan_out* merged;
  uint64_t bound;                        // poll bound, s_memrealtime ticks (100 MHz)
  int32_t G, rank, nan_first;
  uint32_t seq;                          // tick number, never 0 (the mailbox starts zeroed)
};
hipError_t launch_peer_exchange(const PeerLaunch& a, hipStream_t s);
// Largest world the plan launch can merge in its own LDS (records + lists, see launch_plan).
constexpr int kPeerFuseMax = 16;
hipError_t launch_dynamics(int32_t op, const double* x, const double* u, const double* params,
                           int64_t P, VehK veh, int64_t n, double* out, hipStream_t s);
hipError_t launch_math(int32_t fn, const double* a, const double* b, int64_t n, double* out,
                       hipStream_t s);
hipError_t launch_integrate(const double* x0, const double* u, int64_t u_stride_lane,
                            const double* h, int32_t S, const double* params, int64_t P,
                            VehK veh, int64_t n, int32_t integrator, double* traj,
                            int32_t final_only, hipStream_t s);

}  // namespace llampc
