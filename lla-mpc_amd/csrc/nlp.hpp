// nlp.hpp — the setupNLP.solve drop-in's launch interface (nlp.hip; llampc_nlp_* in capi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ctl.hpp"
#include "kernels.hpp"
#include "llampc.h"

namespace llampc {

// The solver's device state (one per solver handle): the sampling distribution of the
// current iteration and the best sequence so far.
struct NlpState {
  double mean[LLAMPC_HMAX][2];
  double std_[LLAMPC_HMAX][2];
  double best_u[LLAMPC_HMAX][2];
  double best_j;                 // +inf until a finite objective is seen
  int32_t best_it;
  int32_t best_s;                // the best sequence's sample index (in round best_it)
};

// A launch of CEM rounds [it, it + rounds): samples / 64 sample blocks, each of which also
// completes every round (nlp.hip).  Every round of the solve in one launch when the blocks are
// few enough to be co-resident (nlp_persistent), else one launch per round.  Blocks exchange a
// round by tagged words (tag nlp_seq(host_seq, round), so no drain, flag or ticket sits between
// a store and its reader): each block's sorted list (list_tag) to every block; across launches
// the next round's mean / std (ms_tag, block 0).  Scalars only (no arrays): the kernel never
// takes the address of its argument (which would copy it to scratch).
// The solve's result as the last round's completion writes it into pinned host memory (then
// a system-scope fence and the host tag): no D2H copy, no stream synchronisation.
struct NlpResult {
  double best_u[LLAMPC_HMAX][2];
  double traj[LLAMPC_HMAX + 1][6];     // xmpc: the NLP's Euler trajectory of best_u
  double best_j;
  int32_t best_it, pad;
};

struct NlpLaunch {
  LookaheadLaunch la;            // params [6][1], veh (NLP form), cost, H, Ts, integrator EULER_NLP
  NlpState* st;
  double* cand;                  // [2][samples][H][2] the round's sequences after the rate clip
                                 //   (by round parity: nlp.hip nlp_cand)
  NlpResult* res;                // the last round: the result, in pinned host memory (device alias)
  uint64_t* host_tag;            //   then this solve's number (host alias spun on by the caller)
  uint64_t host_seq;
  uint64_t* list_tag;            // [2][3][samples]: by round parity, each sample block's sorted
                                 //   list (samples / 64 x len entries) as tagged words: key high
                                 //   halves, key low halves, sample indices
  uint64_t* ms_tag;              // [2][4 H]: the mean [H][2] then std [H][2] of a launch's first
                                 //   round r >= 1, each double as tagged halves (low, high)
  uint64_t seed, call;           // Philox key; counter word 1 = the solve call number
  double up0, up1;               // uprev (du_0, nmpc.py:65-66)
  double umin0, umin1, umax0, umax1;
  double rlo0, rlo1, rhi0, rhi1; // per-step rate bounds (x Ts); lo > hi: none
  double std_floor;
  double sig0, sig1;             // the first round's std (llampc_nlp_cfg.sigma0)
  int32_t it, rounds, iters;     // the launch's first round, its round count, the solve's
  int32_t H, samples, elite, has_hold;
  int32_t ltraj;                 // the last round's sample rollouts keep their states in LDS and
                                 //   a best from that round is copied from there (else re-run)
};

// The solve's inputs in the kernarg segment (the plan kernel's InlinePack idea): x0 [6] | xref
// [2][H+1] | the first round's mean [H][2] — the launch carries them, so a solve needs no H2D
// copy (it cost ~8 us of a 212 us solve).  The state (best so far, NlpState) starts in registers.
constexpr int kNlpInlineDoubles = 6 + 2 * (LLAMPC_HMAX + 1) + 2 * LLAMPC_HMAX;
struct NlpInline {
  double v[kNlpInlineDoubles];
};

// every round in one launch: the sample blocks (one per CU: the LDS request) must all be
// resident at once, since each waits for the others' rounds
constexpr int kNlpPersistentBlocks = 64;
// the round tags' sequence: the solve's number x kNlpMaxIters + the round (llampc_nlp_create
// bounds iters by it), 32 bits — never a stale word's
constexpr int kNlpMaxIters = 1024;
__host__ __device__ __forceinline__ uint32_t nlp_seq(uint64_t host_seq, int it) {
  return (uint32_t)host_seq * (uint32_t)kNlpMaxIters + (uint32_t)it;
}
__host__ __device__ __forceinline__ bool nlp_persistent(int samples) { return samples / 64 <= kNlpPersistentBlocks; }

// the length of each sample block's sorted list: next power of two >= elite (elite <= 64)
__host__ __device__ __forceinline__ int nlp_list_len(int elite) {
  int l = 1;
  while (l < elite) l <<= 1;
  return l;
}
size_t nlp_lds_bytes(int H, int samples, int elite, bool ltraj = false);
bool nlp_ltraj_fits(int H, int samples, int elite);
hipError_t launch_nlp(const NlpLaunch& a, const NlpInline& pk, hipStream_t s);

}  // namespace llampc
