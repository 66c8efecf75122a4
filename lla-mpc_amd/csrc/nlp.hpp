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
  int32_t pad;
};

// A launch of CEM rounds [it, it + rounds): every round of the solve in one launch when the
// sample blocks are few enough to be co-resident (nlp_persistent), the blocks then waiting for
// each round's completion on a tagged word (round_tag); else one launch per round.  Scalars
// only (no arrays): the kernel never takes the address of its argument (which would copy it to
// scratch).
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
  const double* x0;              // [6] device
  const double* xref;            // [2][H+1] device
  uint64_t* top_key;             // [samples / 64][len] each sample block's best (sorted keys),
  uint32_t* top_idx;             //   then their sample indices (len = nlp_list_len(elite))
  double* cand;                  // [samples][H][2] the round's sequences after the rate clip
  NlpResult* res;                // the last round: the result, in pinned host memory (device alias)
  uint64_t* host_tag;            //   then this solve's number (host alias spun on by the caller)
  uint64_t host_seq;
  unsigned* ticket;
  uint64_t* round_tag;           // (host_seq, r): round r's state is published (r >= 1)
  uint64_t seed, call;           // Philox key; counter word 1 = the solve call number
  double up0, up1;               // uprev (du_0, nmpc.py:65-66)
  double umin0, umin1, umax0, umax1;
  double rlo0, rlo1, rhi0, rhi1; // per-step rate bounds (x Ts); lo > hi: none
  double std_floor;
  int32_t it, rounds, iters;     // the launch's first round, its round count, the solve's
  int32_t H, samples, elite, has_hold;
};

// every round in one launch: the sample blocks (one per CU: the LDS request) must all be
// resident at once, since each waits for the others' rounds
constexpr int kNlpPersistentBlocks = 64;
__host__ __device__ __forceinline__ bool nlp_persistent(int samples) { return samples / 64 <= kNlpPersistentBlocks; }

// the length of each sample block's sorted list: next power of two >= elite (elite <= 64)
__host__ __device__ __forceinline__ int nlp_list_len(int elite) {
  int l = 1;
  while (l < elite) l <<= 1;
  return l;
}
size_t nlp_lds_bytes(int H, int samples, int elite);
hipError_t launch_nlp(const NlpLaunch& a, hipStream_t s);

}  // namespace llampc
