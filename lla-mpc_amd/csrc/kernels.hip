// kernels.hip — gfx950 (CDNA4) kernels of the LLA-MPC model-bank hot path.
//
//   lookback_kernel    one lane per model: RK4 step from (x_{t-1}, u_{t-1}), 4-state MSE
//                      against x_t, in-place ring write, W-window mean in NumPy's pairwise
//                      order, then per-block argmin + top-K by wave64 shuffles.
//                      Reference: evaluate_models_vectorized.py:4-24, rt.py:347-366.
//   lookahead_kernel   one lane per (model, candidate): H-step rollout (RK4 / NLP-Euler /
//                      RK6) with the MPC objective accumulated in registers; candidates'
//                      controls and xref staged in LDS; group (per-model) argmin over the
//                      candidates by xor-shuffles; per-block argmin.
//                      Reference: model.py:32-40 composed H times + nmpc.py:44-111.
//   select_kernel      one block: merges the per-block partials into llampc_plan_out.
//   merge_kernel       cross-shard merge after the RCCL all-gather (merge.hpp).
//   dynamics_kernel / integrate_kernel   raw batched Dynamic API (dynamic.py:98-154,
//                      model.py:18-40, rk6.py).
//
// This translation unit: the plan-launch dispatcher (launch_plan) and the non-plan kernels.
// The device code of the plan launch is plan_dev.hpp; its instantiations live in plan_*.hip
// (one TU per variant group, so the library builds in parallel), the controller tick in ctl.hip.
#include "plan_dev.hpp"

namespace llampc {

__global__ __launch_bounds__(kBlock) void merge_kernel(const llampc_plan_out* parts, int32_t G,
                                                       int32_t nan_first, llampc_plan_out* m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  // the G gathered records -> LDS in ONE round trip of 16-B loads (every later read is LDS)
  llampc_plan_out* rec = reinterpret_cast<llampc_plan_out*>(smem);
  constexpr int kWords = sizeof(llampc_plan_out) / 16;
  static_assert(sizeof(llampc_plan_out) % 16 == 0, "records staged as 16-B words");
  const uint4* srcw = reinterpret_cast<const uint4*>(parts);
  uint4* dstw = reinterpret_cast<uint4*>(rec);
  for (int e = tid; e < G * kWords; e += kBlock) dstw[e] = srcw[e];
  __syncthreads();
  merge_staged(rec, G, nan_first, m, reinterpret_cast<EntS*>(smem + (size_t)G * sizeof(llampc_plan_out)), 0);
}

// Peer exchange (xGMI, no collective library): every rank's mailbox is uncached device
// memory mapped into every peer process (IPC).  One block per rank per tick:
//  1. push — this rank's record as tagged 64-bit words (tick seq << 32 | 32 payload bits)
//     into slot [seq & 1][rank] of every peer's mailbox, system-scope stores that go straight
//     over xGMI into the peer's HBM (its own copy goes straight to LDS);
//  2. poll — every thread spins on its share of the G slots of its own mailbox until each
//     word carries this tick's seq (every word validates itself: no fence pairing across
//     devices), unpacking the payloads into the LDS records;
//  3. merge_staged — the same merge as merge_kernel.
// Two slots by tick parity: a peer can only push tick t+2 after its own exchange of t+1,
// which needs this rank's push of t+1, issued after this rank's exchange of t has finished
// reading slot (t & 1) — so a slot is never overwritten while it is read.  A poll that
// waits longer than `bound` (s_memrealtime ticks) gives status LLAMPC_STATUS_POLL_TIMEOUT.
__global__ __launch_bounds__(kBlock) void peer_exchange_kernel(PeerLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kW = kRecWords;
  const int tid = threadIdx.x;
  const int G = a.G;
  const size_t slot0 = (size_t)(a.seq & 1) * G * kW;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.local);
  uint32_t* rec32 = reinterpret_cast<uint32_t*>(smem);
  for (int w = tid; w < kW; w += kBlock) {
    const uint32_t x = src[w];
    rec32[a.rank * kW + w] = x;                 // this rank's record: straight to LDS
    const uint64_t v = tag_word(a.seq, x);
    const size_t off = slot0 + (size_t)a.rank * kW + w;
    for (int g = 0; g < G; ++g)
      if (g != a.rank) __hip_atomic_store(a.box[g] + off, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint64_t* own = a.box[a.rank] + slot0;
  constexpr int kPerK = (kPeerMax * kRecWords + kBlock - 1) / kBlock;
  int late = poll_mailbox<kPerK>(own, G, a.rank, a.seq, a.bound, rec32);
  // one flag per wave after the lists (no static LDS: the launch asks for all 160 KB)
  EntS* lists = reinterpret_cast<EntS*>(smem + (size_t)G * sizeof(llampc_plan_out));
  int* wave_late = reinterpret_cast<int*>(lists + 2 * (size_t)G * LLAMPC_KMAX);
  const int wl = __any(late);
  if ((tid & 63) == 0) wave_late[tid >> 6] = wl;
  __syncthreads();
  late = 0;
  for (int w = 0; w < kBlock / 64; ++w) late |= wave_late[w];
  if (late) {                                   // block-uniform
    peer_timeout_record(rec32, a.rank, a.merged);
    return;
  }
  merge_staged(reinterpret_cast<const llampc_plan_out*>(smem), G, a.nan_first, a.merged, lists, 0);
}

// ------------------------------------------------------------------------------------
// Raw batched dynamics (Dynamic API)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void dynamics_kernel(int32_t op, const double* x,
                                                          const double* u, const double* params,
                                                          int64_t P, VehK veh, int64_t n,
                                                          double* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Tire t = load_tire(params, P, P == 1 ? 0 : i);
  double xi[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) xi[j] = x[6 * i + j];
  if (op == LLAMPC_OP_FORCES) {
    const Forces f = forces<Form::Ref>(veh, t, xi[3], xi[4], xi[5], u[2 * i], u[2 * i + 1]);
    out[i] = f.Ffy;
    out[n + i] = f.Frx;
    out[2 * n + i] = f.Fry;
    out[3 * n + i] = f.af;
    out[4 * n + i] = f.ar;
  } else {
    const Input in = make_input(u[2 * i], u[2 * i + 1]);
    double d[6];
    rhs<Form::Ref>(veh, t, xi, in, d);
#pragma unroll
    for (int j = 0; j < 6; ++j) out[6 * i + j] = d[j];
  }
}

// Elementwise transcendentals of the model (accuracy tests of fastmath.hpp).
__global__ __launch_bounds__(kBlock) void math_kernel(int32_t fn, const double* a, const double* b,
                                                      int64_t n, double* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double r = 0.0, s, c;
  const fm::FmK K = fm::FmK::load();
  switch (fn) {
    case 0: r = LL_ATAN2P(a[i], b[i]); break;
    case 1: r = LL_ATAN(a[i]); break;
    case 2: LL_SINCOS(a[i], &s, &c); r = s; break;
    case 3: LL_SINCOS(a[i], &s, &c); r = c; break;
    case 4: r = fm::atan2_fast(a[i], b[i], K); break;
    case 5: r = fm::atan_fast(a[i], K); break;
    case 6: r = fm::sin_wide(a[i], K); break;
    case 7: fm::sincos_fast(a[i], &s, &c, K); r = s; break;
    case 8: fm::sincos_fast(a[i], &s, &c, K); r = c; break;
    case 9: r = fm::div6(a[i], K); break;
    case 10: r = fm::atan2_fast<true>(a[i], b[i], fm::FmK::load<true>()); break;
    case 11: r = fm::atan_fast<true>(a[i], fm::FmK::load<true>()); break;
    case 12: r = fm::sin_wide<true>(a[i], fm::FmK::load<true>()); break;
    case 13:   // paired atan2 (dyn.hpp chain_pair): partner element n-1-i, the same x
    case 14: { // paired atan: partner element n-1-i
      const int64_t j = n - 1 - i;
      double af, ar, hf, hr, dp;
      if (fn == 13) fm::atan2_fast_pair(a[i], a[j], b[i], fm::FmK::load<true>(), af, ar, hf, hr, dp);
      else fm::atan_fast_pair(a[i], a[j], fm::FmK::load<true>(), af, ar, dp);
      r = af;
      break;
    }
    default: r = __builtin_nan("");
  }
  out[i] = r;
}

template <int INTEG>
__global__ __launch_bounds__(kBlock) void integrate_kernel(const double* x0, const double* u,
                                                           int64_t us, const double* h, int32_t S,
                                                           const double* params, int64_t P,
                                                           VehK veh, int64_t n, double* traj,
                                                           int32_t final_only) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Tire t = load_tire(params, P, P == 1 ? 0 : i);
  double x[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) x[j] = x0[6 * i + j];
  if (!final_only) {
#pragma unroll
    for (int j = 0; j < 6; ++j) traj[6 * i + j] = x[j];
  }
  for (int s = 0; s < S; ++s) {
    const Input in = make_input(u[i * us + 2 * s], u[i * us + 2 * s + 1]);
    step<INTEG>(veh, t, x, in, h[s]);
    if (!final_only) {
#pragma unroll
      for (int j = 0; j < 6; ++j) traj[((int64_t)(s + 1) * n + i) * 6 + j] = x[j];
    }
  }
  if (final_only) {
#pragma unroll
    for (int j = 0; j < 6; ++j) traj[6 * i + j] = x[j];
  }
}

// ------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------
int lookback_blocks(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

// Lanes (candidate slots) per model: the power of two >= C, at most one block (256); a
// model's candidates beyond G run sequentially in its lanes (cpl = ceil(C / G)).
int lookahead_group(int32_t C) {
  int G = 1;
  while (G < C && G < kBlock) G <<= 1;
  return G;
}

// Lanes per rollout while the launch has fewer waves than the chip has SIMDs (latency-
// bound: a wave's time is its instruction stream): a quad (LPM = 4: front chain, rear
// chain, sin psi, cos psi in one stream) up to 16k rollouts, a lane pair (front / rear
// chain) up to 32k; one lane per rollout once the chip fills (fewest instructions per
// rollout).
// share: the number of banks the caller ticks concurrently on the device (llampc_bank_set_
// concurrency): each launch is sized for 1/share of the SIMDs (BASELINE config 5, two tracks
// at N = 10^4, H = 40: LPM 2 instead of 4, so both launches are resident together — 111 ->
// 86 us per paced step, profiles/r04/config5_lpm.log).
int lookahead_lpm(int64_t n, int32_t C, int32_t integrator, int32_t share) {
  if (integrator == LLAMPC_RK6) return 1;
  const int G = lookahead_group(C);
  if (const char* e = getenv("LLAMPC_LPM")) {     // benchmarking override
    const int v = atoi(e);
    if (v == 1 || ((v == 2 || v == 4) && v * G <= kBlock)) return v;
  }
  const int64_t lanes = n * G * std::max(share, 1);
  if (lanes <= 16384 && 4 * G <= kBlock) return 4;
  return (lanes <= 32768 && 2 * G <= kBlock) ? 2 : 1;
}

int lookahead_blocks(int64_t n, int32_t C, int lpm) {
  const int mpb = kBlock / (lookahead_group(C) * lpm);
  return (int)((n + mpb - 1) / mpb);
}

// Staged inputs per (step, candidate): RK4 the fused stages' input terms and delta, else pwm,
// delta, sin delta, cos delta; then the input-rate cost term and the feasibility (1/0) —
// kStageW doubles.  One block per CU (the launch's LDS
// request), so the staging may use most of the CU's 160 KiB.
constexpr size_t kStageLimit = 128 * 1024;

// knots [n] + the +inf pad [kKnotPad] + xy [8(n-1)] + mus [M] (padded to 16 B) (the speed
// window on top: launch_plan)
size_t raceline_lds_bytes(int32_t n, int32_t M) {
  return 8 * (size_t)(n + kKnotPad) + 64 * (size_t)(n - 1) + 8 * (size_t)((M + 1) & ~1);
}

size_t lookahead_lds_bytes(int32_t C, int32_t H, bool* stage_u) {
  const size_t base = kScratchBytes + 16 * (size_t)(H + 1);
  const size_t ub = 8 * kStageW * (size_t)C * H;
  *stage_u = base + ub <= kStageLimit;
  return *stage_u ? base + ub : base;
}

// Models per look-back lane: keep the block lists small enough for the in-LDS tree merge
// (nb_lb * K <= 640 entries = 20 KB for both buffers).
// Models per lane: lb_final holds blocks * kWaves * K entries in LDS and merges at most
// 64 * kListsPerLane lists; R grows once blocks * K would pass 640 (40 KB of LDS) or the
// blocks 64 * kListsPerLane / kWaves.
int lookback_r(int64_t n, int32_t K) {
  const int64_t blocks = std::min<int64_t>(640 / std::max(1, K), 64 * kListsPerLane / kWaves);
  const int64_t per = (int64_t)kBlock * std::max<int64_t>(1, blocks);   // models per R step
  return (int)std::max<int64_t>(1, (n + per - 1) / per);
}

int lookback_blocks_r(int64_t n, int R) { return (int)((n + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R)); }

// Every plan launch requests more than half of the CU's 160 KiB of LDS, so each block has
// its CU — and each wave its SIMD — to itself.  (Letting LPM-1 launches pack two blocks per
// CU measured no gain at C = 64: 567-574 vs 568-569 us.)  Every cross-block hand-off is an
// agent-scope atomic (sc1: L1-bypassing, st_wt / ld_wt).

bool plan_inline_ok(int32_t C, int32_t H, int32_t integrator, int32_t xref_mode) {
  if (integrator != LLAMPC_RK4 || xref_mode != LLAMPC_XREF_GIVEN || C < 1 || H < 1) return false;
  if (16 + 2 * ((int64_t)H + 1) + 2 * (int64_t)C * H > kInlineDoubles) return false;
  bool stage = false;
  (void)lookahead_lds_bytes(C, H, &stage);
  return stage;
}


// Compute units of the current device (cached): the work-queue layout launches one
// look-ahead block per CU, minus the one the completing look-back block holds.
static int device_cus() {
  static int cus[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
  if (!cus[d]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || c < 2) c = 256;
    cus[d] = c;
  }
  return cus[d];
}

hipError_t launch_plan(const LookbackLaunch* lb, const LookaheadLaunch* la, FinalLaunch f,
                       hipStream_t s, const InlinePack* pk, int32_t share) {
  LookbackLaunch lbv{};
  LookaheadLaunch lav{};
  int G = 1, cpl = 1, lpm = 1, integ = LLAMPC_RK4;
  bool stage = false;
  size_t lds = kScratchBytes;
  f.nb_lb = 0;
  f.nb_la = 0;
  if (lb) {
    lbv = *lb;
    lbv.R = lookback_r(lb->n, std::max(1, lb->K));
    // A/B knob: at least LLAMPC_LB_R models per look-back lane (fewer look-back blocks)
    static const int r_min = getenv("LLAMPC_LB_R") ? std::max(1, atoi(getenv("LLAMPC_LB_R"))) : 1;
    lbv.R = std::max(lbv.R, r_min);
    f.nb_lb = lookback_blocks_r(lb->n, lbv.R);
    if (lb->full) {
      const size_t M = (size_t)f.nb_lb * lb->K, L = f.nb_lb;   // lb_final (layout there)
      lds = std::max(lds, kScratchBytes + 8 * (3 * M + L) + sizeof(Ent) * L * kWaves +
                              4 * (3 * M + L + LLAMPC_KMAX + 2) + 8 + 16);
      lds = std::max(lds, kScratchBytes + (size_t)kWaves * kRankBytes + kBlockMergeBytes);  // wave lists
    }
  }
  if (la) {
    lav = *la;
    G = lookahead_group(la->C);
    cpl = (la->C + G - 1) / G;
    integ = la->integrator;
    lpm = lookahead_lpm(la->n, la->C, integ, share);
    f.nb_la = lookahead_blocks(la->n, la->C, lpm);
    if (la->xref_mode == LLAMPC_XREF_RACELINE) {
      // knots + x/y rows in LDS, the staged inputs when they fit beside them, and the rest
      // of the CU's LDS (up to the whole track) for the speed-profile window
      constexpr size_t kLdsMax = 160 * 1024 - 1024;
      const size_t rl = raceline_lds_bytes(la->rl.n, la->rl.M);
      size_t base = lookahead_lds_bytes(la->C, la->H, &stage);
      if (base + rl > kLdsMax) {
        stage = false;
        base = kScratchBytes + 16 * (size_t)(la->H + 1);
      }
      const size_t per_seg = 32 * (size_t)std::max(1, la->rl.M);
      const size_t room = base + rl < kLdsMax ? kLdsMax - base - rl : 0;
      lav.rl.wcap = (int32_t)std::min<size_t>(room / per_seg, (size_t)(la->rl.n - 1));
      lds = std::max(lds, base + rl + per_seg * (size_t)lav.rl.wcap);
    } else {
      lds = std::max(lds, lookahead_lds_bytes(la->C, la->H, &stage));
    }
  }
  f.do_lb = lb != nullptr;
  f.do_la = la != nullptr;
  if (f.nb_lb + f.nb_la == 0) return hipErrorInvalidValue;
  // Work queue (the throughput regime): LPM 1 with a model inside one wave (G <= 64), RK4 on
  // the shared xref, device inputs, at least 1.75 rounds of look-ahead blocks per CU — then one
  // block per CU (minus the completing look-back block's) takes units of models from the
  // bank's counter: 8 waves per block (two rollout waves per SIMD) from 4 units per wave
  // slot of the 4-wave layout on, else 4 waves.  C = 64 N-sweep on one box (static / 4-wave /
  // 8-wave, us per tick; profiles/r03/v31/c64_sweep.txt): N = 1500: 92.0 / 99.5 / 106.9;
  // 2000: 128.1 / 106.5 / 155.8; 3000: 163.9 / 137.7 / 164.4; 5000: 239.4 / 206.3 / 209.5;
  // 10^4: 468.7 / 391.2 / 372.6; 2 10^4: 899.7 / 732.2 / 681.4 — the 8-wave layout's second
  // wave of a SIMD only fills the first one's bubbles, so with few units per wave the launch
  // waits for those slow units.  LLAMPC_NO_WQ=1 keeps the block-per-models layout,
  // LLAMPC_WQ_WAVES=4|8 forces a work-queue block size (A/B runs).
  int wq = 0;
  if (la && la->wq && lpm == 1 && G <= 64 && integ == LLAMPC_RK4 && la->xref_mode == LLAMPC_XREF_GIVEN &&
      !pk && getenv("LLAMPC_NO_WQ") == nullptr) {
    const int nw = std::max(1, device_cus() - 1);
    const char* force = getenv("LLAMPC_WQ_WAVES");
    const int forced = force ? atoi(force) : 0;
    if ((int64_t)f.nb_la * 4 >= (int64_t)nw * 7 || (forced && f.nb_la > nw)) {
      const int64_t mpw = 64 / G;
      const int64_t units = (la->n + mpw - 1) / mpw;
      f.nb_la = nw;
      wq = (stage && (forced ? forced == 8 : units >= 4 * (int64_t)nw * kWaves)) ? 2 : 1;
    }
  }
  if (f.px_G) {                          // fused peer exchange: RK4, given xref, device inputs
    if (pk || integ != LLAMPC_RK4 || (la && la->xref_mode == LLAMPC_XREF_RACELINE) || f.px_G > kPeerFuseMax)
      return hipErrorInvalidValue;
    lds = std::max(lds, 256 + (size_t)f.px_G * (sizeof(llampc_plan_out) + 2 * LLAMPC_KMAX * sizeof(EntS)) +
                            kWaves * sizeof(int));
  }

  if (pk) {
    if (!la || !plan_inline_ok(la->C, la->H, integ, la->xref_mode) || !stage) return hipErrorInvalidValue;
    if (lpm == 4) launch_plan_inline_group<4>(lbv, lav, f, G, cpl, lds, s, *pk);
    else if (lpm == 2) launch_plan_inline_group<2>(lbv, lav, f, G, cpl, lds, s, *pk);
    else launch_plan_inline_group<1>(lbv, lav, f, G, cpl, lds, s, *pk);
    return hipGetLastError();
  }
  switch (integ) {
    case LLAMPC_RK4:
    case LLAMPC_EULER_NLP: {
      const bool rk4 = integ == LLAMPC_RK4;
      const int w = rk4 ? wq : 0;
      if (lpm == 4) (rk4 ? launch_plan_group<0, 4> : launch_plan_group<1, 4>)(lbv, lav, f, G, cpl, stage, lds, s, w);
      else if (lpm == 2) (rk4 ? launch_plan_group<0, 2> : launch_plan_group<1, 2>)(lbv, lav, f, G, cpl, stage, lds, s, w);
      else (rk4 ? launch_plan_group<0, 1> : launch_plan_group<1, 1>)(lbv, lav, f, G, cpl, stage, lds, s, w);
      break;
    }
    case LLAMPC_RK6:
      launch_plan_group<2, 1>(lbv, lav, f, G, cpl, stage, lds, s, 0);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}


hipError_t launch_merge(const llampc_plan_out* parts, int32_t G, int32_t nan_first,
                        llampc_plan_out* merged, hipStream_t s) {
  if (G < 1 || G > 32) return hipErrorInvalidValue;   // LDS: 95 KB at G = 32
  const size_t M = (size_t)G * LLAMPC_KMAX;      // K <= KMAX (read on device)
  const size_t lds = (size_t)G * sizeof(llampc_plan_out) + 2 * M * sizeof(EntS);
  allow_lds(merge_kernel);
  hipLaunchKernelGGL(merge_kernel, dim3(1), dim3(kBlock), lds, s, parts, G, nan_first, merged);
  return hipGetLastError();
}

hipError_t launch_peer_exchange(const PeerLaunch& a, hipStream_t s) {
  if (a.G < 1 || a.G > kPeerMax || a.rank < 0 || a.rank >= a.G || a.seq == 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)a.G * sizeof(llampc_plan_out) + 2 * (size_t)a.G * LLAMPC_KMAX * sizeof(EntS) +
                     (kBlock / 64) * sizeof(int);
  allow_lds(peer_exchange_kernel);
  hipLaunchKernelGGL(peer_exchange_kernel, dim3(1), dim3(kBlock), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_dynamics(int32_t op, const double* x, const double* u, const double* params,
                           int64_t P, VehK veh, int64_t n, double* out, hipStream_t s) {
  const int nb = (int)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(dynamics_kernel, dim3(nb), dim3(kBlock), 0, s, op, x, u, params, P, veh, n, out);
  return hipGetLastError();
}

hipError_t launch_math(int32_t fn, const double* a, const double* b, int64_t n, double* out,
                       hipStream_t s) {
  const int nb = (int)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(math_kernel, dim3(nb), dim3(kBlock), 0, s, fn, a, b, n, out);
  return hipGetLastError();
}

hipError_t launch_integrate(const double* x0, const double* u, int64_t us, const double* h,
                            int32_t S, const double* params, int64_t P, VehK veh, int64_t n,
                            int32_t integrator, double* traj, int32_t final_only, hipStream_t s) {
  const int nb = (int)((n + kBlock - 1) / kBlock);
  switch (integrator) {
    case LLAMPC_RK4:
      hipLaunchKernelGGL(integrate_kernel<0>, dim3(nb), dim3(kBlock), 0, s, x0, u, us, h, S, params, P, veh, n, traj, final_only);
      break;
    case LLAMPC_EULER_NLP:
      hipLaunchKernelGGL(integrate_kernel<1>, dim3(nb), dim3(kBlock), 0, s, x0, u, us, h, S, params, P, veh, n, traj, final_only);
      break;
    case LLAMPC_RK6:
      hipLaunchKernelGGL(integrate_kernel<2>, dim3(nb), dim3(kBlock), 0, s, x0, u, us, h, S, params, P, veh, n, traj, final_only);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace llampc
