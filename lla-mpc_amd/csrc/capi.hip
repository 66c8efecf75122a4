// capi.hip — extern "C" boundary (include/llampc.h): the device-resident model-bank
// handle, host<->device staging and the per-tick launch sequence.
//
// A bank owns, on its device: params SoA [6][n] (48 B/model, read coalesced by lane),
// the look-back ring [W][n] (slot-major, so each tick writes one contiguous row — the
// reference's np.roll copy of N*W doubles per tick, rt.py:352, is gone), per-block
// reduction partials, the per-model look-ahead result, and pinned host staging so one
// host-pointer tick = 1 H2D copy + 1 kernel on one stream, the record coming back through
// pinned host memory with a completion tag (llampc_plan / llampc_plan_wait).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ctl.hpp"
#include "kernels.hpp"
#include "nlp.hpp"
#include "merge.hpp"

using namespace llampc;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(LLAMPC_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                  __FILE__, __LINE__);                                                    \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

VehK make_veh(const llampc_vehicle& v) {
  VehK k;
  k.lf = v.lf;
  k.lr = v.lr;
  k.mass = v.mass;
  k.inv_mass = 1 / v.mass;  // the reference's `1/self.mass` scalar (dynamic.py:111-112)
  k.inv_Iz = 1 / v.Iz;      // `1/self.Iz` (dynamic.py:113)
  k.Cm1 = v.Cm1;
  k.Cm2 = v.Cm2;
  k.Cr0 = v.Cr0;
  k.Cr2 = v.Cr2;
  k.input_acc = v.input_acc;
  k.approx = v.approx;
  return k;
}

// The constants an integrator sees: the NLP transcription (Dynamic.casadi + Euler,
// dynamic.py:214-218, nmpc.py:58-60) always uses the pwm motor model and the Pacejka tires,
// so input_acc / approx apply to the batch (RK4 / RK6) forms only.
VehK integrator_veh(VehK k, int32_t integrator) {
  if (integrator == LLAMPC_EULER_NLP) {
    k.input_acc = 0;
    k.approx = 0;
  }
  return k;
}

CostK make_cost(const llampc_cost& c, double Ts) {
  CostK k;
  for (int i = 0; i < 4; ++i) {
    k.Q[i] = c.Q[i];
    k.R[i] = c.R[i];
    k.P[i] = c.P[i];
  }
  for (int i = 0; i < 2; ++i) {
    k.umin[i] = c.umin[i];
    k.umax[i] = c.umax[i];
    // nmpc.py:104-105, tested with a relative tolerance of 1e-9: a sequence rate-clipped to the
    // bound (u_k = u_{k-1} + rate Ts, the candidate samplers) can exceed it by one rounding
    // of u_k - u_{k-1}; IPOPT itself accepts violations up to constr_viol_tol (1e-4)
    k.dmax[i] = c.rate_max[i] < 0 ? -1.0 : c.rate_max[i] * Ts * (1.0 + 1e-9);
  }
  k.enforce = c.enforce_bounds;
  k.pad = 0;
  return k;
}

template <class T>
int dev_alloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
  if (e != hipSuccess)
    return fail(LLAMPC_E_OOM, "hipMalloc(%zu B) failed: %s", count * sizeof(T), hipGetErrorString(e));
  return LLAMPC_OK;
}

}  // namespace

// ---- peer exchange (xGMI mailboxes) -------------------------------------------------
struct llampc_mailbox {
  int32_t world = 0, rank = 0, device = 0;
  uint64_t* own = nullptr;               // [2][world][kRecWords], uncached device memory
  uint64_t* box[kPeerMax] = {};          // every rank's mailbox as mapped in this process
  bool opened[kPeerMax] = {};            // box[g] came from hipIpcOpenMemHandle
  uint32_t seq = 0;
  uint64_t bound = 1000000000ull;        // 10 s of s_memrealtime (100 MHz): ranks may drift apart
                                         // by host-side pauses; only a missing rank should time out
  uint64_t** d_box = nullptr;            // device copy of box[] (the fused exchange reads it)
  bool box_synced = false;
  std::mutex mu;                         // serialises the tick sequence (seq) and the table
};

struct llampc_bank {
  int device = 0;
  int64_t n = 0, goff = 0;
  int32_t W = 0, count = 0, slot = 0;
  VehK veh{};
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool dedicated = false;                // its own stream has a hardware queue of its own (bank_stream)
  int32_t share = 1;                     // banks ticked concurrently (llampc_bank_set_concurrency)
  double* d_params = nullptr;
  double* d_ring = nullptr;
  double* d_am_val = nullptr;
  int64_t* d_am_idx = nullptr;
  double* d_tk_val = nullptr;
  int64_t* d_tk_idx = nullptr;
  double* d_pv = nullptr;
  int64_t* d_pidx = nullptr;
  int32_t* d_pnf = nullptr;
  int32_t* d_best_cand = nullptr;
  double* d_best_cost = nullptr;
  double* h_in = nullptr;          // pinned input pack
  double* d_in = nullptr;
  size_t in_cap = 0;               // doubles
  llampc_plan_out* h_out = nullptr;
  llampc_plan_out* d_out = nullptr;
  double* d_err = nullptr;         // [n]
  double* d_wmean = nullptr;       // [n]
  double* d_cost = nullptr;        // [n*C]
  unsigned* d_tickets = nullptr;   // [2] in-launch completion tickets
  size_t cost_cap = 0;
  std::mutex mu;
  // optional per-kernel event timing: [kernel][2*i] start, [kernel][2*i+1] stop
  std::vector<hipEvent_t> ev[3];
  size_t ev_used[3] = {0, 0, 0};
  bool timing = false;
  int64_t timing_stride = 1;       // group of stride launches per pair (or sampling period)
  bool timing_sample = false;      // pair around one launch of every stride
  bool async_pending = false;      // llampc_plan_async issued, llampc_plan_wait not yet
  double* d_rl = nullptr;          // raceline table: knots | xy | speed | mus
  int32_t rl_n = 0, rl_M = 0;
  double rl_hmin = 1.0, rl_vmax = 0.0;   // the walkers' speed-window bounds (raceline.hpp)
  std::vector<double> rl_mus;            // the profiles' mu values (host copy: the controller's bracket)
  double* d_xref_pm = nullptr;     // per-model references [n][H][2] (RACELINE ticks)
  size_t xref_pm_cap = 0;
  int64_t timing_seen[3] = {0, 0, 0};
  uint64_t* d_la_tag = nullptr;    // polled completion: [3][n] tagged per-model results
  uint64_t* d_blk_tag = nullptr;   // [blocks][5] tagged look-ahead block partials
  uint32_t seq = 0;                // launch tag (1, 2, ...; never 0 = the zeroed buffers)
  // host completion (llampc_plan, llampc_plan_async/wait): the plan kernel writes the record
  // straight into pinned host memory and then stores the tick's number into h_tag; the host
  // spins on h_tag (no D2H copy, no stream synchronisation on the path)
  llampc_plan_out* h_rec = nullptr;  // pinned, coherent; d_rec is its device alias
  llampc_plan_out* d_rec = nullptr;
  uint64_t* h_tag = nullptr;
  uint64_t* d_tag = nullptr;
  uint64_t hseq = 0;
  uint64_t async_seq = 0;          // the outstanding llampc_plan_async tick's tag (0: copy path)
  int64_t launches = 0;            // plan-kernel launches enqueued on this bank (llampc_bank_launches)
  uint64_t* d_wq = nullptr;        // work-queue unit counter (0 between launches; launch_plan's WQ layout)
  // the controller whose armed launch waits on this bank's stream (llampc_ctl_set_prelaunch):
  // every other call that enqueues on the stream cancels it first (bank_disarm)
  llampc_ctl* armed = nullptr;
};

// Cancels the armed controller launch waiting on the bank's stream, if any (defined with the
// controller below): the launch exits without touching anything, and work enqueued after it
// runs once it has.
static void bank_disarm(llampc_bank* b);

namespace {

int ensure_in(llampc_bank* b, size_t doubles) {
  if (doubles <= b->in_cap) return LLAMPC_OK;
  if (b->h_in) (void)hipHostFree(b->h_in);
  if (b->d_in) (void)hipFree(b->d_in);
  b->h_in = nullptr;
  b->d_in = nullptr;
  b->in_cap = 0;
  size_t cap = std::max<size_t>(doubles, 1024);
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&b->h_in), cap * sizeof(double), hipHostMallocDefault));
  int rc = dev_alloc(&b->d_in, cap);
  if (rc) return rc;
  b->in_cap = cap;
  return LLAMPC_OK;
}

int ensure_cost(llampc_bank* b, size_t count) {
  if (count <= b->cost_cap) return LLAMPC_OK;
  if (b->d_cost) (void)hipFree(b->d_cost);
  b->d_cost = nullptr;
  b->cost_cap = 0;
  int rc = dev_alloc(&b->d_cost, count);
  if (rc) return rc;
  b->cost_cap = count;
  return LLAMPC_OK;
}

int ensure_xref_pm(llampc_bank* b, const llampc_plan_in* in) {
  if (!in->do_lookahead || in->xref_mode != LLAMPC_XREF_RACELINE) return LLAMPC_OK;
  const size_t count = (size_t)b->n * 2 * in->H;
  if (count <= b->xref_pm_cap) return LLAMPC_OK;
  if (b->d_xref_pm) (void)hipFree(b->d_xref_pm);
  b->d_xref_pm = nullptr;
  b->xref_pm_cap = 0;
  int rc = dev_alloc(&b->d_xref_pm, count);
  if (rc) return rc;
  b->xref_pm_cap = count;
  return LLAMPC_OK;
}

int check_plan_in(const llampc_bank* b, const llampc_plan_in* in) {
  if (!in) return fail(LLAMPC_E_ARG, "plan input is NULL");
  if (in->do_lookback && (in->K < 1 || in->K > LLAMPC_KMAX))
    return fail(LLAMPC_E_ARG, "K=%d outside [1, %d]", in->K, LLAMPC_KMAX);
  if (in->do_lookback && (!in->x_prev || !in->u_prev || !in->x_now))
    return fail(LLAMPC_E_ARG, "look-back needs x_prev, u_prev and x_now");
  if (in->do_lookahead) {
    if (in->C < 1 || in->H < 1) return fail(LLAMPC_E_ARG, "C=%d H=%d must be >= 1", in->C, in->H);
    if ((int64_t)in->C * in->H > (1 << 26)) return fail(LLAMPC_E_ARG, "C*H too large");
    if (!in->x_now || !in->U || !in->xref || !in->uprev)
      return fail(LLAMPC_E_ARG, "look-ahead needs x_now, U, xref and uprev");
    if (in->integrator < LLAMPC_RK4 || in->integrator > LLAMPC_RK6)
      return fail(LLAMPC_E_ARG, "unknown integrator %d", in->integrator);
    if (in->xref_mode != LLAMPC_XREF_GIVEN && in->xref_mode != LLAMPC_XREF_RACELINE)
      return fail(LLAMPC_E_ARG, "unknown xref_mode %d", in->xref_mode);
    if (in->xref_mode == LLAMPC_XREF_RACELINE && !b->d_rl)
      return fail(LLAMPC_E_STATE, "xref_mode RACELINE needs llampc_bank_set_raceline first");
    if ((b->n + 1) * (int64_t)in->C <= 0 || b->n > INT64_MAX / std::max(1, in->C) - 1)
      return fail(LLAMPC_E_ARG, "n*C overflows");
  }
  if (!in->do_lookback && !in->do_lookahead) return fail(LLAMPC_E_ARG, "nothing to do: look-back and look-ahead both off");
  if (!(in->Ts > 0) || !std::isfinite(in->Ts)) return fail(LLAMPC_E_ARG, "Ts must be finite > 0");
  return LLAMPC_OK;
}

// Event pair around a GROUP of timing_stride consecutive launches of kernel `k` (0 the plan
// kernel; 1, 2 reserved): start before the group's first launch, stop after its last, so a
// launch's mean duration is elapsed / group — the events' own cost (~2 us per record on
// this stack) is spread over the group instead of inflating every bracketed launch.
struct TimedLaunch {
  llampc_bank* b;
  int k;
  hipStream_t s;
  hipEvent_t stop = nullptr;
  TimedLaunch(llampc_bank* b_, int k_, hipStream_t s_) : b(b_), k(k_), s(s_) {
    if (!b->timing || 2 * (b->ev_used[k] + 1) > b->ev[k].size()) return;
    const int64_t pos = b->timing_seen[k]++ % b->timing_stride;
    const size_t i = b->ev_used[k];
    if (pos == 0) (void)hipEventRecord(b->ev[k][2 * i], s);
    // sampling: the pair brackets the period's first launch alone
    if (pos == (b->timing_sample ? 0 : b->timing_stride - 1)) stop = b->ev[k][2 * i + 1];
  }
  ~TimedLaunch() {
    if (stop) {
      (void)hipEventRecord(stop, s);
      b->ev_used[k]++;
    }
  }
};

void timing_free(llampc_bank* b) {
  for (auto& v : b->ev) {
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
    v.clear();
  }
  for (size_t& u : b->ev_used) u = 0;
  for (int64_t& u : b->timing_seen) u = 0;
  b->timing = false;
  b->timing_stride = 1;
  b->timing_sample = false;
}

// The polled completion's wait bound in s_memrealtime ticks (100 MHz): a 2 s floor plus
// 40 ns per look-ahead rollout step of the launch (a rate floor of 2.5e7 steps/s, ~10^3
// below the fast path's, so the general-path re-runs, the raceline walker and launches
// sharing the chip all fit).  A valid long tick (n = 1e7, C = 64, H = 40: ~4 s) therefore
// never reads as a timeout; only a poll that could never finish does.
// LLAMPC_POLL_BOUND_S overrides the floor and LLAMPC_POLL_STEP_NS the per-step term (tests).
uint64_t poll_bound_ticks(int64_t n, int32_t C, int32_t H) {
  double floor_s = 2.0, step_ns = 40.0;
  if (const char* e = getenv("LLAMPC_POLL_BOUND_S")) floor_s = std::max(0.0, atof(e));
  if (const char* e = getenv("LLAMPC_POLL_STEP_NS")) step_ns = std::max(0.0, atof(e));
  const double steps = (double)n * (double)C * (double)H;    // <= 2^57 (check_plan_in)
  const double ticks = 1e8 * floor_s + 0.1 * step_ns * steps;
  return ticks >= 1.8e19 ? ~0ull : (uint64_t)ticks;
}

// Next tick number of a tag sequence: never 0 (the zeroed buffers' tag), and the parity
// alternates across the 32-bit wrap (0xFFFFFFFF -> 2), so consecutive ticks of a peer
// mailbox always use different slots (seq & 1).  Callers commit it only after the launch
// that uses it was enqueued: a failed launch must not leave this rank a tick ahead.
uint32_t next_seq(uint32_t s) { return s == 0xFFFFFFFFu ? 2u : s + 1u; }

// The tick on device pointers: ONE launch (look-back + look-ahead + completion).
// Advances the window bookkeeping when a look-back runs.
int plan_launch(llampc_bank* b, const llampc_plan_in& in, llampc_plan_out* d_out, double* d_err,
                double* d_wmean, double* d_cost, hipStream_t s, uint64_t* host_tag = nullptr,
                uint64_t host_seq = 0, const InlinePack* pk = nullptr,
                llampc_mailbox* px = nullptr, llampc_plan_out* px_merged = nullptr) {
  if (int rc = ensure_xref_pm(b, &in)) return rc;
  const bool lb = in.do_lookback != 0;
  const bool la = in.do_lookahead != 0;
  int32_t count = b->count;
  int32_t full = count >= b->W;
  const int32_t slot = b->slot;
  LookbackLaunch lbl{};
  if (lb) {
    count = std::min(count + 1, b->W);             // rt.py:354
    full = count >= b->W;                          // rt.py:357
    lbl.params = b->d_params;
    lbl.n = b->n;
    lbl.goff = b->goff;
    lbl.veh = b->veh;
    lbl.x_prev = in.x_prev;
    lbl.u_prev = in.u_prev;
    lbl.x_now = in.x_now;
    lbl.Ts = in.Ts;
    lbl.ring = b->d_ring;
    lbl.W = b->W;
    lbl.slot = slot;
    lbl.full = full;
    lbl.K = in.K;
    lbl.nan_first = in.nan_policy == LLAMPC_NAN_FIRST;
    lbl.err_out = d_err;
    lbl.wm_buf = d_wmean ? d_wmean : b->d_wmean;
    lbl.wm_keep = d_wmean != nullptr;              // else only the R > 1 second pass reads it
    lbl.am_val = b->d_am_val;
    lbl.am_idx = b->d_am_idx;
    lbl.tk_val = b->d_tk_val;
    lbl.tk_idx = b->d_tk_idx;
  }
  LookaheadLaunch lal{};
  if (la) {
    lal.params = b->d_params;
    lal.n = b->n;
    lal.goff = b->goff;
    lal.veh = integrator_veh(b->veh, in.integrator);
    lal.x0 = in.x_now;
    lal.U = in.U;
    lal.xref = in.xref;
    lal.uprev = in.uprev;
    lal.C = in.C;
    lal.H = in.H;
    lal.integrator = in.integrator;
    lal.Ts = in.Ts;
    lal.cost = make_cost(in.cost, in.Ts);
    lal.cost_out = d_cost;
    lal.best_cand = b->d_best_cand;
    lal.best_cost = b->d_best_cost;
    lal.pv = b->d_pv;
    lal.pidx = b->d_pidx;
    lal.pnf = b->d_pnf;
    lal.xref_mode = in.xref_mode;
    if (in.xref_mode == LLAMPC_XREF_RACELINE) {
      const size_t m = (size_t)b->rl_n - 1;
      lal.rl.knots = b->d_rl;
      lal.rl.xy = b->d_rl + b->rl_n;
      lal.rl.speed = lal.rl.xy + 8 * m;
      lal.rl.mus = lal.rl.speed + 4 * m * b->rl_M;
      lal.rl.n = b->rl_n;
      lal.rl.M = b->rl_M;
      lal.rl.hmin = b->rl_hmin;
      lal.rl.vmax = b->rl_vmax;
      lal.rl.wcap = 0;                    // set by launch_plan from the LDS it leaves
      lal.xref_pm = b->d_xref_pm;       // sized by ensure_xref_pm before the launch
    }
  }
  FinalLaunch f{};
  f.out = d_out;
  f.tickets = b->d_tickets;
  f.full = full;
  f.window_count = count;
  f.K = lb ? in.K : 0;
  f.nan_first = in.nan_policy == LLAMPC_NAN_FIRST;
  f.C = la ? in.C : 1;
  f.current_model = in.current_model;
  f.n = b->n;
  f.goff = b->goff;
  f.params = b->d_params;
  f.best_cand = b->d_best_cand;
  f.best_cost = b->d_best_cost;
  f.am_val = b->d_am_val;
  f.am_idx = b->d_am_idx;
  f.tk_val = b->d_tk_val;
  f.tk_idx = b->d_tk_idx;
  f.pv = b->d_pv;
  f.pidx = b->d_pidx;
  f.pnf = b->d_pnf;
  // polled completion whenever look-back blocks exist to host the poller (LLAMPC_NO_POLL=1:
  // the ticket + last-block path, for A/B runs)
  const bool no_poll = getenv("LLAMPC_NO_POLL") != nullptr;
  const int32_t poll = (lb && la && !no_poll) ? 1 : 0;
  const uint32_t seq = poll ? next_seq(b->seq) : b->seq;
  f.la_tag = b->d_la_tag;
  f.blk_tag = b->d_blk_tag;
  f.seq = seq;
  if (poll) {                           // the bound in 2^16-tick units, at least one
    const uint64_t units = (poll_bound_ticks(b->n, in.C, in.H) + 0xFFFF) >> 16;
    f.poll = (int32_t)std::min<uint64_t>(std::max<uint64_t>(units, 1), INT32_MAX);
  } else {
    f.poll = 0;
  }
  f.host_tag = host_tag;
  f.host_seq = host_seq;
  const uint32_t px_seq = px ? next_seq(px->seq) : 0;
  if (px) {                             // fused peer exchange (llampc_plan_exchange)
    f.px_box = px->d_box;
    f.px_merged = px_merged;
    f.px_G = px->world;
    f.px_rank = px->rank;
    f.px_seq = px_seq;
    f.px_bound = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((px->bound + 0xFFFF) >> 16, 1), UINT32_MAX);
  }
  if (la) {
    lal.la_tag = b->d_la_tag;
    lal.blk_tag = b->d_blk_tag;
    lal.seq = seq;
    lal.poll = poll;
    lal.wq = b->d_wq;
  }
  f.wq = b->d_wq;
  {
    TimedLaunch tl(b, 0, s);
    HIP_TRY(launch_plan(lb ? &lbl : nullptr, la ? &lal : nullptr, f, s, pk, b->share));
  }
  b->seq = seq;
  if (px) px->seq = px_seq;
  b->launches++;
  if (lb) {
    b->slot = (slot + 1) % b->W;
    b->count = count;
  }
  return LLAMPC_OK;
}

// Doubles of the packed inputs: x_prev[6] u_prev[2] x_now[6] uprev[2] xref[2][H+1] U[C][H][2].
size_t pack_len(const llampc_plan_in* in) {
  const int64_t H = in->do_lookahead ? in->H : 0, C = in->do_lookahead ? in->C : 0;
  return 16 + 2 * (H + 1) + 2 * C * H;
}

void pack_into(const llampc_plan_in* in, double* h) {
  const int64_t H = in->do_lookahead ? in->H : 0, C = in->do_lookahead ? in->C : 0;
  std::memset(h, 0, 16 * sizeof(double));
  if (in->x_prev) std::memcpy(h + 0, in->x_prev, 6 * sizeof(double));
  if (in->u_prev) std::memcpy(h + 6, in->u_prev, 2 * sizeof(double));
  if (in->x_now) std::memcpy(h + 8, in->x_now, 6 * sizeof(double));
  if (in->uprev) std::memcpy(h + 14, in->uprev, 2 * sizeof(double));
  if (in->do_lookahead) {
    if (in->xref_mode == LLAMPC_XREF_RACELINE) {       // {s0, v0, scale, 0} (<= 2(H+1) slots)
      std::memset(h + 16, 0, 2 * (H + 1) * sizeof(double));
      std::memcpy(h + 16, in->xref, 3 * sizeof(double));
    } else {
      std::memcpy(h + 16, in->xref, 2 * (H + 1) * sizeof(double));
    }
    std::memcpy(h + 16 + 2 * (H + 1), in->U, 2 * C * H * sizeof(double));
  }
}

// Host ticks whose inputs travel as kernel arguments (InlinePack): no H2D copy.
// LLAMPC_NO_INLINE=1 keeps the copy (A/B runs).
bool inline_inputs(const llampc_plan_in* in) {
  return in->do_lookahead && plan_inline_ok(in->C, in->H, in->integrator, in->xref_mode) &&
         getenv("LLAMPC_NO_INLINE") == nullptr;
}

// Pack a host plan input into the pinned buffer; return a device-pointer copy of `in`.
int stage_inputs(llampc_bank* b, const llampc_plan_in* in, llampc_plan_in* dev_in, hipStream_t s) {
  const size_t total = pack_len(in);
  const int64_t H = in->do_lookahead ? in->H : 0;
  int rc = ensure_in(b, total);
  if (rc) return rc;
  double* h = b->h_in;
  pack_into(in, h);
  HIP_TRY(hipMemcpyAsync(b->d_in, h, total * sizeof(double), hipMemcpyHostToDevice, s));
  *dev_in = *in;
  double* d = b->d_in;
  dev_in->x_prev = d;
  dev_in->u_prev = d + 6;
  dev_in->x_now = d + 8;
  dev_in->uprev = d + 14;
  dev_in->xref = d + 16;
  dev_in->U = d + 16 + 2 * (H + 1);
  return LLAMPC_OK;
}

hipStream_t pick_stream(llampc_bank* b, void* s) { return s ? (hipStream_t)s : b->stream; }

// Host completion is the default for host-pointer ticks that return only the record;
// LLAMPC_SYNC_COMPLETION=1 selects the D2H copy + hipStreamSynchronize path (A/B runs).
bool host_completion(const llampc_bank* b) {
  return b->h_tag && b->h_rec && getenv("LLAMPC_SYNC_COMPLETION") == nullptr;
}

// After a tick whose record reports a device-side status (an in-launch wait gave up) or whose
// completion never arrived: once the stream has drained, every in-launch counter is zeroed —
// the work-queue counter (straggler blocks may have taken units after final_write reset it)
// and the tickets — so the next launch starts from a clean hand-off state.
int recover_counters(llampc_bank* b) {
  HIP_TRY(hipStreamSynchronize(b->stream));
  HIP_TRY(hipMemsetAsync(b->d_wq, 0, sizeof(uint64_t), b->stream));
  HIP_TRY(hipMemsetAsync(b->d_tickets, 0, 2 * sizeof(unsigned), b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  return LLAMPC_OK;
}

int status_fail(llampc_bank* b, int32_t status) {
  (void)recover_counters(b);
  return fail(LLAMPC_E_DEVICE, "tick record status %d (in-launch completion timed out)", status);
}

// Spin until the plan kernel has published tick `seq` in h_tag, then copy the record out.
// A tag that never arrives (a device fault) ends the spin after 10 s: the stream is then
// synchronised so the HIP error, if any, is the one reported.
int wait_host_tag(llampc_bank* b, uint64_t seq, llampc_plan_out* out) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  while (__atomic_load_n(b->h_tag, __ATOMIC_ACQUIRE) != seq) {
    __builtin_ia32_pause();
    if ((++spins & 0xFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      HIP_TRY(hipStreamSynchronize(b->stream));
      if (__atomic_load_n(b->h_tag, __ATOMIC_ACQUIRE) == seq) break;
      (void)recover_counters(b);
      return fail(LLAMPC_E_DEVICE, "tick %llu: completion tag never arrived", (unsigned long long)seq);
    }
  }
  std::memcpy(out, const_cast<const llampc_plan_out*>(b->h_rec), sizeof(llampc_plan_out));
  return LLAMPC_OK;
}



}  // namespace

namespace {
// A bank's stream.  HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 by
// default, least-used first), so two banks ticked concurrently — the two controllers of
// config 5 — can land on one queue and run one after the other: the two-track controller
// step measured 172 us instead of 98 us whenever two other streams were in use first
// (tools/diag/bench_extra.py).  A stream with a CU mask gets a hardware queue of its own;
// the mask holds every CU, so nothing else changes.  LLAMPC_SHARED_QUEUES=1 keeps the plain
// stream; the plain stream is also the fallback.  Only banks ticked concurrently get one
// (llampc_bank_set_concurrency(> 1), or LLAMPC_DEDICATED_QUEUE=1 at create): every other bank
// — a setupNLP's one-model bank, a host-mode nominal bank — keeps a plain non-blocking stream,
// so a process never opens more hardware queues than it has concurrent banks.
hipError_t bank_stream(int device, bool dedicated, hipStream_t* s) {
  if (dedicated && !std::getenv("LLAMPC_SHARED_QUEUES")) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) {
      std::vector<uint32_t> mask((cus + 31) / 32, 0xFFFFFFFFu);
      if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
      if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return hipSuccess;
      (void)hipGetLastError();
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
}  // namespace

extern "C" {

int32_t llampc_abi_version(void) { return LLAMPC_ABI_VERSION; }

const char* llampc_last_error(void) { return g_err.c_str(); }

int llampc_device_count(int32_t* count) {
  if (!count) return fail(LLAMPC_E_ARG, "count is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return fail(LLAMPC_E_NODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = c;
  return LLAMPC_OK;
}

int llampc_bank_create(const double* params, int64_t n, int64_t global_offset,
                       const llampc_vehicle* veh, int32_t W, int32_t device, llampc_bank** out) {
  if (!out) return fail(LLAMPC_E_ARG, "out is NULL");
  *out = nullptr;
  if (!params || !veh) return fail(LLAMPC_E_ARG, "params/veh is NULL");
  if (n < 1 || n > INT32_MAX)   // the kernels rank models by a 32-bit local index
    return fail(LLAMPC_E_ARG, "n=%lld must be in [1, 2^31-1]", (long long)n);
  if (W < 1 || W > LLAMPC_WMAX) return fail(LLAMPC_E_ARG, "W=%d outside [1, %d]", W, LLAMPC_WMAX);
  if (global_offset < 0) return fail(LLAMPC_E_ARG, "global_offset < 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return fail(LLAMPC_E_NODEV, "no HIP device visible (the HIP path has no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(LLAMPC_E_ARG, "device %d of %d", device, ndev);
  DeviceGuard g(device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", device);

  auto* b = new llampc_bank();
  b->device = device;
  b->n = n;
  b->goff = global_offset;
  b->W = W;
  b->veh = make_veh(*veh);
  int rc = LLAMPC_OK;
  auto cleanup = [&](int code) {
    llampc_bank_destroy(b);
    return code;
  };
  if (const char* e = std::getenv("LLAMPC_DEDICATED_QUEUE")) b->dedicated = e[0] == '1';
  if (bank_stream(device, b->dedicated, &b->stream) != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "hipStreamCreate failed"));
  b->own_stream = true;
  const int64_t lbl = (int64_t)lookback_blocks(n) * (kBlock / 64);   // look-back lists (waves)
  const int64_t lab = n;                 // worst case: one model per block (wave-role, G=64)
  if ((rc = dev_alloc(&b->d_params, 6 * (size_t)n)) || (rc = dev_alloc(&b->d_ring, (size_t)W * n)) ||
      (rc = dev_alloc(&b->d_am_val, lbl)) || (rc = dev_alloc(&b->d_am_idx, lbl)) ||
      (rc = dev_alloc(&b->d_tk_val, (size_t)lbl * LLAMPC_KMAX)) ||
      (rc = dev_alloc(&b->d_tk_idx, (size_t)lbl * LLAMPC_KMAX)) || (rc = dev_alloc(&b->d_pv, lab)) ||
      (rc = dev_alloc(&b->d_pidx, lab)) || (rc = dev_alloc(&b->d_pnf, lab)) ||
      (rc = dev_alloc(&b->d_best_cand, n)) || (rc = dev_alloc(&b->d_best_cost, n)) ||
      (rc = dev_alloc(&b->d_err, n)) || (rc = dev_alloc(&b->d_wmean, n)) ||
      (rc = dev_alloc(&b->d_out, 1)) || (rc = dev_alloc(&b->d_tickets, 2)) ||
      (rc = dev_alloc(&b->d_la_tag, 3 * (size_t)n)) || (rc = dev_alloc(&b->d_blk_tag, 5 * (size_t)lab)) ||
      (rc = dev_alloc(&b->d_wq, 1)))
    return cleanup(rc);
  if (hipHostMalloc(reinterpret_cast<void**>(&b->h_out), sizeof(llampc_plan_out), hipHostMallocDefault) != hipSuccess)
    return cleanup(fail(LLAMPC_E_OOM, "hipHostMalloc(out) failed"));
  if (hipHostMalloc(reinterpret_cast<void**>(&b->h_rec), sizeof(llampc_plan_out),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&b->h_tag), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return cleanup(fail(LLAMPC_E_OOM, "hipHostMalloc(host completion record) failed"));
  *b->h_tag = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&b->d_rec), b->h_rec, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&b->d_tag), b->h_tag, 0) != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "hipHostGetDevicePointer(host completion record) failed"));
  if (hipMemcpy(b->d_params, params, 6 * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(b->d_ring, 0, (size_t)W * n * sizeof(double)) != hipSuccess ||
      hipMemset(b->d_tickets, 0, 2 * sizeof(unsigned)) != hipSuccess ||
      hipMemset(b->d_la_tag, 0, 3 * (size_t)n * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(b->d_blk_tag, 0, 5 * (size_t)lab * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(b->d_wq, 0, sizeof(uint64_t)) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "bank upload failed"));
  *out = b;
  return LLAMPC_OK;
}

int llampc_bank_destroy(llampc_bank* b) {
  if (!b) return LLAMPC_OK;
  bank_disarm(b);
  {
    DeviceGuard g(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    void* dptrs[] = {b->d_params, b->d_ring, b->d_am_val, b->d_am_idx, b->d_tk_val, b->d_tk_idx,
                     b->d_pv, b->d_pidx, b->d_pnf, b->d_best_cand, b->d_best_cost, b->d_in,
                     b->d_out, b->d_err, b->d_wmean, b->d_cost, b->d_tickets, b->d_rl,
                     b->d_xref_pm, b->d_la_tag, b->d_blk_tag, b->d_wq};
    for (void* p : dptrs)
      if (p) (void)hipFree(p);
    if (b->h_in) (void)hipHostFree(b->h_in);
    if (b->h_out) (void)hipHostFree(b->h_out);
    if (b->h_rec) (void)hipHostFree(b->h_rec);
    if (b->h_tag) (void)hipHostFree(b->h_tag);
    timing_free(b);
    if (b->own_stream && b->stream) (void)hipStreamDestroy(b->stream);
  }
  delete b;
  return LLAMPC_OK;
}

int llampc_bank_info(const llampc_bank* b, int64_t* n, int64_t* goff, int32_t* W,
                     int32_t* window_count, int32_t* device) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  if (n) *n = b->n;
  if (goff) *goff = b->goff;
  if (W) *W = b->W;
  if (window_count) *window_count = b->count;
  if (device) *device = b->device;
  return LLAMPC_OK;
}

int llampc_bank_launches(const llampc_bank* b, int64_t* launches) {
  if (!b || !launches) return fail(LLAMPC_E_ARG, "bank/launches is NULL");
  *launches = b->launches;
  return LLAMPC_OK;
}

int llampc_bank_reset(llampc_bank* b) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  DeviceGuard g(b->device);
  HIP_TRY(hipMemsetAsync(b->d_ring, 0, (size_t)b->W * b->n * sizeof(double), b->stream));
  HIP_TRY(hipMemsetAsync(b->d_tickets, 0, 2 * sizeof(unsigned), b->stream));
  HIP_TRY(hipMemsetAsync(b->d_wq, 0, sizeof(uint64_t), b->stream));
  HIP_TRY(hipStreamSynchronize(b->stream));
  b->count = 0;
  b->slot = 0;
  return LLAMPC_OK;
}

int llampc_bank_window(llampc_bank* b, double* ring, int32_t* window_count) {
  if (!b || !ring) return fail(LLAMPC_E_ARG, "bank/ring is NULL");
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  DeviceGuard g(b->device);
  std::vector<double> raw((size_t)b->W * b->n);
  HIP_TRY(hipStreamSynchronize(b->stream));
  HIP_TRY(hipMemcpy(raw.data(), b->d_ring, raw.size() * sizeof(double), hipMemcpyDeviceToHost));
  // rt.py layout [n][W]: newest in column W-1, unfilled (oldest) columns zero.
  const int W = b->W, cnt = b->count;
  for (int64_t i = 0; i < b->n; ++i) {
    for (int c = 0; c < W; ++c) {
      const int age = W - 1 - c;                   // 0 = newest
      double v = 0.0;
      if (age < cnt) {
        const int s = ((b->slot - 1 - age) % W + W) % W;
        v = raw[(size_t)s * b->n + i];
      }
      ring[(size_t)i * W + c] = v;
    }
  }
  if (window_count) *window_count = cnt;
  return LLAMPC_OK;
}

int llampc_bank_stream(const llampc_bank* b, void** stream) {
  if (!b || !stream) return fail(LLAMPC_E_ARG, "NULL argument");
  *stream = (void*)b->stream;
  return LLAMPC_OK;
}

// The bank's own stream on a hardware queue of its own (bank_stream), replacing a plain one
// (the caller holds b->mu; nothing may be armed on it).
static int bank_dedicate(llampc_bank* b) {
  if (b->dedicated) return LLAMPC_OK;
  b->dedicated = true;
  if (b->own_stream) {
    DeviceGuard g(b->device);
    HIP_TRY(hipStreamSynchronize(b->stream));
    hipStream_t s = nullptr;
    HIP_TRY(bank_stream(b->device, true, &s));
    (void)hipStreamDestroy(b->stream);
    b->stream = s;
  }
  return LLAMPC_OK;
}

int llampc_bank_set_concurrency(llampc_bank* b, int32_t banks) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  if (banks < 1 || banks > 64) return fail(LLAMPC_E_ARG, "banks=%d outside [1, 64]", banks);
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  b->share = banks;
  if (banks > 1) return bank_dedicate(b);   // concurrent banks: a hardware queue of its own
  return LLAMPC_OK;
}

int llampc_bank_set_stream(llampc_bank* b, void* stream) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  DeviceGuard g(b->device);
  HIP_TRY(hipStreamSynchronize(b->stream));
  if (b->own_stream) (void)hipStreamDestroy(b->stream);
  if (stream) {
    b->stream = (hipStream_t)stream;
    b->own_stream = false;
  } else {
    HIP_TRY(bank_stream(b->device, b->dedicated, &b->stream));
    b->own_stream = true;
  }
  return LLAMPC_OK;
}

int llampc_bank_timing(llampc_bank* b, int32_t enable, int32_t max_launches) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  std::lock_guard<std::mutex> lk(b->mu);
  DeviceGuard g(b->device);
  HIP_TRY(hipStreamSynchronize(b->stream));
  timing_free(b);
  if (!enable) return LLAMPC_OK;
  if (enable == INT32_MIN) return fail(LLAMPC_E_ARG, "bad enable");
  if (max_launches < 1) return fail(LLAMPC_E_ARG, "max_launches must be >= 1");
  for (auto& v : b->ev) {
    v.resize(2 * (size_t)max_launches, nullptr);
    for (hipEvent_t& e : v) HIP_TRY(hipEventCreate(&e));
  }
  b->timing = true;
  b->timing_stride = enable < 0 ? -(int64_t)enable : enable;
  b->timing_sample = enable < 0;
  return LLAMPC_OK;
}

int llampc_bank_timing_read(llampc_bank* b, double* avg_ms, int64_t* count) {
  if (!b || !avg_ms || !count) return fail(LLAMPC_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(b->mu);
  DeviceGuard g(b->device);
  for (int k = 0; k < 3; ++k) {
    double tot = 0.0;
    for (size_t i = 0; i < b->ev_used[k]; ++i) {
      HIP_TRY(hipEventSynchronize(b->ev[k][2 * i + 1]));
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, b->ev[k][2 * i], b->ev[k][2 * i + 1]));
      tot += ms;
    }
    const int64_t per = b->timing_sample ? 1 : b->timing_stride;   // launches per pair
    count[k] = (int64_t)b->ev_used[k] * per;
    avg_ms[k] = b->ev_used[k] ? tot / ((double)b->ev_used[k] * per) : 0.0;
    b->ev_used[k] = 0;
    b->timing_seen[k] = 0;
  }
  return LLAMPC_OK;
}

int llampc_plan(llampc_bank* b, const llampc_plan_in* in, llampc_plan_out* out, double* err_out,
                double* wmean_out, double* cost_out) {
  if (!b || !out) return fail(LLAMPC_E_ARG, "bank/out is NULL");
  int rc = check_plan_in(b, in);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async tick is outstanding: call llampc_plan_wait");
  DeviceGuard g(b->device);
  hipStream_t s = b->stream;
  if (cost_out && in->do_lookahead && (rc = ensure_cost(b, (size_t)b->n * in->C))) return rc;
  if (!err_out && !wmean_out && !cost_out && host_completion(b)) {
    // the record only: the kernel writes it to pinned host memory and publishes a tag
    llampc_plan_in din = *in;
    InlinePack pk;
    const bool inl = inline_inputs(in);
    if (inl) pack_into(in, pk.v);
    else if ((rc = stage_inputs(b, in, &din, s))) return rc;
    const uint64_t seq = ++b->hseq;
    if ((rc = plan_launch(b, din, b->d_rec, nullptr, nullptr, nullptr, s, b->d_tag, seq, inl ? &pk : nullptr)))
      return rc;
    if ((rc = wait_host_tag(b, seq, out))) return rc;
    if (out->status) return status_fail(b, out->status);
    return LLAMPC_OK;
  }
  llampc_plan_in din;
  if ((rc = stage_inputs(b, in, &din, s))) return rc;
  double* d_cost = (cost_out && in->do_lookahead) ? b->d_cost : nullptr;
  if ((rc = plan_launch(b, din, b->d_out, err_out ? b->d_err : nullptr,
                        wmean_out ? b->d_wmean : nullptr, d_cost, s)))
    return rc;
  HIP_TRY(hipMemcpyAsync(b->h_out, b->d_out, sizeof(llampc_plan_out), hipMemcpyDeviceToHost, s));
  if (err_out && in->do_lookback)
    HIP_TRY(hipMemcpyAsync(err_out, b->d_err, b->n * sizeof(double), hipMemcpyDeviceToHost, s));
  if (wmean_out && in->do_lookback && b->count >= b->W)
    HIP_TRY(hipMemcpyAsync(wmean_out, b->d_wmean, b->n * sizeof(double), hipMemcpyDeviceToHost, s));
  if (d_cost)
    HIP_TRY(hipMemcpyAsync(cost_out, d_cost, (size_t)b->n * in->C * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *out = *b->h_out;
  if (out->status) return status_fail(b, out->status);
  return LLAMPC_OK;
}

int llampc_bank_set_raceline(llampc_bank* b, const double* knots, int32_t n, const double* xy,
                             const double* speed, const double* mus, int32_t M) {
  if (!b || !knots || !xy || !speed || !mus) return fail(LLAMPC_E_ARG, "NULL argument");
  if (n < 2 || M < 1 || M > 64) return fail(LLAMPC_E_ARG, "n=%d (>= 2) M=%d (1..64)", n, M);
  if (raceline_lds_bytes(n, M) > 60 * 1024)
    return fail(LLAMPC_E_ARG, "raceline of %d knots exceeds the 60 KB LDS stage", n);
  for (int32_t i = 1; i < n; ++i)
    if (!(knots[i] > knots[i - 1])) return fail(LLAMPC_E_ARG, "knots must increase (at %d)", i);
  for (int32_t i = 1; i < M; ++i)
    if (!(mus[i] >= mus[i - 1])) return fail(LLAMPC_E_ARG, "mus must be ascending (at %d)", i);
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  DeviceGuard g(b->device);
  HIP_TRY(hipStreamSynchronize(b->stream));
  const size_t m = (size_t)n - 1;
  const size_t total = (size_t)n + 8 * m + 4 * m * M + M;
  if (b->d_rl) (void)hipFree(b->d_rl);
  b->d_rl = nullptr;
  b->rl_n = b->rl_M = 0;
  int rc = dev_alloc(&b->d_rl, total);
  if (rc) return rc;
  double* d = b->d_rl;
  HIP_TRY(hipMemcpy(d, knots, n * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d + n, xy, 8 * m * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d + n + 8 * m, speed, 4 * m * M * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d + n + 8 * m + 4 * m * M, mus, M * sizeof(double), hipMemcpyHostToDevice));
  b->rl_n = n;
  b->rl_M = M;
  b->rl_mus.assign(mus, mus + M);
  double hmin = knots[1] - knots[0];
  for (int32_t i = 2; i < n; ++i) hmin = std::min(hmin, knots[i] - knots[i - 1]);
  b->rl_hmin = hmin;
  b->rl_vmax = speed_bound(knots, speed, n, M);
  return LLAMPC_OK;
}

int llampc_plan_async(llampc_bank* b, const llampc_plan_in* in) {
  if (!b) return fail(LLAMPC_E_ARG, "bank is NULL");
  int rc = check_plan_in(b, in);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async tick is outstanding: call llampc_plan_wait");
  DeviceGuard g(b->device);
  hipStream_t s = b->stream;
  llampc_plan_in din = *in;
  if (host_completion(b)) {
    InlinePack pk;
    const bool inl = inline_inputs(in);
    if (inl) pack_into(in, pk.v);
    else if ((rc = stage_inputs(b, in, &din, s))) return rc;
    b->async_seq = ++b->hseq;
    if ((rc = plan_launch(b, din, b->d_rec, nullptr, nullptr, nullptr, s, b->d_tag, b->async_seq,
                          inl ? &pk : nullptr)))
      return rc;
  } else {
    if ((rc = stage_inputs(b, in, &din, s))) return rc;
    b->async_seq = 0;
    if ((rc = plan_launch(b, din, b->d_out, nullptr, nullptr, nullptr, s))) return rc;
    HIP_TRY(hipMemcpyAsync(b->h_out, b->d_out, sizeof(llampc_plan_out), hipMemcpyDeviceToHost, s));
  }
  b->async_pending = true;
  return LLAMPC_OK;
}

int llampc_plan_wait(llampc_bank* b, llampc_plan_out* out) {
  if (!b || !out) return fail(LLAMPC_E_ARG, "bank/out is NULL");
  std::lock_guard<std::mutex> lk(b->mu);
  if (!b->async_pending) return fail(LLAMPC_E_STATE, "no async tick outstanding");
  DeviceGuard g(b->device);
  b->async_pending = false;
  if (b->async_seq) {
    if (int rc = wait_host_tag(b, b->async_seq, out)) return rc;
  } else {
    HIP_TRY(hipStreamSynchronize(b->stream));
    *out = *b->h_out;
  }
  if (out->status) return status_fail(b, out->status);
  return LLAMPC_OK;
}

int llampc_plan_device(llampc_bank* b, const llampc_plan_in* in, void* d_out, double* d_err,
                       double* d_wmean, double* d_cost, void* stream) {
  if (!b || !d_out) return fail(LLAMPC_E_ARG, "bank/d_out is NULL");
  int rc = check_plan_in(b, in);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  // an outstanding async tick shares the tickets, tags, ring slot and window count
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async tick is outstanding: call llampc_plan_wait");
  DeviceGuard g(b->device);
  return plan_launch(b, *in, (llampc_plan_out*)d_out, d_err, d_wmean, d_cost, pick_stream(b, stream));
}

int llampc_lookback(llampc_bank* b, const double* x_prev, const double* u_prev, const double* x_now,
                    double Ts, int32_t K, int32_t nan_policy, double* err_out, double* wmean_out,
                    int64_t* best, int64_t* topk, double* topk_val, int32_t* window_count) {
  llampc_plan_in in{};
  in.x_prev = x_prev;
  in.u_prev = u_prev;
  in.x_now = x_now;
  in.K = K;
  in.do_lookback = 1;
  in.do_lookahead = 0;
  in.nan_policy = nan_policy;
  in.current_model = -1;
  in.Ts = Ts;
  llampc_plan_out o;
  int rc = llampc_plan(b, &in, &o, err_out, wmean_out, nullptr);
  if (rc) return rc;
  if (best) *best = o.window_full ? o.lb_best : -1;
  for (int k = 0; k < K; ++k) {
    if (topk) topk[k] = o.topk[k];
    if (topk_val) topk_val[k] = o.topk_val[k];
  }
  if (window_count) *window_count = o.window_count;
  return LLAMPC_OK;
}

int llampc_lookahead(llampc_bank* b, const double* x0, const double* U, int32_t C, int32_t H,
                     const double* xref, const double* uprev, const llampc_cost* cost, double Ts,
                     int32_t integrator, double* cost_out, int32_t* best_cand_out,
                     int64_t* best_model, int32_t* best_cand, double* best_cost) {
  if (!cost) return fail(LLAMPC_E_ARG, "cost is NULL");
  llampc_plan_in in{};
  in.x_now = x0;
  in.U = U;
  in.C = C;
  in.H = H;
  in.xref = xref;
  in.uprev = uprev;
  in.K = 1;
  in.integrator = integrator;
  in.do_lookback = 0;
  in.do_lookahead = 1;
  in.current_model = -1;
  in.Ts = Ts;
  in.cost = *cost;
  llampc_plan_out o;
  int rc = llampc_plan(b, &in, &o, nullptr, nullptr, cost_out);
  if (rc) return rc;
  if (best_cand_out) {
    DeviceGuard g(b->device);
    HIP_TRY(hipMemcpy(best_cand_out, b->d_best_cand, b->n * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  if (best_model) *best_model = o.la_best_model;
  if (best_cand) *best_cand = o.la_best_cand;
  if (best_cost) *best_cost = o.la_best_cost;
  return LLAMPC_OK;
}

int llampc_merge(const llampc_plan_out* parts, int32_t G, int32_t nan_policy, llampc_plan_out* merged) {
  if (!parts || !merged || G < 1) return fail(LLAMPC_E_ARG, "bad merge arguments");
  for (int g = 1; g < G; ++g)
    if (parts[g].K != parts[0].K || parts[g].window_count != parts[0].window_count)
      return fail(LLAMPC_E_STATE, "shard %d disagrees on K/window (K %d vs %d, count %d vs %d)", g,
                  parts[g].K, parts[0].K, parts[g].window_count, parts[0].window_count);
  merge_plan_parts(parts, G, nan_policy == LLAMPC_NAN_FIRST, merged);
  return LLAMPC_OK;
}

int llampc_merge_device(const void* d_parts, int32_t G, int32_t nan_policy, void* d_merged,
                        int32_t device, void* stream) {
  if (!d_parts || !d_merged || G < 1) return fail(LLAMPC_E_ARG, "bad merge arguments");
  DeviceGuard g(device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", device);
  HIP_TRY(launch_merge((const llampc_plan_out*)d_parts, G, nan_policy == LLAMPC_NAN_FIRST,
                       (llampc_plan_out*)d_merged, (hipStream_t)stream));
  return LLAMPC_OK;
}

}  // extern "C"

// ---- RCCL: the library's own communicator (rccl.h) ----------------------------------
// RCCL is resolved at first use, not linked: the librccl.so.1 the process already holds
// (torch's bundled RCCL carries that soname: one RCCL per process, whatever the import order
// of torch and this library), else the system's.  A process that never exchanges over RCCL
// never loads it.
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
  bool ok = false;
  std::string why;
};
const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      x.why = e ? e : "librccl.so.1 not found";
      return x;
    }
    x.get_id = reinterpret_cast<decltype(x.get_id)>(dlsym(h, "ncclGetUniqueId"));
    x.init_rank = reinterpret_cast<decltype(x.init_rank)>(dlsym(h, "ncclCommInitRank"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(h, "ncclAllGather"));
    x.err_str = reinterpret_cast<decltype(x.err_str)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_id && x.init_rank && x.destroy && x.all_gather && x.err_str;
    if (!x.ok) x.why = "librccl.so.1 lacks an ncclGetUniqueId/ncclCommInitRank/ncclAllGather symbol";
    return x;
  }();
  return r;
}
static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes (llampc_comm_unique_id)");
}  // namespace

struct llampc_comm {
  ncclComm_t comm = nullptr;
  int32_t world = 0, rank = 0, device = 0;
};

#define RCCL_TRY(expr)                                                                         \
  do {                                                                                         \
    const ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) return fail(LLAMPC_E_HIP, "%s failed: %s", #expr, rccl().err_str(r_)); \
  } while (0)

extern "C" {

int llampc_comm_unique_id(void* id) {
  if (!id) return fail(LLAMPC_E_ARG, "id is NULL");
  if (!rccl().ok) return fail(LLAMPC_E_STATE, "RCCL unavailable: %s", rccl().why.c_str());
  ncclUniqueId u;
  RCCL_TRY(rccl().get_id(&u));
  std::memcpy(id, &u, sizeof u);
  return LLAMPC_OK;
}

int llampc_comm_create(const void* id, int32_t world, int32_t rank, int32_t device, llampc_comm** out) {
  if (!out) return fail(LLAMPC_E_ARG, "out is NULL");
  *out = nullptr;
  if (!id || world < 1 || rank < 0 || rank >= world) return fail(LLAMPC_E_ARG, "bad comm arguments (world=%d rank=%d)", world, rank);
  if (!rccl().ok) return fail(LLAMPC_E_STATE, "RCCL unavailable: %s", rccl().why.c_str());
  DeviceGuard g(device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", device);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  RCCL_TRY(rccl().init_rank(&comm, world, u, rank));
  auto* c = new llampc_comm();
  c->comm = comm;
  c->world = world;
  c->rank = rank;
  c->device = device;
  *out = c;
  return LLAMPC_OK;
}

int llampc_comm_destroy(llampc_comm* c) {
  if (!c) return LLAMPC_OK;
  if (c->comm && rccl().ok) {
    DeviceGuard g(c->device);
    (void)rccl().destroy(c->comm);
  }
  delete c;
  return LLAMPC_OK;
}

int llampc_exchange_rccl(llampc_comm* comm, const void* d_local, void* d_all, void* d_merged, int32_t nan_policy,
                         void* stream) {
  if (!comm || !d_local || !d_all || !d_merged || comm->world > 32)
    return fail(LLAMPC_E_ARG, "bad exchange arguments (world 1..32)");
  DeviceGuard g(comm->device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", comm->device);
  RCCL_TRY(rccl().all_gather(d_local, d_all, sizeof(llampc_plan_out), ncclUint8, comm->comm, (hipStream_t)stream));
  HIP_TRY(launch_merge((const llampc_plan_out*)d_all, comm->world, nan_policy == LLAMPC_NAN_FIRST,
                       (llampc_plan_out*)d_merged, (hipStream_t)stream));
  return LLAMPC_OK;
}

}  // extern "C"

extern "C" {

int llampc_mailbox_create(int32_t world, int32_t rank, int32_t device, llampc_mailbox** out) {
  if (!out || world < 1 || world > kPeerMax || rank < 0 || rank >= world)
    return fail(LLAMPC_E_ARG, "bad mailbox arguments (world=%d rank=%d, world 1..%d)", world, rank, kPeerMax);
  DeviceGuard g(device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", device);
  auto* mb = new llampc_mailbox();
  mb->world = world;
  mb->rank = rank;
  mb->device = device;
  const size_t bytes = (size_t)2 * world * kRecWords * sizeof(uint64_t);
  hipError_t e = hipExtMallocWithFlags((void**)&mb->own, bytes, hipDeviceMallocUncached);
  if (e == hipSuccess) e = hipMemset(mb->own, 0, bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    if (mb->own) (void)hipFree(mb->own);
    delete mb;
    return fail(LLAMPC_E_HIP, "mailbox allocation: %s", hipGetErrorString(e));
  }
  e = hipMalloc((void**)&mb->d_box, kPeerMax * sizeof(uint64_t*));
  if (e != hipSuccess) {
    (void)hipFree(mb->own);
    delete mb;
    return fail(LLAMPC_E_HIP, "mailbox table allocation: %s", hipGetErrorString(e));
  }
  mb->box[rank] = mb->own;
  *out = mb;
  return LLAMPC_OK;
}

int llampc_mailbox_ipc_handle(llampc_mailbox* mb, void* handle) {
  if (!mb || !handle) return fail(LLAMPC_E_ARG, "null mailbox/handle");
  DeviceGuard g(mb->device);
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, mb->own));
  memcpy(handle, &h, sizeof(h));
  return LLAMPC_OK;
}

int llampc_mailbox_open_peer(llampc_mailbox* mb, int32_t peer, const void* handle) {
  if (!mb || !handle || peer < 0 || peer >= mb->world || peer == mb->rank || mb->box[peer])
    return fail(LLAMPC_E_ARG, "bad peer %d (world %d, rank %d, or already open)", mb ? peer : -1,
                mb ? mb->world : 0, mb ? mb->rank : 0);
  DeviceGuard g(mb->device);
  std::lock_guard<std::mutex> lm(mb->mu);
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  mb->box[peer] = (uint64_t*)p;
  mb->opened[peer] = true;
  mb->box_synced = false;
  return LLAMPC_OK;
}

int llampc_mailbox_link(llampc_mailbox* mb, int32_t peer, const llampc_mailbox* other) {
  if (!mb || !other || peer < 0 || peer >= mb->world || peer == mb->rank || mb->box[peer] ||
      other->world != mb->world || other->rank != peer || other->device != mb->device)
    return fail(LLAMPC_E_ARG, "bad mailbox link (peer %d)", peer);
  std::lock_guard<std::mutex> lm(mb->mu);
  mb->box[peer] = other->own;
  mb->box_synced = false;
  return LLAMPC_OK;
}

int llampc_mailbox_set_bound(llampc_mailbox* mb, double seconds) {
  if (!mb || !(seconds > 0) || seconds > 1e6) return fail(LLAMPC_E_ARG, "bad poll bound");
  mb->bound = (uint64_t)(seconds * 1e8);
  return LLAMPC_OK;
}

int llampc_exchange_peer(llampc_mailbox* mb, const void* d_local, void* d_merged, int32_t nan_policy,
                         void* stream) {
  if (!mb || !d_local || !d_merged) return fail(LLAMPC_E_ARG, "bad exchange arguments");
  for (int g = 0; g < mb->world; ++g)
    if (!mb->box[g]) return fail(LLAMPC_E_STATE, "mailbox of peer %d not open", g);
  DeviceGuard g(mb->device);
  if (!g.ok) return fail(LLAMPC_E_HIP, "hipSetDevice(%d) failed", mb->device);
  std::lock_guard<std::mutex> lm(mb->mu);
  const uint32_t seq = next_seq(mb->seq);
  PeerLaunch a{};
  a.local = (const llampc_plan_out*)d_local;
  for (int r = 0; r < mb->world; ++r) a.box[r] = mb->box[r];
  a.merged = (llampc_plan_out*)d_merged;
  a.bound = mb->bound;
  a.G = mb->world;
  a.rank = mb->rank;
  a.nan_first = nan_policy == LLAMPC_NAN_FIRST;
  a.seq = seq;
  HIP_TRY(launch_peer_exchange(a, (hipStream_t)stream));
  mb->seq = seq;
  return LLAMPC_OK;
}

int llampc_plan_exchange(llampc_bank* b, const llampc_plan_in* in, void* d_local, void* d_merged,
                         llampc_mailbox* mb, void* stream) {
  if (!b || !d_local || !d_merged || !mb) return fail(LLAMPC_E_ARG, "bank/d_local/d_merged/mailbox is NULL");
  if (mb->device != b->device) return fail(LLAMPC_E_ARG, "mailbox on device %d, bank on %d", mb->device, b->device);
  for (int g = 0; g < mb->world; ++g)
    if (!mb->box[g]) return fail(LLAMPC_E_STATE, "mailbox of peer %d not open", g);
  int rc = check_plan_in(b, in);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async tick is outstanding: call llampc_plan_wait");
  DeviceGuard g(b->device);
  hipStream_t s = pick_stream(b, stream);
  std::unique_lock<std::mutex> lm(mb->mu);
  if (!mb->box_synced) {                 // the peers are open: publish the table once
    HIP_TRY(hipMemcpy(mb->d_box, mb->box, kPeerMax * sizeof(uint64_t*), hipMemcpyHostToDevice));
    mb->box_synced = true;
  }
  const bool split = getenv("LLAMPC_PEER_SPLIT") != nullptr;   // A/B: separate kernel
  const bool fusable = !in->do_lookahead || (in->integrator == LLAMPC_RK4 && in->xref_mode == LLAMPC_XREF_GIVEN);
  if (!split && fusable && mb->world <= kPeerFuseMax)
    return plan_launch(b, *in, (llampc_plan_out*)d_local, nullptr, nullptr, nullptr, s, nullptr, 0, nullptr,
                       mb, (llampc_plan_out*)d_merged);
  rc = plan_launch(b, *in, (llampc_plan_out*)d_local, nullptr, nullptr, nullptr, s);
  if (rc) return rc;
  lm.unlock();                           // llampc_exchange_peer takes it
  return llampc_exchange_peer(mb, d_local, d_merged, in->nan_policy, s);
}

int llampc_mailbox_destroy(llampc_mailbox* mb) {
  if (!mb) return LLAMPC_OK;
  DeviceGuard g(mb->device);
  (void)hipDeviceSynchronize();
  for (int r = 0; r < mb->world; ++r)
    if (mb->opened[r]) (void)hipIpcCloseMemHandle(mb->box[r]);
  if (mb->own) (void)hipFree(mb->own);
  if (mb->d_box) (void)hipFree(mb->d_box);
  delete mb;
  return LLAMPC_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// Controller tick (ctl.hip): the control loop body rt.py:278-366 as ONE launch per step, the
// controller state resident on the device between steps.
// ------------------------------------------------------------------------------------
static_assert(sizeof(llampc_nlp_cfg) == 16 + 8 + 16 + 8 + 8 + sizeof(llampc_cost) + 32, "llampc_nlp_cfg layout");
static_assert(sizeof(llampc_ctl_cfg) == 280, "llampc_ctl_cfg layout (llampc/_native.py CtlCfg)");
static_assert(sizeof(llampc_ctl_out) == sizeof(llampc_plan_out) + 56 + 16 * LLAMPC_HMAX, "llampc_ctl_out layout");

struct llampc_ctl {
  llampc_bank* b = nullptr;
  llampc_ctl_cfg cfg{};
  bool no_stage = false;                 // LLAMPC_CTL_NO_STAGE=1: unstaged look-ahead inputs (A/B)
  // the state's projidx / mu-hat as the last record left them (the look-ahead prologue's
  // projection and mu bracket come as kernel arguments); hint_ok = false after a failed wait:
  // the next tick reads them from the device first
  bool hint_ok = true;
  int32_t hint_p0 = 0;
  double hint_mu = std::nan("");
  CtlState* d_st = nullptr;
  double* d_pts = nullptr;               // points [2][np] | prefix [np - 1]
  int32_t np = 0;
  llampc_ctl_out* h_out = nullptr;       // pinned, coherent; d_out is its device alias
  llampc_ctl_out* d_out = nullptr;
  uint64_t* h_tag = nullptr;             // completion tag (pinned), d_tag its alias
  uint64_t* d_tag = nullptr;
  uint64_t hseq = 0;
  uint64_t* d_sel_tag = nullptr;         // [kCtlSlotsMax]
  uint64_t* d_slot_tag = nullptr;        // [kCtlSlotsMax][4]
  unsigned* d_tickets = nullptr;         // [1]
  double* d_dbg = nullptr;               // xref [2][H+1] | U [C][H][2] (debug_inputs)
  double* d_znoise = nullptr;            // [2][C H][2] the candidates' variates (CtlLaunch.znoise)
  uint64_t* d_ztag = nullptr;            // [2]
  uint32_t seq = 0;
  int64_t t = 0;
  bool pending = false;
  uint64_t pend_seq = 0;
  // sharded (llampc_ctl_set_exchange): the peers' mailboxes and the replicated global table
  llampc_mailbox* mb = nullptr;
  double* d_gparams = nullptr;           // [6][n_global]
  int64_t n_global = 0;
  // sharded over a gather transport (llampc_ctl_set_gather; CtlLaunch.px_phase): RCCL, or the
  // caller carries the records (xg_comm null) between the two launches of a full-window tick
  int32_t xg_world = 0, xg_rank = 0;
  llampc_comm* xg_comm = nullptr;
  uint64_t* d_xsend = nullptr;           // [nw] this shard's record (the first launch writes it)
  uint64_t* d_xgath = nullptr;           // [G][nw] the gathered records
  uint64_t* h_xstage = nullptr;          // pinned [G][nw] (the host transport's staging)
  uint32_t xg_seq = 0;
  bool xg_wait = false;                  // the host transport's second launch awaits llampc_ctl_resume
  bool xg_read = false;                  //   and this rank's record has been read
  int32_t xg_nw = 0;
  // armed launches (llampc_ctl_set_prelaunch): the next tick's launch is enqueued behind this
  // one and waits for x_t on the doorbell (CtlLaunch.door)
  bool prelaunch = false;
  bool armed = false;
  bool arm_next = false;                 // arm the next tick in llampc_ctl_wait (before its spin)
  uint64_t* h_door = nullptr;            // pinned: kCtlDoorWords tagged words (CtlLaunch.door)
  uint64_t* d_door = nullptr;            //   its device alias
  uint64_t* d_door_dev = nullptr;        // block 0's device copy (CtlLaunch.door_dev)
  // the speculative look-ahead of armed ticks (CtlLaunch.n_spec; LLAMPC_CTL_NO_SPEC=1: never)
  bool no_spec = false;
  // spec models per armed tick: 32 (LLAMPC_CTL_SPEC_N, <= kCtlSpecMax).  The paced two-track step
  // measured p50 56.1 / 55.9 us with 32, 57.8 / 58.0 with 64, 57.9 with 96 (profiles/r05/specn/):
  // fewer busy CUs outweigh the 2-3 % more misses (profiles/r05/spec_topm.json)
  int32_t spec_cap = 32;
  int32_t spec_nb = 0;                   // look-back blocks the lists were sized for
  double* d_spec_val = nullptr;          // [spec_nb][kCtlSpecMax]
  int64_t* d_spec_idx = nullptr;
  uint64_t* d_spec_tag = nullptr;        // [kCtlSpecMax]
  uint64_t* d_spec_res = nullptr;        // [kCtlSpecMax][4]
  uint64_t* d_xref_tag = nullptr;        // [2 (HMAX + 1)][2]
  uint32_t door_ctr = 0;                 // never reused: a cancelled word cannot match a later launch
  uint64_t dev_ticks = 0;                // the last completed tick's device time (llampc_ctl_device_us)
  std::chrono::steady_clock::time_point arm_t{};
  struct Prep {                          // a prepared tick: its launch and what it commits
    CtlLaunch L{};
    int lpm = 4;
    size_t lds = 0;
    uint64_t hs = 0;
    uint32_t seq = 0, px_seq = 0;
    int64_t t = 0;
    bool do_lb = false;
    int32_t count = 0;
  } arm, xg_second;                      // xg_second: the host transport's pending second launch
  std::mutex mu;
};

// An armed launch waits at most kArmBound for its doorbell; the host fires it only while it is
// younger than kArmFresh (else cancels it and launches the tick normally), so the launch
// cannot expire between the host's check and its store short of a ~1 s stall of that thread.
constexpr double kArmBoundS = 2.0;
constexpr double kArmFreshS = 0.5;

static void ctl_cancel(llampc_ctl* c) {
  if (!c || !c->armed) return;
  __atomic_store_n(&c->h_door[kCtlDoorWords - 1], ((uint64_t)c->arm.L.door_seq << 32) | kCtlDoorCancel,
                   __ATOMIC_RELEASE);
  // its completion number is spent: a launch that expired before the cancel has stored it
  // (with kCtlTagExpired) into the tag the next tick's wait reads.  So is its selection tag: the
  // cancelled launch may have published spec_tag words tagged arm.seq before its doorbell, which
  // a relaunch with the same tag would read as its own
  c->hseq = c->arm.hs;
  c->seq = c->arm.seq;
  c->armed = false;
  if (c->b && c->b->armed == c) c->b->armed = nullptr;
}

static void bank_disarm(llampc_bank* b) {
  if (b && b->armed) ctl_cancel(b->armed);
}

// Controllers whose tick was rung and whose next launch is still to be armed (arm_next).  The
// first llampc_ctl_wait of a step arms them ALL before it spins: with two tracks (tick_async on
// both, then wait on both) the second controller's launch call would otherwise sit between the
// first's result and its own (~5 us on the two-track step).  The arming pass holds g_arm_mu
// throughout and only try-locks the controllers it visits; llampc_ctl_destroy removes its
// controller under g_arm_mu before anything is freed, so the pass never holds a controller that
// is being destroyed.
static std::mutex g_arm_mu;
static std::vector<llampc_ctl*> g_arm_list;
static void arm_list_add(llampc_ctl* c) {
  std::lock_guard<std::mutex> g(g_arm_mu);
  g_arm_list.push_back(c);
}
static void arm_list_remove(llampc_ctl* c) {
  std::lock_guard<std::mutex> g(g_arm_mu);
  g_arm_list.erase(std::remove(g_arm_list.begin(), g_arm_list.end(), c), g_arm_list.end());
}

// A failed controller tick (a wait that gave up, or a completion that never arrived): once the
// stream has drained, the look-back ticket is zeroed so the next launch's ticket_last counts
// from 0.  The tick still consumed its step on the device (the window slot, the tick number);
// the Python controller refuses further ticks until it is rebuilt (LLAMPC.tick).
static int ctl_recover(llampc_ctl* c) {
  ctl_cancel(c);                         // an armed launch behind the failed one exits at once
  HIP_TRY(hipStreamSynchronize(c->b->stream));
  HIP_TRY(hipMemsetAsync(c->d_tickets, 0, 2 * sizeof(unsigned), c->b->stream));
  HIP_TRY(hipStreamSynchronize(c->b->stream));
  return LLAMPC_OK;
}

extern "C" {

int llampc_ctl_destroy(llampc_ctl* c) {
  if (!c) return LLAMPC_OK;
  arm_list_remove(c);
  ctl_cancel(c);
  {
    DeviceGuard g(c->b ? c->b->device : 0);
    if (c->b && c->b->stream) (void)hipStreamSynchronize(c->b->stream);
    void* d[] = {c->d_st, c->d_pts, c->d_sel_tag, c->d_slot_tag, c->d_tickets, c->d_dbg, c->d_znoise, c->d_ztag,
                 c->d_gparams, c->d_door_dev, c->d_spec_val, c->d_spec_idx, c->d_spec_tag, c->d_spec_res,
                 c->d_xref_tag};
    for (void* p : d)
      if (p) (void)hipFree(p);
    if (c->d_xsend) (void)hipFree(c->d_xsend);
    if (c->d_xgath) (void)hipFree(c->d_xgath);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->h_tag) (void)hipHostFree(c->h_tag);
    if (c->h_door) (void)hipHostFree(c->h_door);
    if (c->h_xstage) (void)hipHostFree(c->h_xstage);
  }
  delete c;
  return LLAMPC_OK;
}

int llampc_ctl_create(llampc_bank* b, const llampc_ctl_cfg* cfg, const double* points, int32_t np,
                      const double* prefix, llampc_ctl** out) {
  if (!out) return fail(LLAMPC_E_ARG, "out is NULL");
  *out = nullptr;
  if (!b || !cfg || !points || !prefix) return fail(LLAMPC_E_ARG, "NULL argument");
  const llampc_ctl_cfg& k = *cfg;
  if (k.C < 1 || k.H < 1 || k.H > LLAMPC_HMAX || k.K < 1 || k.K > LLAMPC_KMAX)
    return fail(LLAMPC_E_ARG, "C=%d H=%d (1..%d) K=%d (1..%d)", k.C, k.H, LLAMPC_HMAX, k.K, LLAMPC_KMAX);
  if (k.S < 1 || k.S > kCtlSMax) return fail(LLAMPC_E_ARG, "S=%d outside [1, %d]", k.S, kCtlSMax);
  if (!(k.Ts > 0) || !std::isfinite(k.Ts)) return fail(LLAMPC_E_ARG, "Ts must be finite > 0");
  if (np < 2) return fail(LLAMPC_E_ARG, "np=%d < 2", np);
  if (k.nan_policy != LLAMPC_NAN_FIRST && k.nan_policy != LLAMPC_NAN_IGNORE) return fail(LLAMPC_E_ARG, "nan_policy");
  if (!b->d_rl) return fail(LLAMPC_E_STATE, "the controller needs the bank's raceline (llampc_bank_set_raceline)");
  const int R = lookback_r(b->n, k.K);
  const int nb_lb = lookback_blocks_r(b->n, R);
  size_t poll_off = 0;
  const size_t lds = ctl_lds_bytes(k.H, k.C, b->rl_n, nb_lb, k.K, &poll_off);
  if (lds > 160 * 1024)
    return fail(LLAMPC_E_ARG, "controller tick needs %zu B of LDS (> 160 KiB): C*H=%d too large for this track", lds,
                k.C * k.H);
  DeviceGuard g(b->device);
  auto* c = new llampc_ctl();
  c->b = b;
  c->cfg = k;
  if (const char* e = std::getenv("LLAMPC_CTL_NO_STAGE")) c->no_stage = e[0] == '1';
  c->np = np;
  auto cleanup = [&](int code) {
    llampc_ctl_destroy(c);
    return code;
  };
  int rc;
  if ((rc = dev_alloc(&c->d_st, 1)) || (rc = dev_alloc(&c->d_pts, 3 * (size_t)np - 1)) ||
      (rc = dev_alloc(&c->d_sel_tag, kCtlSlotsMax)) || (rc = dev_alloc(&c->d_slot_tag, 4 * (size_t)kCtlSlotsMax)) ||
      (rc = dev_alloc(&c->d_tickets, 2)) || (rc = dev_alloc(&c->d_znoise, 4 * (size_t)k.C * k.H)) ||
      (rc = dev_alloc(&c->d_ztag, 2)) || (rc = dev_alloc(&c->d_door_dev, 16)) ||
      (rc = dev_alloc(&c->d_spec_val, (size_t)nb_lb * kCtlSpecMax)) ||
      (rc = dev_alloc(&c->d_spec_idx, (size_t)nb_lb * kCtlSpecMax)) || (rc = dev_alloc(&c->d_spec_tag, kCtlSpecMax)) ||
      (rc = dev_alloc(&c->d_spec_res, 4 * (size_t)kCtlSpecMax)) || (rc = dev_alloc(&c->d_xref_tag, 4 * (size_t)(LLAMPC_HMAX + 1))))
    return cleanup(rc);
  c->spec_nb = nb_lb;
  if (const char* e = std::getenv("LLAMPC_CTL_NO_SPEC")) c->no_spec = e[0] == '1';
  if (const char* e = std::getenv("LLAMPC_CTL_SPEC_N")) c->spec_cap = std::max(1, std::min(kCtlSpecMax, std::atoi(e)));
  if (k.debug_inputs && (rc = dev_alloc(&c->d_dbg, 2 * (size_t)(k.H + 1) + 2 * (size_t)k.C * k.H))) return cleanup(rc);
  if (hipHostMalloc(reinterpret_cast<void**>(&c->h_out), sizeof(llampc_ctl_out),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_tag), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_door), 16 * sizeof(uint64_t),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return cleanup(fail(LLAMPC_E_OOM, "hipHostMalloc(controller record) failed"));
  *c->h_tag = 0;
  for (int j = 0; j < 16; ++j) c->h_door[j] = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_out), c->h_out, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_tag), c->h_tag, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->d_door), c->h_door, 0) != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "hipHostGetDevicePointer(controller record) failed"));
  CtlState st{};
  st.mu_pred = std::nan("");
  st.current_model = 0;                  // rt.py:264: the nominal model's index
  if (hipMemcpy(c->d_st, &st, sizeof st, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_pts, points, 2 * (size_t)np * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_pts + 2 * (size_t)np, prefix, ((size_t)np - 1) * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_sel_tag, 0, kCtlSlotsMax * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_slot_tag, 0, 4 * kCtlSlotsMax * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_tickets, 0, 2 * sizeof(unsigned)) != hipSuccess ||
      hipMemset(c->d_spec_tag, 0, kCtlSpecMax * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_spec_res, 0, 4 * kCtlSpecMax * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_xref_tag, 0, 4 * (LLAMPC_HMAX + 1) * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_ztag, 0, 2 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(c->d_door_dev, 0, 16 * sizeof(uint64_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "controller upload failed"));
  *out = c;
  return LLAMPC_OK;
}

}  // extern "C"

// The launch of tick c->t (x_t null: armed — the doorbell carries x_t) and what it commits
// (ctl_commit), from the host's copy of the controller and bank state.
static int ctl_prepare(llampc_ctl* c, const double* x_t, llampc_ctl::Prep& P) {
  llampc_bank* b = c->b;
  const llampc_ctl_cfg& k = c->cfg;
  const int64_t t = c->t;
  const int32_t W = b->W;
  const bool do_lb = t >= 2;             // rt.py:347 (the transition idt -> idt+1 from idt >= 1)
  const bool warm = t <= W;              // rt.py:300-301
  int32_t count = b->count;
  if (do_lb) count = std::min(count + 1, W);
  const bool full = do_lb && count >= W;
  if (!warm && !full)
    return fail(LLAMPC_E_STATE, "tick %lld: the look-back window is not full after the warm-up (was the bank reset?)",
                (long long)t);
  CtlLaunch L{};
  const int R = lookback_r(b->n, k.K);
  // look-back (rt.py:347-366 on the bank's ring)
  L.lb.params = b->d_params;
  L.lb.n = b->n;
  L.lb.goff = b->goff;
  L.lb.veh = b->veh;
  L.lb.x_prev = c->d_st->x_prev;
  L.lb.u_prev = c->d_st->u_prev;
  L.lb.Ts = k.Ts;
  L.lb.ring = b->d_ring;
  L.lb.W = W;
  L.lb.slot = b->slot;
  L.lb.full = full;
  L.lb.K = k.K;
  L.lb.nan_first = k.nan_policy == LLAMPC_NAN_FIRST;
  L.lb.R = R;
  L.lb.wm_keep = 0;
  L.lb.wm_buf = b->d_wmean;
  L.lb.am_val = b->d_am_val;
  L.lb.am_idx = b->d_am_idx;
  L.lb.tk_val = b->d_tk_val;
  L.lb.tk_idx = b->d_tk_idx;
  // look-ahead constants (RK4 on the bank's vehicle, the NLP objective)
  L.la.params = b->d_params;
  L.la.n = b->n;
  L.la.goff = b->goff;
  L.la.veh = integrator_veh(b->veh, LLAMPC_RK4);
  L.la.C = k.C;
  L.la.H = k.H;
  L.la.integrator = LLAMPC_RK4;
  L.la.Ts = k.Ts;
  L.la.cost = make_cost(k.cost, k.Ts);
  L.la.xref_mode = LLAMPC_XREF_GIVEN;
  {
    const size_t m = (size_t)b->rl_n - 1;
    L.la.rl.knots = b->d_rl;
    L.la.rl.xy = b->d_rl + b->rl_n;
    L.la.rl.speed = L.la.rl.xy + 8 * m;
    L.la.rl.mus = L.la.rl.speed + 4 * m * b->rl_M;
    L.la.rl.n = b->rl_n;
    L.la.rl.M = b->rl_M;
    L.la.rl.hmin = b->rl_hmin;
    L.la.rl.vmax = b->rl_vmax;
    L.la.rl.wcap = b->rl_n - 1;
  }
  // lb_final's view
  L.fin.out = &c->d_out->plan;
  L.fin.do_lb = do_lb;
  L.fin.do_la = 1;
  L.fin.full = full;
  L.fin.window_count = do_lb ? count : b->count;
  L.fin.K = k.K;
  L.fin.nan_first = k.nan_policy == LLAMPC_NAN_FIRST;
  L.fin.nb_lb = do_lb ? lookback_blocks_r(b->n, R) : 1;
  L.fin.C = k.C;
  L.fin.n = b->n;
  L.fin.goff = b->goff;
  L.fin.params = b->d_params;
  L.fin.am_val = b->d_am_val;
  L.fin.am_idx = b->d_am_idx;
  L.fin.tk_val = b->d_tk_val;
  L.fin.tk_idx = b->d_tk_idx;
  // controller
  const uint64_t hs = c->hseq + 1;
  const uint32_t seq = next_seq(c->seq);
  L.st = c->d_st;
  L.out = c->d_out;
  L.host_tag = c->d_tag;
  L.host_seq = hs;
  L.sel_tag = c->d_sel_tag;
  L.slot_tag = c->d_slot_tag;
  L.tickets = c->d_tickets;
  L.dbg = c->d_dbg;
  L.znoise = c->d_znoise;
  L.ztag = c->d_ztag;
  L.pts = c->d_pts;
  L.prefix = c->d_pts + 2 * (size_t)c->np;
  L.tick = (uint64_t)t;
  L.seed = k.seed;
  for (int j = 0; j < 6; ++j) {
    L.x_t[j] = x_t ? x_t[j] : 0.0;      // armed (x_t null): the doorbell carries it
    L.nominal[j] = k.nominal[j];
  }
  const double sqrt3 = std::sqrt(3.0);
  for (int j = 0; j < 2; ++j) {
    L.nscale[j] = sqrt3 * k.sigma[j];    // sqrt(3) sigma_j, one rounding (ctl.hpp ctl_cand_one)
    L.rate[j] = k.cost.rate_max[j] < 0 ? -1.0 : k.cost.rate_max[j] * k.Ts;
    L.umin[j] = k.cost.umin[j];
    L.umax[j] = k.cost.umax[j];
  }
  L.mu_fixed = 1.0;                      // ConstantSpeed's defaults (rt.py:282)
  L.scale_fixed = 1.0;
  L.v_factor = k.v_factor;
  L.mu_init = k.mu_init;
  L.seq = seq;
  {
    const uint64_t units = (poll_bound_ticks(b->n, k.C, k.H) + 0xFFFF) >> 16;
    L.poll = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(units, 1), UINT32_MAX);
  }
  L.np = c->np;
  L.lap_projidx = k.lap_projidx;
  L.do_lb = do_lb;
  L.warm = warm;
  L.use_mu = t > W + 1;                  // rt.py:278
  L.door_dev = c->d_door_dev;            // every launch: its x_t time (kCtlTimeWord)
  if (!x_t) {                            // armed: the launch reads projidx / mu-hat from the state
    L.door = c->d_door;
    c->door_ctr = c->door_ctr == 0xFFFFFFFFu ? 1u : c->door_ctr + 1u;
    L.door_seq = c->door_ctr;
    L.door_bound = (uint32_t)(kArmBoundS * 1e8 / 65536.0) + 1;
  } else if (!c->hint_ok) {              // after a failed wait: the state itself
    CtlState hs{};
    HIP_TRY(hipStreamSynchronize(b->stream));
    HIP_TRY(hipMemcpy(&hs, c->d_st, sizeof hs, hipMemcpyDeviceToHost));
    c->hint_p0 = hs.projidx;
    c->hint_mu = hs.mu_pred;
    c->hint_ok = true;
  }
  if (x_t) {
    L.p0_walk = c->hint_p0;
    L.br_walk = mu_bracket(b->rl_mus.data(), b->rl_M, L.use_mu ? c->hint_mu : L.mu_fixed);   // rt.py:278-282
  }
  L.full = full;
  L.nslots = warm ? 1 : k.K + 1;
  L.G = lookahead_group(k.C);
  L.cpl = (k.C + L.G - 1) / L.G;
  const int lpm = 4 * L.G <= kBlock ? 4 : (2 * L.G <= kBlock ? 2 : 1);
  L.mpb = kBlock / (L.G * lpm);
  L.S = k.S;
  L.K = k.K;
  L.nb_lb = L.fin.nb_lb;
  L.nb_la = (L.nslots + L.mpb - 1) / L.mpb;
  // sharded: the exchange runs on every tick whose window is full (the same ticks on every
  // rank); the selection is global, the look-ahead reads the replicated global table
  L.sel_goff = b->goff;
  uint32_t px_seq = 0;
  if (c->mb || c->xg_world) {            // (the caller holds mb->mu)
    L.la.params = c->d_gparams;
    L.la.n = c->n_global;
    L.la.goff = 0;
    L.sel_goff = 0;
  }
  if (c->mb) {
    llampc_mailbox* mb = c->mb;
    if (!mb->box_synced) {
      HIP_TRY(hipMemcpy(mb->d_box, mb->box, kPeerMax * sizeof(uint64_t*), hipMemcpyHostToDevice));
      mb->box_synced = true;
    }
    if (full) {
      px_seq = next_seq(mb->seq);
      L.px_box = mb->d_box;
      L.px_G = mb->world;
      L.px_rank = mb->rank;
      L.px_seq = px_seq;
      L.px_bound = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((mb->bound + 0xFFFF) >> 16, 1), UINT32_MAX);
      L.poll = std::max(L.poll, L.px_bound);   // the look-ahead blocks wait for the merged selection
    }
  } else if (c->xg_world && full) {      // gather transport: two launches (CtlLaunch.px_phase)
    px_seq = next_seq(c->xg_seq);
    L.px_G = c->xg_world;
    L.px_rank = c->xg_rank;
    L.px_seq = px_seq;
    L.px_phase = 1;
    L.px_send = c->d_xsend;
    L.px_gath = c->d_xgath;
    L.px_bound = 16;                     // ~10 ms: the records are there when the launch starts
  }
  // the look-ahead blocks stage every (candidate, step)'s input terms when they fit in LDS
  // (CtlLaunch.s4; LLAMPC_CTL_NO_STAGE=1 at create: never, for A/B runs)
  size_t poll_s4 = 0;
  const size_t lds_s4 = ctl_lds_bytes(k.H, k.C, b->rl_n, L.nb_lb, k.K, &poll_s4, true, L.px_G);
  L.s4 = (!c->no_stage && lds_s4 <= 160 * 1024) ? 1 : 0;
  size_t lds = L.s4 ? lds_s4 : ctl_lds_bytes(k.H, k.C, b->rl_n, L.nb_lb, k.K, &L.poll_off, false, L.px_G);
  if (lds > 160 * 1024) return fail(LLAMPC_E_ARG, "controller tick needs %zu B of LDS (> 160 KiB)", lds);
  if (L.s4) L.poll_off = poll_s4;
  // the speculative look-ahead (CtlLaunch.n_spec): armed ticks past the warm-up whose rollouts
  // are one model per block in fused quads with diagonal Q / P (the spec blocks' layout)
  {
    const llampc_cost& cq = k.cost;
    const bool diag = cq.Q[1] == 0.0 && cq.Q[2] == 0.0 && cq.P[1] == 0.0 && cq.P[2] == 0.0;
    // sharded over the peer mailboxes: the ranks' lists are exchanged too (ctl.hip
    // ctl_spec_exchange), in the slot after the selection record's words
    // the armed footprint: every block of an armed launch holds a CU from the end of the tick
    // before to its doorbell, and all launches of the banks ticked together
    // (llampc_bank_set_concurrency) must be resident at once — the exchange's peers and the
    // tick's own look-back wait on each other — so the spec blocks take what is left of the
    // banks' share of the CUs (INTEGRATION.md "What armed launches cost")
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b->device) != hipSuccess || cus < 1) cus = 256;
    const int room = cus / std::max(1, b->share) - (L.nb_lb + L.nb_la);
    const int ns = (int)std::min<int64_t>(std::min<int64_t>(c->spec_cap, room), c->mb ? c->n_global : b->n);
    const int spec_off = ctl_rec_words(k.K);
    const bool px_fits = !c->mb || (L.px_G && spec_off + 4 * ns <= kRecWords);
    if (!x_t && !c->no_spec && !warm && full && R == 1 && L.s4 && lpm == 4 && L.cpl == 1 && L.G == k.C && diag &&
        !c->xg_world && px_fits && ns >= 4 && L.nb_lb <= c->spec_nb) {
      size_t poll_sp = 0;
      const size_t lds_sp = ctl_lds_bytes(k.H, k.C, b->rl_n, L.nb_lb, k.K, &poll_sp, true, L.px_G, ns);
      if (lds_sp <= 160 * 1024) {
        L.px_spec_off = spec_off;
        L.px_spec_wait = 20000;           // 200 us: the ranks arm within microseconds of each other
        L.n_spec = ns;
        L.spec_val = c->d_spec_val;
        L.spec_idx = c->d_spec_idx;
        L.spec_tag = c->d_spec_tag;
        L.spec_res = c->d_spec_res;
        L.xref_tag = c->d_xref_tag;
        L.poll_off = poll_sp;
        lds = lds_sp;
      }
    }
  }
  lds = std::max<size_t>(lds, 82 * 1024); // one block per CU, as the plan launch (sc1 hand-offs)
  P.L = L;
  P.lpm = lpm;
  P.lds = lds;
  P.hs = hs;
  P.seq = seq;
  P.px_seq = px_seq;
  P.t = t;
  P.do_lb = do_lb;
  P.count = count;
  return LLAMPC_OK;
}

// The host state after tick P.t was enqueued (or its armed launch fired).
static void ctl_commit(llampc_ctl* c, const llampc_ctl::Prep& P) {
  llampc_bank* b = c->b;
  c->hseq = P.hs;
  c->seq = P.seq;
  if (P.L.px_G) {                        // committed after the launch was enqueued (next_seq)
    if (c->mb) c->mb->seq = P.px_seq;
    else c->xg_seq = P.px_seq;
  }
  c->t = P.t + 1;
  c->pending = true;
  c->pend_seq = P.hs;
  b->launches++;
  if (P.do_lb) {
    b->slot = (b->slot + 1) % b->W;
    b->count = P.count;
  }
}

// Enqueues tick c->t's launch armed (llampc_ctl_set_prelaunch): it runs behind the tick in
// flight and waits for the doorbell.  The caller holds c->mu, c->b->mu and, with a peer
// exchange, c->mb->mu.  With the peer exchange the armed launch takes the mailbox's next tick
// number (the exchange runs after its doorbell, inside it); the number is committed only when
// the doorbell fires (ctl_commit), so a cancelled armed launch — which exits before the doorbell,
// never pushing — leaves the sequence to its relaunch, and the ranks' sequences stay in step
// whichever of them armed, fired or relaunched.  Not with a gather transport (two launches).
static int ctl_arm(llampc_ctl* c) {
  if (c->armed || c->xg_world) return LLAMPC_OK;
  if (!c->b->own_stream || !c->b->dedicated)   // the stream changed since set_prelaunch
    return fail(LLAMPC_E_STATE, "an armed launch needs the bank's own dedicated-queue stream");
  llampc_ctl::Prep P;
  int rc = ctl_prepare(c, nullptr, P);
  if (rc) return rc;
  HIP_TRY(launch_ctl(P.L, P.lpm, P.lds, c->b->stream));
  c->arm = P;
  c->armed = true;
  c->arm_t = std::chrono::steady_clock::now();
  c->b->armed = c;
  return LLAMPC_OK;
}

extern "C" {

int llampc_ctl_tick_async(llampc_ctl* c, const double* x_t) {
  if (!c || !x_t) return fail(LLAMPC_E_ARG, "controller/x_t is NULL");
  std::lock_guard<std::mutex> lc(c->mu);
  if (c->pending) return fail(LLAMPC_E_STATE, "a controller tick is outstanding: call llampc_ctl_wait");
  llampc_bank* b = c->b;
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async plan tick is outstanding on the bank");
  DeviceGuard g(b->device);
  std::unique_lock<std::mutex> lm;
  if (c->mb) lm = std::unique_lock<std::mutex>(c->mb->mu);
  if (c->armed) {
    const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - c->arm_t).count();
    // (with a peer exchange the armed launch's tick number must still be the mailbox's next)
    const bool px_ok = !c->arm.L.px_G || !c->mb || c->arm.px_seq == next_seq(c->mb->seq);
    if (age < kArmFreshS && c->arm.t == c->t && px_ok) {
      // fire: every word tagged (block 0 polls until all carry the tag: no order needed)
      const uint64_t tg = (uint64_t)c->arm.L.door_seq << 32;
      for (int j = 0; j < 6; ++j) {
        uint64_t w;
        std::memcpy(&w, &x_t[j], 8);
        __atomic_store_n(&c->h_door[2 * j], tg | (w >> 32), __ATOMIC_RELAXED);
        __atomic_store_n(&c->h_door[2 * j + 1], tg | (w & 0xFFFFFFFFull), __ATOMIC_RELAXED);
      }
      __atomic_store_n(&c->h_door[kCtlDoorWords - 1], tg | kCtlDoorFire, __ATOMIC_RELEASE);
      c->armed = false;
      b->armed = nullptr;
      ctl_commit(c, c->arm);
      c->arm_next = c->prelaunch;
      if (c->arm_next) arm_list_add(c);
      return LLAMPC_OK;
    }
    ctl_cancel(c);                       // stale: this tick launches normally
  }
  llampc_ctl::Prep P;
  int rc = ctl_prepare(c, x_t, P);
  if (rc) return rc;
  if (P.L.px_phase == 1) {               // gather transport: the look-back launch, the gather, the rest
    llampc_ctl::Prep P2 = P;
    P2.L.px_phase = 2;
    P2.L.nb_lb = 1;                      // block 0 merges and completes
    llampc_ctl::Prep P1 = P;
    P1.L.nb_la = 0;                      // the look-back blocks alone
    P1.L.n_spec = 0;
    {
      TimedLaunch tl(b, 0, b->stream);
      HIP_TRY(launch_ctl(P1.L, P1.lpm, P1.lds, b->stream));
      if (c->xg_comm) {
        RCCL_TRY(rccl().all_gather(c->d_xsend, c->d_xgath, (size_t)c->xg_nw, ncclUint64, c->xg_comm->comm, b->stream));
        HIP_TRY(launch_ctl(P2.L, P2.lpm, P2.lds, b->stream));
      }
    }
    ctl_commit(c, P);
    if (!c->xg_comm) {                   // the caller carries the records (llampc_ctl_resume)
      c->xg_second = P2;
      c->xg_wait = true;
      c->xg_read = false;
      return LLAMPC_OK;
    }
    c->arm_next = c->prelaunch;
    if (c->arm_next) arm_list_add(c);
    return LLAMPC_OK;
  }
  {
    TimedLaunch tl(b, 0, b->stream);
    HIP_TRY(launch_ctl(P.L, P.lpm, P.lds, b->stream));
  }
  ctl_commit(c, P);
  c->arm_next = c->prelaunch;
  if (c->arm_next) arm_list_add(c);
  return LLAMPC_OK;
}

int llampc_ctl_wait(llampc_ctl* c, llampc_ctl_out* out) {
  if (!c || !out) return fail(LLAMPC_E_ARG, "controller/out is NULL");
  std::lock_guard<std::mutex> lc(c->mu);
  if (!c->pending) return fail(LLAMPC_E_STATE, "no controller tick outstanding");
  if (c->xg_wait) return fail(LLAMPC_E_STATE, "the tick's records are not gathered yet: call llampc_ctl_resume");
  c->pending = false;
  c->hint_ok = false;                    // until this tick's record is read
  DeviceGuard g(c->b->device);
  {
    // the next ticks' launches, armed behind the ones in flight — here rather than in
    // tick_async, so that several controllers' ticks (two tracks) are all rung before any
    // launch call, and for every rung controller at once (g_arm_list); the launch calls overlap
    // the device time.  Another controller is armed only if its locks are free (else its own
    // wait arms it).  A failed arm only turns prelaunch off.
    std::lock_guard<std::mutex> ga(g_arm_mu);
    std::vector<llampc_ctl*> keep;
    for (llampc_ctl* x : g_arm_list) {
      const bool self = x == c;
      if (!self && !x->mu.try_lock()) {
        keep.push_back(x);
        continue;
      }
      if (x->arm_next) {
        if (x->b->mu.try_lock()) {
          if (!x->mb || x->mb->mu.try_lock()) {
            x->arm_next = false;
            DeviceGuard gx(x->b->device);
            if (!x->b->async_pending && ctl_arm(x) != LLAMPC_OK) x->prelaunch = false;
            if (x->mb) x->mb->mu.unlock();
          } else {
            keep.push_back(x);
          }
          x->b->mu.unlock();
        } else {
          keep.push_back(x);
        }
      }
      if (!self) x->mu.unlock();
    }
    g_arm_list.swap(keep);
  }
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  uint64_t tag;
  while ((tag = __atomic_load_n(c->h_tag, __ATOMIC_ACQUIRE)) != c->pend_seq) {
    __builtin_ia32_pause();
    if (tag == (c->pend_seq | kCtlTagExpired)) {   // an armed launch that never saw its doorbell
      (void)ctl_recover(c);
      return fail(LLAMPC_E_DEVICE, "controller tick %llu: the armed launch expired before its doorbell",
                  (unsigned long long)c->pend_seq);
    }
    if ((++spins & 0xFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      ctl_cancel(c);
      HIP_TRY(hipStreamSynchronize(c->b->stream));
      if (__atomic_load_n(c->h_tag, __ATOMIC_ACQUIRE) == c->pend_seq) break;
      (void)ctl_recover(c);
      return fail(LLAMPC_E_DEVICE, "controller tick %llu: completion tag never arrived", (unsigned long long)c->pend_seq);
    }
  }
  std::memcpy(out, const_cast<const llampc_ctl_out*>(c->h_out), sizeof(llampc_ctl_out));
  c->dev_ticks = __atomic_load_n(c->h_tag + 1, __ATOMIC_RELAXED);
  if (out->plan.status) {
    (void)ctl_recover(c);
    return fail(LLAMPC_E_DEVICE, "controller tick record status %d (an in-launch wait timed out)", out->plan.status);
  }
  c->hint_p0 = out->projidx;             // the state this tick left (ctl_complete writes both)
  c->hint_mu = out->mu_pred;
  c->hint_ok = true;
  return LLAMPC_OK;
}

int llampc_ctl_device_us(llampc_ctl* c, double* us) {
  if (!c || !us) return fail(LLAMPC_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lc(c->mu);
  *us = c->dev_ticks ? (double)c->dev_ticks * 1e-2 : std::nan("");   // s_memrealtime: 100 MHz
  return LLAMPC_OK;
}

int llampc_ctl_set_prelaunch(llampc_ctl* c, int32_t on) {
  if (!c) return fail(LLAMPC_E_ARG, "controller is NULL");
  std::lock_guard<std::mutex> lc(c->mu);
  if (on && c->xg_world) return fail(LLAMPC_E_STATE, "prelaunch is not available with a gather transport");
  llampc_bank* b = c->b;
  std::lock_guard<std::mutex> lk(b->mu);
  DeviceGuard g(b->device);
  if (on) {
    if (!b->own_stream)
      return fail(LLAMPC_E_STATE, "prelaunch needs the bank's own stream (the bank launches on a caller's stream)");
    if (!b->dedicated) {                  // an armed launch must not sit on a shared hardware queue
      bank_disarm(b);
      if (int rc = bank_dedicate(b)) return rc;
    }
  }
  c->prelaunch = on != 0;
  c->arm_next = c->prelaunch && c->pending;   // a tick in flight: armed by its wait
  if (c->arm_next) arm_list_add(c);
  if (!c->prelaunch) {
    ctl_cancel(c);
    return LLAMPC_OK;
  }
  if (c->pending || b->async_pending) return LLAMPC_OK;
  bank_disarm(b);                         // another controller's launch on this bank
  std::unique_lock<std::mutex> lm;
  if (c->mb) lm = std::unique_lock<std::mutex>(c->mb->mu);
  return ctl_arm(c);
}

int llampc_ctl_tick(llampc_ctl* c, const double* x_t, llampc_ctl_out* out) {
  if (!out) return fail(LLAMPC_E_ARG, "out is NULL");
  int rc = llampc_ctl_tick_async(c, x_t);
  return rc ? rc : llampc_ctl_wait(c, out);
}

int llampc_ctl_reference(llampc_ctl* c, const double* x0, double v0, int32_t H, int32_t projidx, double curr_mu,
                         double scale, double* xref, int32_t* projidx_out, double* vr) {
  if (!c || !x0 || !xref) return fail(LLAMPC_E_ARG, "NULL argument");
  if (H < 1 || H > LLAMPC_HMAX) return fail(LLAMPC_E_ARG, "H=%d outside [1, %d]", H, LLAMPC_HMAX);
  if (projidx < 0 || projidx > c->np - 2) return fail(LLAMPC_E_ARG, "projidx=%d outside [0, %d]", projidx, c->np - 2);
  std::lock_guard<std::mutex> lc(c->mu);
  llampc_bank* b = c->b;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  DeviceGuard g(b->device);
  const size_t n = 2 * (size_t)(H + 1) + 2;
  double* d = nullptr;
  if (int rc = dev_alloc(&d, n)) return rc;
  CsLaunch a{};
  const size_t m = (size_t)b->rl_n - 1;
  a.rl.knots = b->d_rl;
  a.rl.xy = b->d_rl + b->rl_n;
  a.rl.speed = a.rl.xy + 8 * m;
  a.rl.mus = a.rl.speed + 4 * m * b->rl_M;
  a.rl.n = b->rl_n;
  a.rl.M = b->rl_M;
  a.rl.hmin = b->rl_hmin;
  a.rl.vmax = b->rl_vmax;
  a.pts = c->d_pts;
  a.prefix = c->d_pts + 2 * (size_t)c->np;
  a.out = d;
  a.x0 = x0[0];
  a.y0 = x0[1];
  a.v0 = v0;
  a.mu = curr_mu;
  a.scale = scale;
  a.Ts = c->cfg.Ts;
  a.np = c->np;
  a.p0 = projidx;
  a.H = H;
  std::vector<double> h(n);
  hipError_t e = launch_constant_speed(a, b->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost, b->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(LLAMPC_E_HIP, "llampc_ctl_reference: %s", hipGetErrorString(e));
  std::memcpy(xref, h.data(), 2 * (size_t)(H + 1) * sizeof(double));
  if (projidx_out) *projidx_out = (int32_t)h[2 * (H + 1)];
  if (vr) *vr = h[2 * (H + 1) + 1];
  return LLAMPC_OK;
}

int llampc_ctl_set_exchange(llampc_ctl* c, llampc_mailbox* mb, const double* gparams, int64_t n_global) {
  if (!c || !mb || !gparams) return fail(LLAMPC_E_ARG, "NULL argument");
  llampc_bank* b = c->b;
  if (mb->device != b->device) return fail(LLAMPC_E_ARG, "mailbox on device %d, bank on %d", mb->device, b->device);
  if (mb->world > kCtlPxMax) return fail(LLAMPC_E_ARG, "world %d > %d (the exchange's LDS)", mb->world, kCtlPxMax);
  if (n_global < b->goff + b->n || n_global >= (int64_t)0xFFFFFFFFll)
    return fail(LLAMPC_E_ARG, "n_global=%lld: must hold this shard [%lld, %lld) and be < 2^32 - 1", (long long)n_global,
                (long long)b->goff, (long long)(b->goff + b->n));
  for (int g = 0; g < mb->world; ++g)
    if (!mb->box[g]) return fail(LLAMPC_E_STATE, "mailbox of peer %d not open", g);
  std::lock_guard<std::mutex> lc(c->mu);
  if (c->pending) return fail(LLAMPC_E_STATE, "a controller tick is outstanding");
  if (c->t != 0) return fail(LLAMPC_E_STATE, "set the exchange before the first tick");
  if (c->xg_world) return fail(LLAMPC_E_STATE, "the controller already exchanges over a gather transport");
  ctl_cancel(c);                         // no armed launches with an exchange
  c->prelaunch = false;
  DeviceGuard g(b->device);
  double* d = nullptr;
  if (int rc = dev_alloc(&d, 6 * (size_t)n_global)) return rc;
  if (hipMemcpy(d, gparams, 6 * (size_t)n_global * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return fail(LLAMPC_E_HIP, "global parameter table upload failed");
  }
  if (c->d_gparams) (void)hipFree(c->d_gparams);
  c->d_gparams = d;
  c->n_global = n_global;
  c->mb = mb;
  return LLAMPC_OK;
}

int32_t llampc_ctl_record_words(int32_t K) { return (K < 1 || K > LLAMPC_KMAX) ? 0 : ctl_rec_words(K); }

int llampc_ctl_set_gather(llampc_ctl* c, int32_t world, int32_t rank, llampc_comm* comm, const double* gparams,
                          int64_t n_global) {
  if (!c || !gparams) return fail(LLAMPC_E_ARG, "NULL argument");
  llampc_bank* b = c->b;
  if (world < 1 || world > kCtlPxMax || rank < 0 || rank >= world)
    return fail(LLAMPC_E_ARG, "world=%d rank=%d (world 1..%d)", world, rank, kCtlPxMax);
  if (comm && (comm->world != world || comm->rank != rank || comm->device != b->device))
    return fail(LLAMPC_E_ARG, "the communicator is rank %d of %d on device %d, the controller rank %d of %d on %d",
                comm->rank, comm->world, comm->device, rank, world, b->device);
  if (n_global < b->goff + b->n || n_global >= (int64_t)0xFFFFFFFFll)
    return fail(LLAMPC_E_ARG, "n_global=%lld: must hold this shard [%lld, %lld) and be < 2^32 - 1", (long long)n_global,
                (long long)b->goff, (long long)(b->goff + b->n));
  std::lock_guard<std::mutex> lc(c->mu);
  if (c->pending) return fail(LLAMPC_E_STATE, "a controller tick is outstanding");
  if (c->t != 0) return fail(LLAMPC_E_STATE, "set the exchange before the first tick");
  if (c->mb) return fail(LLAMPC_E_STATE, "the controller already exchanges over peer mailboxes");
  ctl_cancel(c);                         // no armed launches with an exchange
  c->prelaunch = false;
  DeviceGuard g(b->device);
  const int nw = ctl_rec_words(c->cfg.K);
  double* d = nullptr;
  if (int rc = dev_alloc(&d, 6 * (size_t)n_global)) return rc;
  if (hipMemcpy(d, gparams, 6 * (size_t)n_global * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return fail(LLAMPC_E_HIP, "global parameter table upload failed");
  }
  if (c->d_gparams) (void)hipFree(c->d_gparams);
  c->d_gparams = d;
  c->n_global = n_global;
  if (!c->d_xsend) {
    int rc;
    if ((rc = dev_alloc(&c->d_xsend, (size_t)nw)) || (rc = dev_alloc(&c->d_xgath, (size_t)kCtlPxMax * nw))) return rc;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_xstage), (size_t)kCtlPxMax * nw * sizeof(uint64_t),
                      hipHostMallocDefault) != hipSuccess)
      return fail(LLAMPC_E_OOM, "hipHostMalloc(gather staging) failed");
    HIP_TRY(hipMemset(c->d_xsend, 0, (size_t)nw * sizeof(uint64_t)));
    HIP_TRY(hipMemset(c->d_xgath, 0, (size_t)kCtlPxMax * nw * sizeof(uint64_t)));
  }
  c->xg_nw = nw;
  c->xg_world = world;
  c->xg_rank = rank;
  c->xg_comm = comm;
  return LLAMPC_OK;
}

int llampc_ctl_shard_record(llampc_ctl* c, uint64_t* words, int32_t* nw) {
  if (!c || !words || !nw) return fail(LLAMPC_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lc(c->mu);
  *nw = 0;
  if (!c->xg_wait) return LLAMPC_OK;     // no exchange on this tick (or RCCL carries it)
  DeviceGuard g(c->b->device);
  const size_t bytes = (size_t)c->xg_nw * sizeof(uint64_t);
  HIP_TRY(hipMemcpyAsync(c->h_xstage, c->d_xsend, bytes, hipMemcpyDeviceToHost, c->b->stream));
  HIP_TRY(hipStreamSynchronize(c->b->stream));
  std::memcpy(words, c->h_xstage, bytes);
  c->xg_read = true;
  *nw = c->xg_nw;
  return LLAMPC_OK;
}

int llampc_ctl_resume(llampc_ctl* c, const uint64_t* all_words) {
  if (!c || !all_words) return fail(LLAMPC_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lc(c->mu);
  if (!c->xg_wait || !c->xg_read)
    return fail(LLAMPC_E_STATE, "no tick awaits its gathered records (llampc_ctl_shard_record first)");
  llampc_bank* b = c->b;
  std::lock_guard<std::mutex> lk(b->mu);
  DeviceGuard g(b->device);
  const size_t bytes = (size_t)c->xg_world * c->xg_nw * sizeof(uint64_t);
  std::memcpy(c->h_xstage, all_words, bytes);
  HIP_TRY(hipMemcpyAsync(c->d_xgath, c->h_xstage, bytes, hipMemcpyHostToDevice, b->stream));
  const llampc_ctl::Prep& P2 = c->xg_second;
  HIP_TRY(launch_ctl(P2.L, P2.lpm, P2.lds, b->stream));
  c->xg_wait = false;
  c->xg_read = false;
  return LLAMPC_OK;
}

int llampc_ctl_merge(const double* vals, const int64_t* gids, int32_t G, int32_t K, int32_t nan_policy,
                     int64_t* topk, double* topk_val, int64_t* best, double* best_val) {
  if (!vals || !gids || !topk || !topk_val || !best || !best_val) return fail(LLAMPC_E_ARG, "NULL argument");
  if (G < 1 || G > kCtlPxMax || K < 1 || K > LLAMPC_KMAX) return fail(LLAMPC_E_ARG, "G=%d (1..%d) K=%d", G, kCtlPxMax, K);
  const int M = G * K;
  std::vector<uint64_t> key(M), id(M);
  for (int e = 0; e < M; ++e) {
    const int g = e / K, j = e - g * K;
    ctl_entry_order(vals[g * (K + 1) + j], gids[g * (K + 1) + j], e, key[e], id[e]);
  }
  for (int k = 0; k < K; ++k) {
    topk[k] = -1;
    topk_val[k] = std::nan("");
  }
  for (int e = 0; e < M; ++e) {
    const int r = ctl_merge_rank([&](int j) { return key[j]; }, [&](int j) { return id[j]; }, M, e);
    if (r < K) {
      const int g = e / K, j = e - g * K;
      const int64_t gid = gids[g * (K + 1) + j];
      topk[r] = gid < 0 ? -1 : gid;
      topk_val[r] = gid < 0 ? std::nan("") : vals[g * (K + 1) + j];
    }
  }
  ctl_merge_argmin([&](int g, double& v, int64_t& i) {
                     v = vals[g * (K + 1) + K];
                     i = gids[g * (K + 1) + K];
                   },
                   G, nan_policy == LLAMPC_NAN_FIRST, *best_val, *best);
  return LLAMPC_OK;
}

int llampc_ctl_inputs(llampc_ctl* c, double* xref, double* U) {
  if (!c || !xref || !U) return fail(LLAMPC_E_ARG, "NULL argument");
  if (!c->d_dbg) return fail(LLAMPC_E_STATE, "controller created without debug_inputs");
  std::lock_guard<std::mutex> lc(c->mu);
  DeviceGuard g(c->b->device);
  ctl_cancel(c);                         // an armed launch would hold the stream (re-armed next tick)
  HIP_TRY(hipStreamSynchronize(c->b->stream));
  const size_t nx = 2 * (size_t)(c->cfg.H + 1), nu = 2 * (size_t)c->cfg.C * c->cfg.H;
  HIP_TRY(hipMemcpy(xref, c->d_dbg, nx * sizeof(double), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(U, c->d_dbg + nx, nu * sizeof(double), hipMemcpyDeviceToHost));
  return LLAMPC_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// setupNLP.solve drop-in (nlp.hip): CEM iterations enqueued back to back on the bank's
// stream, the Euler trajectory of the best sequence, one copy back.
// ------------------------------------------------------------------------------------
struct llampc_nlp {
  llampc_bank* b = nullptr;
  llampc_nlp_cfg cfg{};
  NlpState* d_st = nullptr;              // the best so far across a solve's launches (device);
                                         // the inputs travel as kernel arguments (NlpInline)
  double* d_cost = nullptr;              // the sample blocks' sorted lists as tagged words
                                         // [2][3][samples], then the rounds' rate-clipped
                                         // sequences [2][samples][H][2] (NlpLaunch.list_tag, cand;
                                         // by round parity)
  uint64_t* d_ms_tag = nullptr;          // [2][4 HMAX]: a round's mean / std (NlpLaunch.ms_tag)
  bool per_round = false;                // one launch per round (LLAMPC_NLP_ROUND_LAUNCHES=1: A/B)
  bool ltraj = false;                    // the last round keeps its states in LDS (NlpLaunch.ltraj;
                                         // LLAMPC_NLP_RERUN_TRAJ=1 at create: always re-run, tests)
  NlpResult* h_res = nullptr;            // pinned, coherent, mapped: the last round writes it
  NlpResult* d_res = nullptr;            //   (device alias), then the solve's number into h_tag
  uint64_t* h_tag = nullptr;
  uint64_t* d_tag = nullptr;
  uint64_t calls = 0;
  std::mutex mu;
};

extern "C" {

int llampc_nlp_destroy(llampc_nlp* p) {
  if (!p) return LLAMPC_OK;
  {
    DeviceGuard g(p->b ? p->b->device : 0);
    if (p->b && p->b->stream) (void)hipStreamSynchronize(p->b->stream);
    if (p->d_st) (void)hipFree(p->d_st);
    if (p->d_cost) (void)hipFree(p->d_cost);
    if (p->d_ms_tag) (void)hipFree(p->d_ms_tag);
    if (p->h_res) (void)hipHostFree(p->h_res);
    if (p->h_tag) (void)hipHostFree(p->h_tag);
  }
  delete p;
  return LLAMPC_OK;
}

int llampc_nlp_create(llampc_bank* b, const llampc_nlp_cfg* cfg, llampc_nlp** out) {
  if (!out) return fail(LLAMPC_E_ARG, "out is NULL");
  *out = nullptr;
  if (!b || !cfg) return fail(LLAMPC_E_ARG, "NULL argument");
  const llampc_nlp_cfg& k = *cfg;
  if (b->n != 1) return fail(LLAMPC_E_ARG, "the NLP solver's bank holds one model (n=%lld)", (long long)b->n);
  if (k.H < 1 || k.H > LLAMPC_HMAX) return fail(LLAMPC_E_ARG, "H=%d outside [1, %d]", k.H, LLAMPC_HMAX);
  if (k.samples < 64 || k.samples > 4096 || (k.samples & (k.samples - 1)))
    return fail(LLAMPC_E_ARG, "samples=%d: a power of two in [64, 4096]", k.samples);
  if (k.elite < 1 || k.elite > 64 || k.elite > k.samples || k.iters < 1 || k.iters > kNlpMaxIters)
    return fail(LLAMPC_E_ARG, "elite=%d (1..64, <= samples) iters=%d (1..%d)", k.elite, k.iters, kNlpMaxIters);
  if (!(k.Ts > 0) || !std::isfinite(k.Ts)) return fail(LLAMPC_E_ARG, "Ts must be finite > 0");
  if (nlp_lds_bytes(k.H, k.samples, k.elite) > 160 * 1024) return fail(LLAMPC_E_ARG, "H x elite too large for LDS");
  DeviceGuard g(b->device);
  auto* p = new llampc_nlp();
  p->b = b;
  p->cfg = k;
  const size_t H = (size_t)k.H;
  auto cleanup = [&](int code) {
    llampc_nlp_destroy(p);
    return code;
  };
  int rc;
  // the lists: 3 words per entry, samples / 64 x len <= samples entries; both by round parity
  if ((rc = dev_alloc(&p->d_st, 1)) || (rc = dev_alloc(&p->d_cost, (size_t)k.samples * (6 + 4 * (size_t)H))) ||
      (rc = dev_alloc(&p->d_ms_tag, 8 * (size_t)LLAMPC_HMAX)))
    return cleanup(rc);
  {
    // every round in one launch needs all samples / 64 blocks resident together (each waits for
    // the others' rounds; one block per CU by its LDS request): not on a device, or a partition
    // of one, with fewer CUs than blocks — then one launch per round
    const char* e = std::getenv("LLAMPC_NLP_ROUND_LAUNCHES");
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b->device) != hipSuccess) cus = 0;
    const bool resident = k.samples / 64 <= cus;
    p->per_round = !nlp_persistent(k.samples) || !resident || (e && e[0] == '1');
    const char* rt = std::getenv("LLAMPC_NLP_RERUN_TRAJ");
    p->ltraj = nlp_ltraj_fits(k.H, k.samples, k.elite) && !(rt && rt[0] == '1');
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&p->h_res), sizeof(NlpResult), hipHostMallocCoherent | hipHostMallocMapped) !=
          hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&p->h_tag), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return cleanup(fail(LLAMPC_E_OOM, "hipHostMalloc(NLP result) failed"));
  *p->h_tag = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_res), p->h_res, 0) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&p->d_tag), p->h_tag, 0) != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "hipHostGetDevicePointer(NLP result) failed"));
  // tagged words start at tag 0, which no solve uses (nlp_seq of a solve number >= 1)
  if (hipMemset(p->d_st, 0, sizeof(NlpState)) != hipSuccess ||
      hipMemset(p->d_cost, 0, (size_t)k.samples * 6 * sizeof(uint64_t)) != hipSuccess ||
      hipMemset(p->d_ms_tag, 0, 8 * LLAMPC_HMAX * sizeof(uint64_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return cleanup(fail(LLAMPC_E_HIP, "NLP solver upload failed"));
  *out = p;
  return LLAMPC_OK;
}

int llampc_nlp_solve(llampc_nlp* p, const double* x0, const double* xref, const double* uprev, const double* base,
                     int32_t has_hold, double* umpc, double* fval, double* xmpc) {
  if (!p || !x0 || !xref || !uprev || !umpc) return fail(LLAMPC_E_ARG, "NULL argument");
  std::lock_guard<std::mutex> lp(p->mu);
  llampc_bank* b = p->b;
  std::lock_guard<std::mutex> lk(b->mu);
  bank_disarm(b);
  if (b->async_pending) return fail(LLAMPC_E_STATE, "an async tick is outstanding on the bank");
  DeviceGuard g(b->device);
  const llampc_nlp_cfg& k = p->cfg;
  const int H = k.H;
  hipStream_t s = b->stream;
  // the launch's inputs (NlpInline): x0, xref, the first mean (base or uprev held); the first
  // std is sigma0, the best so far starts at +inf (the kernel's round 0)
  NlpInline pk;
  std::memcpy(pk.v, x0, 6 * sizeof(double));
  std::memcpy(pk.v + 6, xref, 2 * (size_t)(H + 1) * sizeof(double));
  double* m0 = pk.v + 6 + 2 * (H + 1);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < 2; ++j) m0[2 * i + j] = base ? base[2 * i + j] : uprev[j];
  NlpLaunch a{};
  a.la.params = b->d_params;
  a.la.n = 1;
  a.la.veh = integrator_veh(b->veh, LLAMPC_EULER_NLP);
  a.la.C = 64;
  a.la.H = H;
  a.la.integrator = LLAMPC_EULER_NLP;
  a.la.Ts = k.Ts;
  a.la.cost = make_cost(k.cost, k.Ts);
  a.st = p->d_st;
  a.list_tag = reinterpret_cast<uint64_t*>(p->d_cost);
  a.cand = p->d_cost + 6 * (size_t)k.samples;
  a.res = p->d_res;
  a.host_tag = p->d_tag;
  a.host_seq = p->calls + 1;
  a.ms_tag = p->d_ms_tag;
  a.ltraj = p->ltraj;
  a.seed = k.seed;
  a.call = p->calls;
  a.up0 = uprev[0];
  a.up1 = uprev[1];
  a.umin0 = k.cost.umin[0];
  a.umin1 = k.cost.umin[1];
  a.umax0 = k.cost.umax[0];
  a.umax1 = k.cost.umax[1];
  a.rlo0 = k.rate_lo[0];
  a.rlo1 = k.rate_lo[1];
  a.rhi0 = k.rate_hi[0];
  a.rhi1 = k.rate_hi[1];
  a.std_floor = k.std_floor;
  a.sig0 = k.sigma0[0];
  a.sig1 = k.sigma0[1];
  a.H = H;
  a.samples = k.samples;
  a.elite = k.elite;
  a.has_hold = has_hold;
  a.iters = k.iters;                    // the last round's completion writes xmpc (nmpc.py:58-60)
  if (p->per_round) {
    a.rounds = 1;
    for (int it = 0; it < k.iters; ++it) {
      a.it = it;
      TimedLaunch tl(b, 0, s);           // llampc_bank_timing on the solver's bank: per round
      HIP_TRY(launch_nlp(a, pk, s));
    }
  } else {                              // every round in one launch (nlp.hpp nlp_persistent)
    a.it = 0;
    a.rounds = k.iters;
    TimedLaunch tl(b, 0, s);             // llampc_bank_timing on the solver's bank: per solve
    HIP_TRY(launch_nlp(a, pk, s));
  }
  // the last round's completion writes the result into pinned memory and then the tag
  const uint64_t want = p->calls + 1;
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  while (__atomic_load_n(p->h_tag, __ATOMIC_ACQUIRE) != want) {
    __builtin_ia32_pause();
    if ((++spins & 0xFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
      HIP_TRY(hipStreamSynchronize(s));
      if (__atomic_load_n(p->h_tag, __ATOMIC_ACQUIRE) == want) break;
      // the launch has ended (its blocks give up a round wait after kNlpRoundWait): the next
      // solve must not meet this one's state — a new call number, so none of this solve's
      // tagged words (lists, mean / std) matches a later round's tag
      p->calls++;
      return fail(LLAMPC_E_DEVICE, "NLP solve %llu: completion tag never arrived", (unsigned long long)want);
    }
  }
  p->calls++;
  b->launches += p->per_round ? k.iters : 1;
  const NlpResult* r = const_cast<const NlpResult*>(p->h_res);
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < 2; ++j) umpc[2 * i + j] = r->best_u[i][j];
  if (fval) *fval = r->best_j;
  if (xmpc) std::memcpy(xmpc, &r->traj[0][0], 6 * (size_t)(H + 1) * sizeof(double));
  if (r->best_it < 0) return fail(LLAMPC_E_DEVICE, "no finite objective in %d rounds of %d samples", k.iters, k.samples);
  return LLAMPC_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// Raw batched dynamics: per-device cached workspace + stream
// ------------------------------------------------------------------------------------
namespace {

struct Workspace {
  std::mutex mu;
  void* d = nullptr;
  size_t cap = 0;
  hipStream_t stream = nullptr;
};
Workspace g_ws[64];

int ws_get(int device, size_t bytes, Workspace** out) {
  if (device < 0 || device >= 64) return fail(LLAMPC_E_ARG, "device %d", device);
  Workspace& w = g_ws[device];
  if (!w.stream) HIP_TRY(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
  if (bytes > w.cap) {
    if (w.d) (void)hipFree(w.d);
    w.d = nullptr;
    w.cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1 << 20);
    hipError_t e = hipMalloc(&w.d, cap);
    if (e != hipSuccess) return fail(LLAMPC_E_OOM, "workspace hipMalloc(%zu): %s", cap, hipGetErrorString(e));
    w.cap = cap;
  }
  *out = &w;
  return LLAMPC_OK;
}

int resolve_device(int32_t device, int* out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
    return fail(LLAMPC_E_NODEV, "no HIP device visible (the HIP path has no CPU fallback)");
  int d = device;
  if (d < 0 && hipGetDevice(&d) != hipSuccess) d = 0;
  if (d >= ndev) return fail(LLAMPC_E_ARG, "device %d of %d", d, ndev);
  *out = d;
  return LLAMPC_OK;
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

extern "C" int llampc_dynamics_batch(int32_t op, const double* x, const double* u,
                                     const double* params, int64_t P, const llampc_vehicle* veh,
                                     int64_t n, double* out, int32_t device, int32_t device_ptrs,
                                     void* stream) {
  if (!x || !u || !params || !veh || !out) return fail(LLAMPC_E_ARG, "NULL argument");
  if (op != LLAMPC_OP_FORCES && op != LLAMPC_OP_DERIV) return fail(LLAMPC_E_ARG, "op %d", op);
  if (n < 0 || !(P == 1 || P == n)) return fail(LLAMPC_E_ARG, "P=%lld must be 1 or n=%lld", (long long)P, (long long)n);
  if (n == 0) return LLAMPC_OK;
  int dev, rc;
  if ((rc = resolve_device(device, &dev))) return rc;
  DeviceGuard g(dev);
  const VehK vk = make_veh(*veh);
  const size_t out_n = (op == LLAMPC_OP_FORCES ? 5 : 6) * (size_t)n;
  if (device_ptrs) {
    HIP_TRY(launch_dynamics(op, x, u, params, P, vk, n, out, (hipStream_t)stream));
    return LLAMPC_OK;
  }
  const size_t bx = align_up(6 * n * 8), bu = align_up(2 * n * 8), bp = align_up(6 * P * 8),
               bo = align_up(out_n * 8);
  Workspace* w;
  std::lock_guard<std::mutex> lk(g_ws[dev].mu);
  if ((rc = ws_get(dev, bx + bu + bp + bo, &w))) return rc;
  char* base = (char*)w->d;
  double *dx = (double*)base, *du = (double*)(base + bx), *dp = (double*)(base + bx + bu),
         *dout = (double*)(base + bx + bu + bp);
  HIP_TRY(hipMemcpyAsync(dx, x, 6 * n * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(du, u, 2 * n * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(dp, params, 6 * P * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(launch_dynamics(op, dx, du, dp, P, vk, n, dout, w->stream));
  HIP_TRY(hipMemcpyAsync(out, dout, out_n * 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  return LLAMPC_OK;
}

extern "C" int llampc_integrate_batch(const double* x0, const double* u, int64_t u_stride_lane,
                                      const double* h, int32_t S, const double* params, int64_t P,
                                      const llampc_vehicle* veh, int64_t n, int32_t integrator,
                                      double* traj_out, int32_t final_only, int32_t device,
                                      int32_t device_ptrs, void* stream) {
  if (!x0 || !u || !h || !params || !veh || !traj_out) return fail(LLAMPC_E_ARG, "NULL argument");
  if (S < 1) return fail(LLAMPC_E_ARG, "S=%d must be >= 1", S);
  if (n < 0 || !(P == 1 || P == n)) return fail(LLAMPC_E_ARG, "P must be 1 or n");
  if (!(u_stride_lane == 0 || u_stride_lane == 2 * (int64_t)S))
    return fail(LLAMPC_E_ARG, "u_stride_lane must be 0 or 2*S");
  if (integrator < LLAMPC_RK4 || integrator > LLAMPC_RK6) return fail(LLAMPC_E_ARG, "integrator %d", integrator);
  if (n == 0) return LLAMPC_OK;
  int dev, rc;
  if ((rc = resolve_device(device, &dev))) return rc;
  DeviceGuard g(dev);
  const VehK vk = integrator_veh(make_veh(*veh), integrator);
  const size_t out_n = (final_only ? 1 : (size_t)(S + 1)) * n * 6;
  if (device_ptrs) {
    HIP_TRY(launch_integrate(x0, u, u_stride_lane, h, S, params, P, vk, n, integrator, traj_out,
                             final_only, (hipStream_t)stream));
    return LLAMPC_OK;
  }
  const size_t un = (u_stride_lane ? (size_t)n : 1) * 2 * S;
  const size_t bx = align_up(6 * n * 8), bu = align_up(un * 8), bh = align_up(S * 8),
               bp = align_up(6 * P * 8), bo = align_up(out_n * 8);
  Workspace* w;
  std::lock_guard<std::mutex> lk(g_ws[dev].mu);
  if ((rc = ws_get(dev, bx + bu + bh + bp + bo, &w))) return rc;
  char* base = (char*)w->d;
  double *dx = (double*)base, *du = (double*)(base + bx), *dh = (double*)(base + bx + bu),
         *dp = (double*)(base + bx + bu + bh), *dout = (double*)(base + bx + bu + bh + bp);
  HIP_TRY(hipMemcpyAsync(dx, x0, 6 * n * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(du, u, un * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(dh, h, S * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(hipMemcpyAsync(dp, params, 6 * P * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(launch_integrate(dx, du, u_stride_lane, dh, S, dp, P, vk, n, integrator, dout, final_only,
                           w->stream));
  HIP_TRY(hipMemcpyAsync(traj_out, dout, out_n * 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  return LLAMPC_OK;
}

extern "C" int llampc_math_batch(int32_t fn, const double* a, const double* b, int64_t n,
                                 double* out, int32_t device) {
  if (!a || !out || ((fn == LLAMPC_MATH_ATAN2_XPOS || fn == LLAMPC_MATH_ATAN2_FAST ||
                      fn == LLAMPC_MATH_ATAN2_LEAN || fn == LLAMPC_MATH_ATAN2_PAIR) && !b))
    return fail(LLAMPC_E_ARG, "NULL argument");
  if (fn < LLAMPC_MATH_ATAN2_XPOS || fn > LLAMPC_MATH_ATAN_PAIR) return fail(LLAMPC_E_ARG, "fn %d", fn);
  if (n <= 0) return LLAMPC_OK;
  int dev, rc;
  if ((rc = resolve_device(device, &dev))) return rc;
  DeviceGuard g(dev);
  const size_t bn = align_up(n * 8);
  Workspace* w;
  std::lock_guard<std::mutex> lk(g_ws[dev].mu);
  if ((rc = ws_get(dev, 3 * bn, &w))) return rc;
  char* base = (char*)w->d;
  double *da = (double*)base, *db = (double*)(base + bn), *dout = (double*)(base + 2 * bn);
  HIP_TRY(hipMemcpyAsync(da, a, n * 8, hipMemcpyHostToDevice, w->stream));
  if (b) HIP_TRY(hipMemcpyAsync(db, b, n * 8, hipMemcpyHostToDevice, w->stream));
  HIP_TRY(launch_math(fn, da, db, n, dout, w->stream));
  HIP_TRY(hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, w->stream));
  HIP_TRY(hipStreamSynchronize(w->stream));
  return LLAMPC_OK;
}
