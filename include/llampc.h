/*
 * llampc.h — C ABI of the MI355X-native LLA-MPC model-bank engine (libllampc_hip.so).
 *
 * Drop-in boundary for the reference's hot path (tianhao-stan-wu/LLA-MPC; all
 * citations relative to the reference root).  Plain pointers and sizes only; every
 * array is row-major fp64 unless stated.  All calls return 0 on success or a negative
 * LLAMPC_E_* code; llampc_last_error() gives the thread's last message.
 *
 *  ABI entry point                 replaces (reference)
 *  ------------------------------  -----------------------------------------------------
 *  llampc_bank_create/destroy      the N-object MODEL_BANK + params_pass tuple
 *                                  (llampc/mpc/run_nmpc_orca_llampc_rt.py:161-179) and the
 *                                  error_windows ring (rt.py:83-84)
 *  llampc_lookback                 evaluate_models_vectorized (llampc/mpc/evaluate_models_
 *                                  vectorized.py:4-24) + the inline error / window / argmin
 *                                  / argsort[:K] block (rt.py:347-366)
 *  llampc_lookahead                H x Model._integrate_batch (llampc/models/model.py:32-40)
 *                                  per (model, candidate) + the NLP objective
 *                                  (llampc/mpc/nmpc.py:44-111) + argmin
 *  llampc_plan / llampc_plan_device one LLA-MPC tick: rt.py:300-366 (look-back on the
 *                                  newest transition, selection, look-ahead from x_t)
 *  llampc_merge / _device          (new) cross-shard merge of per-GPU plan results
 *  llampc_exchange_rccl / _peer    (new) the per-tick gather + merge of the sharded bank
 *                                  (SURVEY.md §8e): RCCL all-gather, or xGMI mailboxes
 *  llampc_nlp_*                    setupNLP / .solve (nmpc.py:14-203), solved by sampling
 *  llampc_dynamics_batch           Dynamic.calc_forces_batch (llampc/models/dynamic.py:
 *                                  117-154), Dynamic._diffequation_batch (:98-115)
 *  llampc_ctl_*                    the control loop body rt.py:278-366 on the device
 *                                  (ConstantSpeed, selection, look-ahead, mu-hat, state)
 *  llampc_integrate_batch          Model._integrate_batch (model.py:32-40, RK4),
 *                                  Model._integrate/odeintRK6 (model.py:18-30,
 *                                  llampc/utils/rk6.py:13-28) and the NLP Euler form
 *                                  (nmpc.py:58-60 with Dynamic.casadi, dynamic.py:195-226)
 */
#ifndef LLAMPC_H_
#define LLAMPC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LLAMPC_ABI_VERSION 1
#define LLAMPC_KMAX 32          /* max top-K (rt.py:69 uses K=10) */
#define LLAMPC_WMAX 128         /* max look-back window (rt.py:67 uses W=10) */
#define LLAMPC_HMAX 64          /* max horizon of the controller tick (rt.py:52 uses 20) */

enum llampc_status {
  LLAMPC_OK = 0,
  LLAMPC_E_ARG = -1,        /* bad argument / shape                       */
  LLAMPC_E_HIP = -2,        /* HIP runtime error                          */
  LLAMPC_E_NODEV = -3,      /* no HIP device                              */
  LLAMPC_E_STATE = -4,      /* call not valid in the handle's state       */
  LLAMPC_E_OOM = -5,        /* device allocation failed                   */
  LLAMPC_E_DEVICE = -6      /* the tick's record reports a device-side status != 0 */
};

/* Integrators.  RK4 = odeintRK4_batch (rk6.py:50-68) on the |vx| dynamics
 * (dynamic.py:98-154); EULER_NLP = the NLP transcription x+Ts*f (nmpc.py:58-60) on
 * Dynamic.casadi (vmin clamp, atan2(.,vx); dynamic.py:195-226); RK6 = odeintRK6
 * (rk6.py:13-28), the plant integrator (dynamic.py:59-74). */
enum llampc_integrator { LLAMPC_RK4 = 0, LLAMPC_EULER_NLP = 1, LLAMPC_RK6 = 2 };

/* argmin NaN policy for the look-back selection: NAN_FIRST reproduces np.argmin
 * (first NaN wins, rt.py:359); NAN_IGNORE treats NaN as +inf.  top-K always orders
 * NaN last (np.argsort, rt.py:360).  The look-ahead argmin always treats NaN as +inf. */
enum llampc_nan_policy { LLAMPC_NAN_FIRST = 0, LLAMPC_NAN_IGNORE = 1 };

/* llampc_dynamics_batch ops */
enum llampc_dyn_op { LLAMPC_OP_FORCES = 0, LLAMPC_OP_DERIV = 1 };

/* Shared (per-bank) vehicle constants (llampc/params/orca.py:13-27). */
typedef struct llampc_vehicle {
  double lf, lr, mass, Iz;
  double Cm1, Cm2, Cr0, Cr2;
  int32_t input_acc;   /* 1: Frx = mass*u0 (dynamic.py:139-142)                    */
  int32_t approx;      /* 1: linear tires Ffy=2*Cf*af (dynamic.py:126-136); params */
                       /*    rows Cf/Cr are then cornering stiffnesses             */
} llampc_vehicle;

/* Look-ahead objective (nmpc.py:44-111) and candidate feasibility (nmpc.py:102-105). */
typedef struct llampc_cost {
  double Q[4];         /* 2x2 row-major tracking weight   (rt.py:60 diag(1,1))      */
  double R[4];         /* 2x2 row-major input-rate weight (rt.py:62 diag(5e-3,1))   */
  double P[4];         /* 2x2 row-major terminal weight   (rt.py:61 diag(0,0))      */
  double umin[2], umax[2];   /* input bounds (orca.py:31-35)                        */
  double rate_max[2];  /* |u_k - u_{k-1}| <= rate_max*Ts; <0 disables (orca.py:35)  */
  int32_t enforce_bounds;    /* 1: infeasible candidates cost +inf                  */
  int32_t reserved;
} llampc_cost;

/* Look-ahead reference.  GIVEN: one shared xref [2][H+1] (ConstantSpeed with mu-hat,
 * rt.py:280).  RACELINE: every model tracks its own ConstantSpeed
 * reference (planner.py:12-67) with mu_n = (Df_n + Dr_n) / (9.81 mass), evaluated on the
 * device from the table of llampc_bank_set_raceline; xref then points to the shared start
 * {s0 = arc length after the projection (planner.py:25-33), v0, scale, 0}. */
enum llampc_xref_mode { LLAMPC_XREF_GIVEN = 0, LLAMPC_XREF_RACELINE = 1 };

/* One tick's inputs.  Pointers are HOST pointers for llampc_plan and DEVICE pointers
 * for llampc_plan_device. */
typedef struct llampc_plan_in {
  const double* x_prev;   /* [6]  x_{t-1}                                          */
  const double* u_prev;   /* [2]  u_{t-1}                                          */
  const double* x_now;    /* [6]  x_t (look-back target, look-ahead start)          */
  const double* U;        /* [C][H][2] candidate control sequences                 */
  const double* xref;     /* [2][H+1] reference (planner.py:12-67 output); with
                             xref_mode RACELINE: [4] {s0, v0, scale, 0} (see below)  */
  const double* uprev;    /* [2]  last applied input for du_0 (nmpc.py:65-66)      */
  int32_t C, H;
  int32_t K;              /* top-K size, <= LLAMPC_KMAX                            */
  int32_t integrator;     /* look-ahead integrator                                 */
  int32_t do_lookback;    /* 0: skip the look-back (first tick, rt.py:347)         */
  int32_t do_lookahead;   /* 0: skip the look-ahead                                */
  int32_t nan_policy;
  int32_t xref_mode;      /* LLAMPC_XREF_GIVEN (0) or LLAMPC_XREF_RACELINE (1)      */
  int64_t current_model;  /* global index used while the window fills (rt.py:264)  */
  double Ts;
  llampc_cost cost;
} llampc_plan_in;

/* One tick's result (fixed size: also the cross-GPU payload, see llampc_merge). */
#define LLAMPC_STATUS_POLL_TIMEOUT 1
typedef struct llampc_plan_out {
  int32_t window_count;   /* transitions in the window, <= W (rt.py:354)           */
  int32_t window_full;    /* window_count >= W: selection valid (rt.py:357)        */
  int32_t K;
  int32_t sel_owned;      /* this shard owns sel_model                             */
  int64_t lb_best;        /* argmin of the window mean (rt.py:359), -1 if not full */
  double  lb_best_val;
  int64_t sel_model;      /* full ? lb_best : current_model                        */
  int32_t sel_cand;       /* argmin_c cost[sel_model, c]  ("chosen control")       */
  int32_t n_nonfinite;    /* look-ahead rollouts whose cost is not finite          */
  double  sel_cost;
  int64_t la_best_model;  /* argmin over all (model, candidate) costs              */
  int32_t la_best_cand;
  int32_t status;         /* 0 ok; LLAMPC_STATUS_POLL_TIMEOUT (1): the in-launch
                             completion (or the peer exchange) gave up waiting (a device
                             fault or a missing rank, never expected) */
  double  la_best_cost;
  int64_t topk[LLAMPC_KMAX];      /* argsort(window mean)[:K] (rt.py:360), -1 pad  */
  double  topk_val[LLAMPC_KMAX];
  double  topk_Df[LLAMPC_KMAX];   /* bank Df/Dr of the top-K (rt.py:336-338)      */
  double  topk_Dr[LLAMPC_KMAX];
  int32_t topk_cand[LLAMPC_KMAX]; /* look-ahead best candidate of each top-K model */
  double  topk_cost[LLAMPC_KMAX];
} llampc_plan_out;

typedef struct llampc_bank llampc_bank;

/* ---- library ---------------------------------------------------------------- */
int32_t     llampc_abi_version(void);
const char* llampc_last_error(void);
int         llampc_device_count(int32_t* count);

/* ---- bank handle -------------------------------------------------------------- */
/* params: [6][n] rows (Bf, Cf, Df, Br, Cr, Dr) = rt.py:179 params_pass order.
 * global_offset: global index of this shard's first model (multi-GPU).  W: window. */
int llampc_bank_create(const double* params, int64_t n, int64_t global_offset,
                       const llampc_vehicle* veh, int32_t W, int32_t device,
                       llampc_bank** out);
int llampc_bank_destroy(llampc_bank* bank);
int llampc_bank_info(const llampc_bank* bank, int64_t* n, int64_t* global_offset,
                     int32_t* W, int32_t* window_count, int32_t* device);
int llampc_bank_reset(llampc_bank* bank);                 /* empty the window       */
/* plan-kernel launches enqueued on this bank so far (every tick entry point is ONE
 * launch; the controller test counts them — replaces nothing in the reference) */
int llampc_bank_launches(const llampc_bank* bank, int64_t* launches);
/* ring: [n][W] oldest -> newest (the rt.py error_windows layout, zeros if unfilled) */
int llampc_bank_window(llampc_bank* bank, double* ring, int32_t* window_count);
/* stream the bank launches on (hipStream_t as void*); NULL = its own stream */
int llampc_bank_set_stream(llampc_bank* bank, void* stream);
/* the stream the bank launches on now (its own or the one set above), for callers that
 * enqueue their own work with it.  The bank's OWN stream may be replaced by a dedicated-queue
 * one (llampc_bank_set_concurrency(banks > 1), llampc_ctl_set_prelaunch(on)): a handle read
 * earlier is then destroyed — read it again after either call. */
int llampc_bank_stream(const llampc_bank* bank, void** stream);
/* the number of banks the caller ticks concurrently on this device (default 1; BASELINE
 * config 5 ticks two tracks together: 2).  The look-ahead sizes its launch for 1/banks of the
 * chip (its lane split), so the concurrent launches are resident together, and banks > 1 gives
 * the bank's own stream a hardware queue of its own (a full-CU-mask stream: two banks' launches
 * on one of HIP's shared queues would run one after the other).  Other banks
 * keep a plain non-blocking stream (LLAMPC_DEDICATED_QUEUE=1 at create: a dedicated queue
 * anyway).  Replaces nothing in the reference (one process per track there) */
int llampc_bank_set_concurrency(llampc_bank* bank, int32_t banks);

/* Per-kernel HIP-event timing of the bank's launches, on the stream they run on (for the
 * benchmark's roofline).  enable=k >= 1 arms `max_launches` event pairs; each pair brackets
 * a group of k consecutive launches of the plan kernel (the whole tick: look-back +
 * look-ahead + selection), so the mean launch duration is elapsed / k (k > 1 spreads the
 * events' own cost over the group); enable=-k (k >= 1) brackets ONE launch out of every k
 * (sampling: for ticks whose launches are separated by other work on the stream, e.g. the
 * multi-GPU exchange, with the events' cost on 1/k of the ticks); enable=0 disarms.
 * count = launches timed. */
int llampc_bank_timing(llampc_bank* bank, int32_t enable, int32_t max_launches);
/* Synchronises, returns avg_ms[3] and count[3] for {plan kernel, reserved, reserved}
 * since the last read, and re-arms the counters. */
int llampc_bank_timing_read(llampc_bank* bank, double* avg_ms, int64_t* count);

/* ---- look-back (host pointers) -------------------------------------------------- */
/* err_out [n] (rt.py:349 errors), wmean_out [n] (rt.py:358 avg_errors, valid when the
 * window is full), topk/topk_val [K] may each be NULL. */
int llampc_lookback(llampc_bank* bank, const double* x_prev, const double* u_prev,
                    const double* x_now, double Ts, int32_t K, int32_t nan_policy,
                    double* err_out, double* wmean_out, int64_t* best, int64_t* topk,
                    double* topk_val, int32_t* window_count);

/* ---- look-ahead (host pointers) ------------------------------------------------- */
/* cost_out [n][C] and best_cand_out [n] may be NULL. */
int llampc_lookahead(llampc_bank* bank, const double* x0, const double* U, int32_t C,
                     int32_t H, const double* xref, const double* uprev,
                     const llampc_cost* cost, double Ts, int32_t integrator,
                     double* cost_out, int32_t* best_cand_out, int64_t* best_model,
                     int32_t* best_cand, double* best_cost);

/* Attach (replace) the raceline library used by LLAMPC_XREF_RACELINE: natural cubic
 * splines over the arc length (pycubicspline.py:17-182, track.py:52-83): knots [n]
 * (Spline2D.s, ascending from 0), xy [2][4][n-1] (x(s) then y(s); rows a, b, c, d per
 * segment), speed [M][4][n-1] (one speed profile per friction), mus [M] ascending.
 * 2 <= n <= 850 (knots and x/y rows are staged in 60 KB of LDS), 1 <= M <= 64.  Copied
 * to the device. */
int llampc_bank_set_raceline(llampc_bank* bank, const double* knots, int32_t n, const double* xy,
                             const double* speed, const double* mus, int32_t M);

/* ---- fused tick ------------------------------------------------------------------ */
/* Host pointers; blocking.  err_out [n], wmean_out [n], cost_out [n][C] may be NULL.
 * With all three NULL the kernel writes the record into the bank's pinned host buffer and
 * then a completion tag; the call spins on the tag (no D2H copy, no stream synchronise).
 * LLAMPC_SYNC_COMPLETION=1 in the environment selects the copy + synchronise path. */
int llampc_plan(llampc_bank* bank, const llampc_plan_in* in, llampc_plan_out* out,
                double* err_out, double* wmean_out, double* cost_out);
/* Host pointers; asynchronous (SURVEY.md §8b "_async" variant): the inputs are copied
 * into the bank's pinned staging buffer before the call returns (the caller may reuse
 * them), and the H2D copy and the plan kernel are enqueued on the bank's stream; the
 * kernel writes the record to pinned host memory + a completion tag, on which
 * llampc_plan_wait spins before returning the record.
 * At most one outstanding async tick per bank (LLAMPC_E_STATE otherwise); independent
 * banks (e.g. two tracks) overlap on the device. */
int llampc_plan_async(llampc_bank* bank, const llampc_plan_in* in);
int llampc_plan_wait(llampc_bank* bank, llampc_plan_out* out);
/* Device pointers in `in`; d_out is a device llampc_plan_out; asynchronous on
 * `stream` (hipStream_t, NULL = the bank's stream).  d_err/d_wmean/d_cost: device
 * arrays or NULL.  LLAMPC_E_STATE while an llampc_plan_async tick is outstanding (both
 * would share the bank's completion state and window). */
int llampc_plan_device(llampc_bank* bank, const llampc_plan_in* in, void* d_out,
                       double* d_err, double* d_wmean, double* d_cost, void* stream);

/* ---- multi-GPU merge ----------------------------------------------------------- */
/* Merge G shard results (shards ordered by global_offset; G <= 32 on the device) into one, deterministic:
 * lowest value, ties -> lowest global index, NaN first for lb_best under NAN_FIRST.
 * Host version runs the same merge code as the device version. */
int llampc_merge(const llampc_plan_out* parts, int32_t G, int32_t nan_policy,
                 llampc_plan_out* merged);
int llampc_merge_device(const void* d_parts, int32_t G, int32_t nan_policy, void* d_merged,
                        int32_t device, void* stream);
/* ---- RCCL, the library's own communicator (public rccl.h API) ---------------------- */
/* The library resolves RCCL at first use: the librccl.so.1 the process has already loaded
 * (torch's, so one RCCL per process), else the system's.  Setup per rank: rank 0 calls
 * llampc_comm_unique_id (ncclGetUniqueId) and shares the 128-byte id out of band (e.g. a
 * torch.distributed store or all_gather_object); every rank calls llampc_comm_create
 * (ncclCommInitRank on `device`; collective: blocks until all `world` ranks joined).
 * LLAMPC_E_STATE when no RCCL can be loaded. */
typedef struct llampc_comm llampc_comm;
int llampc_comm_unique_id(void* id /* 128 bytes out */);
int llampc_comm_create(const void* id /* 128 bytes */, int32_t world, int32_t rank, int32_t device, llampc_comm** out);
int llampc_comm_destroy(llampc_comm* comm);
/* The per-tick exchange of the sharded bank, enqueued on `stream` (hipStream_t) with no
 * host round trip: ncclAllGather of this rank's record d_local (one llampc_plan_out) into
 * d_all [world] over `comm`, then merge_kernel into d_merged.  Replaces the reference-side
 * gather that SURVEY.md §8e specifies (the reference itself is single-process). */
int llampc_exchange_rccl(llampc_comm* comm, const void* d_local, void* d_all, void* d_merged, int32_t nan_policy,
                         void* stream);

/* Peer exchange: the same per-tick gather + merge with no collective library.  Each rank
 * owns a mailbox (uncached device memory, [2][world] record slots of tagged words) that every
 * peer process maps through HIP IPC; per tick ONE kernel pushes this rank's record into slot
 * [rank] of every mailbox over xGMI (system-scope stores), polls its own mailbox until all
 * `world` records of this tick have arrived and runs merge_kernel's merge — the output equals
 * llampc_exchange_rccl's.  Setup: create, export the IPC handle (64 bytes), share the
 * handles out of band (e.g. a torch.distributed all_gather_object), open every peer's.  All
 * ranks must call llampc_exchange_peer the same number of times (the tick number is the tag).
 * A rank that waits more than the poll bound (default 10 s; set_bound) gets status
 * LLAMPC_STATUS_POLL_TIMEOUT in d_merged.  Replaces the same reference-side gather as
 * llampc_exchange_rccl. */
typedef struct llampc_mailbox llampc_mailbox;
int llampc_mailbox_create(int32_t world, int32_t rank, int32_t device, llampc_mailbox** out);
int llampc_mailbox_ipc_handle(llampc_mailbox* mb, void* handle /* 64 bytes out */);
int llampc_mailbox_open_peer(llampc_mailbox* mb, int32_t peer, const void* handle /* 64 bytes */);
/* Use `other`, a mailbox of rank `peer` created in THIS process on the same device, as that
 * peer's (several ranks driven from one process; tests). */
int llampc_mailbox_link(llampc_mailbox* mb, int32_t peer, const llampc_mailbox* other);
int llampc_mailbox_set_bound(llampc_mailbox* mb, double seconds);
int llampc_exchange_peer(llampc_mailbox* mb, const void* d_local, void* d_merged, int32_t nan_policy,
                         void* stream);
/* The sharded tick in ONE launch per rank: llampc_plan_device's tick on this rank's shard
 * (record -> d_local) whose completing block then runs the peer exchange itself (push, poll,
 * merge -> d_merged), so no second kernel follows the plan (RK4 look-ahead with the given
 * xref; otherwise, for world > 16 (the merge's LDS) or with LLAMPC_PEER_SPLIT=1: the plan
 * launch followed by llampc_exchange_peer).  Same rules as
 * llampc_plan_device (stream, LLAMPC_E_STATE while an async tick is outstanding) and as
 * llampc_exchange_peer (every rank makes the same sequence of exchange calls). */
int llampc_plan_exchange(llampc_bank* bank, const llampc_plan_in* in, void* d_local, void* d_merged,
                         llampc_mailbox* mb, void* stream);
int llampc_mailbox_destroy(llampc_mailbox* mb);

/* ---- controller tick (the whole control step on the device) ------------------------- */
/* One LLA-MPC control step of rt.py:269-366 in ONE kernel launch, the controller state kept
 * on the device between ticks (replaces the host loop body rt.py:278-366: ConstantSpeed with
 * mu-hat, planner.py:12-67 + track.py:147-160; the per-tick solve, nmpc.py:161-203 — here a
 * candidate search; the look-back selection rt.py:347-366; the mu-hat estimator rt.py:326-344):
 *   reference   ConstantSpeed(x_t, projidx, mu-hat, v_factor) once the window has been full
 *               for a tick (rt.py:278-282), ConstantSpeed(x_t, projidx) before; the start arc
 *               length from `prefix` (one entry per projection index, the reference's own sum);
 *               lap wrap projidx > lap_projidx -> 0 (rt.py:287-296)
 *   candidates  C sequences: candidate 0 = the previous chosen sequence shifted one step (or
 *               u_{t-1} held), candidate c >= 1 adds Philox4x32-10 noise (four-word sum, unit
 *               variance) x sigma_j, clipped to cost.umin/umax and, in order over the horizon,
 *               to |du| <= cost.rate_max Ts (oracle/llampc_oracle.py candidates_ctl)
 *   look-back   the transition (x_{t-1}, u_{t-1}) -> x_t from tick 2 on (rt.py:347)
 *   look-ahead  ticks t <= W: the nominal model (nlp_initial, rt.py:300-301); afterwards the
 *               selected model (nlp_bank[current_model_idx], rt.py:303) and the K top-K models,
 *               every candidate, RK4 + the NLP objective (llampc_plan's look-ahead)
 *   mu-hat      warm-up split (rt.py:326-330), then the top-K Dr / Df means (rt.py:331-344)
 * The bank must carry a raceline (llampc_bank_set_raceline) and is driven by the controller
 * from its creation on (its window advances with the ticks). */
typedef struct llampc_ctl_cfg {
  int32_t C, H, K, nan_policy;   /* candidates, horizon (<= LLAMPC_HMAX), top-K, look-back NaN */
  double Ts;
  double v_factor;               /* ConstantSpeed scale once mu-hat is used (rt.py:73: 0.9)  */
  double mu_init;                /* rt.py:327 (1.0)                                          */
  int32_t S;                     /* mu-hat smoothing window (rt.py:68: 20), <= 64            */
  int32_t lap_projidx;           /* rt.py:287 (ETHZ 656, ETHZMobil 440)                      */
  double sigma[2];               /* candidate noise std per input (pwm, steer)              */
  uint64_t seed;
  double nominal[6];             /* warm-up model (Bf, Cf, Df, Br, Cr, Dr), rt.py:207       */
  llampc_cost cost;              /* objective, bounds and rate bound of the look-ahead       */
  int32_t debug_inputs;          /* 1: keep each tick's xref and U (llampc_ctl_inputs)       */
  int32_t reserved;
} llampc_ctl_cfg;

typedef struct llampc_ctl_out {
  llampc_plan_out plan;          /* the tick record (sel_model / sel_cand: the chosen control;
                                    la_best_*: over the rolled-out models only; -1 while warm) */
  int64_t tick;
  int32_t projidx;               /* planner state after this tick (lap wrap applied)         */
  int32_t warm;                  /* 1: planned with the nominal model (tick <= W)            */
  double mu_used, scale_used;    /* curr_mu / scale of this tick's reference                 */
  double mu_pred;                /* mu-hat after this tick (NaN until the first update)      */
  double dr_mean, df_mean;       /* what this tick appended to the Dr / Df histories          */
  double u_seq[LLAMPC_HMAX][2];  /* [H][2]: the chosen control sequence; u_seq[0] is applied  */
} llampc_ctl_out;

typedef struct llampc_ctl llampc_ctl;
/* points [2][np]: the raceline polyline project_fast projects on (track.raceline);
 * prefix [np-1]: prefix[p] = sum of the segment lengths of points 0..p+1 (planner.py:29-36's
 * start arc length for projection index p). */
int llampc_ctl_create(llampc_bank* bank, const llampc_ctl_cfg* cfg, const double* points, int32_t np,
                      const double* prefix, llampc_ctl** out);
/* x_t [6] (host): one control step, blocking; the record comes back through pinned host memory. */
int llampc_ctl_tick(llampc_ctl* ctl, const double* x_t, llampc_ctl_out* out);
/* The same step enqueued (x_t copied into the launch); at most one outstanding per controller;
 * controllers of different banks (e.g. two tracks) overlap on the device. */
int llampc_ctl_tick_async(llampc_ctl* ctl, const double* x_t);
int llampc_ctl_wait(llampc_ctl* ctl, llampc_ctl_out* out);
/* on = 1: every tick also enqueues the NEXT tick's launch behind itself ("armed"): it runs the
 * part of the tick that does not need x_t (the raceline tables, the state, the variates) and
 * then waits on a doorbell in pinned host memory; the next llampc_ctl_tick_async stores x_t and
 * rings it instead of launching, so the launch call and the dispatch leave the control step's
 * latency (rt.py:269-366's step starts when x_t is known).  Results are those of unarmed ticks.
 * While armed, the bank's stream holds that launch: every other call on the bank or the
 * controller cancels it first (it exits untouched; the next tick launches normally and re-arms),
 * as does a tick more than 0.5 s after the arming; an armed launch never rung exits after 2 s.
 * The armed launch must not hold a hardware queue other work shares (a solve or another bank's
 * tick enqueued behind it on that queue would wait for the doorbell): on = 1 gives the bank's
 * own stream a hardware queue of its own (as llampc_bank_set_concurrency(> 1) does) and is
 * refused (LLAMPC_E_STATE) on a bank launching on a caller's stream (llampc_bank_set_stream).
 * With llampc_ctl_set_exchange (peer mailboxes) the armed launch runs the exchange after its
 * doorbell; its mailbox tick number is committed when it fires, so every rank may arm, cancel
 * or launch independently (call set_exchange first).  Not with llampc_ctl_set_gather (two
 * launches per tick; LLAMPC_E_STATE).  on = 0 cancels. */
int llampc_ctl_set_prelaunch(llampc_ctl* ctl, int32_t on);
/* The last completed tick's device time in microseconds: from x_t reaching the device (an armed
 * launch's block 0 seeing the doorbell; else block 0 starting) to the record's stores issued, by
 * the GPU's 100 MHz clock (s_memrealtime).  NaN before the first tick.  Not the step latency:
 * that adds the doorbell / launch and the record's path to the host. */
int llampc_ctl_device_us(llampc_ctl* ctl, double* us);
/* ConstantSpeed (planner.py:12-67) alone on the device with the controller's tables and Ts:
 * x0 [2], v0, horizon H (<= LLAMPC_HMAX), projidx, curr_mu, scale -> xref [2][H+1], the new
 * projidx (no lap wrap) and vr.  Blocking; leaves the controller state alone. */
int llampc_ctl_reference(llampc_ctl* ctl, const double* x0, double v0, int32_t H, int32_t projidx, double curr_mu,
                         double scale, double* xref, int32_t* projidx_out, double* vr);
/* The last tick's reference xref [2][H+1] and candidates U [C][H][2] (cfg.debug_inputs = 1). */
int llampc_ctl_inputs(llampc_ctl* ctl, double* xref, double* U);
/* The controller over a bank SHARDED across ranks (BASELINE config 5: one process per GPU, each
 * rank's controller on its contiguous shard; replaces the single-process loop rt.py:269-366 with
 * its look-back over the whole bank).  Call on every rank before the first tick: `mb` is this
 * rank's mailbox with every peer open (llampc_mailbox_*), `gparams` [6][n_global] the whole
 * bank (rows Bf, Cf, Df, Br, Cr, Dr), copied to the device.  Then on every tick with a full
 * window the look-back's completing block pushes the shard's top-K and argmin (window mean,
 * global index) into every peer's mailbox, merges the `world` records (llampc_ctl_merge's order)
 * and publishes the merged selection: every rank rolls out the same K + 1 models from the global
 * table, so every rank's record and controller state equal the unsharded controller's.  All
 * ranks must tick the same number of times (the mailbox's tick number is the tag); the tick's
 * own launch does the exchange (no second kernel).  world <= 16, n_global < 2^32 - 1. */
int llampc_ctl_set_exchange(llampc_ctl* ctl, llampc_mailbox* mb, const double* gparams, int64_t n_global);
/* The same sharded controller over a GATHER transport (no peer mailbox; world <= 16): every
 * full-window tick is two launches on the bank's stream.  The first runs the look-back and
 * leaves this shard's record — llampc_ctl_record_words(K) words: its top-K and argmin as
 * (window mean, global index) entries, tagged with the exchange's tick number — in device
 * memory; the G records are all-gathered; the second launch merges them (the peer exchange's
 * merge, so the results are the same bitwise) and runs the look-ahead and the completion.
 * comm != NULL: the library issues ncclAllGather between the launches (stream-ordered, no host
 * round trip).  comm == NULL: the caller carries the records — after llampc_ctl_tick_async,
 * llampc_ctl_shard_record(ctl, words, &nw) waits for the first launch and returns this rank's
 * record (nw = 0: this tick has no exchange, e.g. the window is not full; llampc_ctl_wait
 * follows directly), the caller all-gathers the records of ranks 0..world-1 in rank order
 * (any transport) and passes them to llampc_ctl_resume, then llampc_ctl_wait as usual.  A
 * record whose tag does not match (ranks out of step) fails the tick (record status). */
int llampc_ctl_set_gather(llampc_ctl* ctl, int32_t world, int32_t rank, llampc_comm* comm, const double* gparams,
                          int64_t n_global);
int32_t llampc_ctl_record_words(int32_t K);
int llampc_ctl_shard_record(llampc_ctl* ctl, uint64_t* words /* [llampc_ctl_record_words(K)] */, int32_t* nw);
int llampc_ctl_resume(llampc_ctl* ctl, const uint64_t* all_words /* [world][nw] */);
/* The sharded controller's merge on the host (the device exchange runs the same functions,
 * csrc/ctl.hpp): G records of K + 1 entries each — vals / gids [G][K+1], entries 0..K-1 the
 * shard's sorted top-K (gid -1: none), entry K its argmin — -> the merged top-K (argsort order
 * of rt.py:360: NaN last, ties to the lower global index; -1 padded) and argmin (rt.py:359;
 * NaN-first under LLAMPC_NAN_FIRST; -1 if none). */
int llampc_ctl_merge(const double* vals, const int64_t* gids, int32_t G, int32_t K, int32_t nan_policy,
                     int64_t* topk, double* topk_val, int64_t* best, double* best_val);
int llampc_ctl_destroy(llampc_ctl* ctl);

/* ---- setupNLP.solve drop-in ------------------------------------------------------ */
/* The selected model's NMPC (nmpc.py:14-203) on the device: the NLP's Euler transcription of
 * Dynamic.casadi (nmpc.py:58-60, dynamic.py:195-226), its objective (nmpc.py:44-111), the input
 * bounds and the rate bound (nmpc.py:102-105), minimised by the cross-entropy method: `iters`
 * rounds of `samples` sequences drawn from a per-(step, input) normal-like distribution (Philox
 * noise, clipped to the bounds, rate-clipped in order), the `elite` best setting the next mean
 * and std.  Replaces nlpsol/IPOPT (nmpc.py:146-157, 192), which this platform lacks: the
 * optimum is NOT IPOPT's (parity unpinned).  The bank holds the ONE model (n = 1).  Every
 * round runs in one launch (every block completes every round from the others' tagged lists;
 * LLAMPC_NLP_ROUND_LAUNCHES=1 in the environment at create: one launch per round).  The solve's
 * inputs travel as kernel arguments (no host-to-device copy). */
typedef struct llampc_nlp_cfg {
  int32_t H, samples, iters, elite;  /* samples: power of two in [64, 4096]; 1 <= elite <= 64      */
  double Ts;
  double sigma0[2];                  /* the first iteration's std per input                     */
  double std_floor;                  /* added to every elite std                                 */
  uint64_t seed;
  llampc_cost cost;                  /* Q, R, P, bounds; rate_max: the symmetric feasibility bound */
  double rate_lo[2], rate_hi[2];     /* per-step rate bounds already x Ts (min_rates / max_rates x
                                        Ts); rate_lo > rate_hi: none on that input             */
} llampc_nlp_cfg;
typedef struct llampc_nlp llampc_nlp;
int llampc_nlp_create(llampc_bank* bank, const llampc_nlp_cfg* cfg, llampc_nlp** out);
/* x0 [6], xref [2][H+1], uprev [2], base [H][2] (the first mean: the previous solution shifted,
 * or NULL = uprev held); has_hold = 1 adds the held uprev as a candidate of the first round.
 * -> umpc [H][2], fval, xmpc [H+1][6] (the Euler trajectory of umpc).  Blocking. */
int llampc_nlp_solve(llampc_nlp* nlp, const double* x0, const double* xref, const double* uprev,
                     const double* base, int32_t has_hold, double* umpc, double* fval, double* xmpc);
int llampc_nlp_destroy(llampc_nlp* nlp);

/* ---- raw batched dynamics (Dynamic API parity) ---------------------------------- */
/* x [n][6], u [n][2]; params [6][P] with P == 1 (one model broadcast) or P == n.
 * OP_FORCES -> out [5][n] = (Ffy, Frx, Fry, alphaf, alphar)   (dynamic.py:117-154)
 * OP_DERIV  -> out [n][6]                                      (dynamic.py:98-115)
 * device_ptrs: 0 = host arrays (blocking), 1 = device arrays (async on stream). */
int llampc_dynamics_batch(int32_t op, const double* x, const double* u,
                          const double* params, int64_t P, const llampc_vehicle* veh,
                          int64_t n, double* out, int32_t device, int32_t device_ptrs,
                          void* stream);
/* S successive integration steps per lane: x0 [n][6]; u [n][S][2] (u_stride_lane =
 * S*2) or [S][2] broadcast (u_stride_lane = 0); h [S] step sizes; traj_out
 * [S+1][n][6] (full trajectory) or [n][6] (final state only, when final_only=1). */
int llampc_integrate_batch(const double* x0, const double* u, int64_t u_stride_lane,
                           const double* h, int32_t S, const double* params, int64_t P,
                           const llampc_vehicle* veh, int64_t n, int32_t integrator,
                           double* traj_out, int32_t final_only, int32_t device,
                           int32_t device_ptrs, void* stream);

/* ---- model transcendentals (accuracy tests) -------------------------------------- */
/* The fp64 atan2 (x >= 0) / atan / sin / cos the kernels use (csrc/fastmath.hpp),
 * elementwise on host arrays: out[i] = f(a[i][, b[i]]).  0-3: the general versions (any
 * argument); 4-9: the branch-free cores of the rollout stage, defined on their domains only
 * (atan2: |a| + b in [2^-1000, 2^1000], b >= 0; atan: |a| <= 2^1000; sin_wide: |a| <= 3;
 * sincos: |a| <= 2^20 pi/2) — the stage re-does out-of-domain lanes with 0-3; 9 = a / 6. */
enum llampc_math_fn { LLAMPC_MATH_ATAN2_XPOS = 0, LLAMPC_MATH_ATAN = 1, LLAMPC_MATH_SIN = 2,
                      LLAMPC_MATH_COS = 3, LLAMPC_MATH_ATAN2_FAST = 4, LLAMPC_MATH_ATAN_FAST = 5,
                      LLAMPC_MATH_SIN_WIDE = 6, LLAMPC_MATH_SIN_FAST = 7, LLAMPC_MATH_COS_FAST = 8,
                      LLAMPC_MATH_DIV6 = 9,
                      /* the look-ahead's lean cores (fastmath.hpp kAtanRL / kSinWQL) */
                      LLAMPC_MATH_ATAN2_LEAN = 10, LLAMPC_MATH_ATAN_LEAN = 11,
                      LLAMPC_MATH_SIN_WIDE_LEAN = 12,
                      /* the LPM-1 look-ahead lane's paired lean cores (front and rear division
                         through one reciprocal): out[i] = the first result of the pair
                         (a[i], a[n-1-i]) — atan2 with x = b[i], or atan */
                      LLAMPC_MATH_ATAN2_PAIR = 13, LLAMPC_MATH_ATAN_PAIR = 14 };
int llampc_math_batch(int32_t fn, const double* a, const double* b, int64_t n, double* out,
                      int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* LLAMPC_H_ */
