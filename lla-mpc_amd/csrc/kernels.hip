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
#include <hip/hip_runtime.h>
#include <math.h>

#include "kernels.hpp"
#include "merge.hpp"

namespace llampc {

namespace {

template <int NAN_FIRST>
__device__ __forceinline__ bool kless(double av, int64_t ai, double bv, int64_t bi) {
  return NAN_FIRST ? less_nan_first(av, ai, bv, bi) : less_nan_last(av, ai, bv, bi);
}

template <int NAN_FIRST>
__device__ __forceinline__ void wave_min(double& v, int64_t& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off, 64);
    const int64_t oi = __shfl_xor(i, off, 64);
    if (kless<NAN_FIRST>(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
}

// Block-wide min of (v, i); every thread returns the result.  sv/si: 4-entry LDS scratch.
template <int NAN_FIRST>
__device__ __forceinline__ void block_min(double& v, int64_t& i, double* sv, int64_t* si) {
  wave_min<NAN_FIRST>(v, i);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = v;
    si[w] = i;
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
  __syncthreads();
}

__device__ __forceinline__ int block_sum(int x, int32_t* sn) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if ((threadIdx.x & 63) == 0) sn[threadIdx.x >> 6] = x;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) s += sn[k];
  __syncthreads();
  return s;
}

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

// np.mean(window, axis=1) for one model: NumPy's pairwise order (8 partial sums) over the
// ring read oldest -> newest, then / W.  W <= LLAMPC_WMAX (one pairwise block).
__device__ __forceinline__ double window_mean(const double* ring, int64_t ld, int64_t n, int o,
                                              int W) {
  auto at = [&](int i) {
    int s = o + i;
    if (s >= W) s -= W;
    return ring[(int64_t)s * ld + n];
  };
  double s;
  if (W < 8) {
    s = 0.0;
    for (int i = 0; i < W; ++i) s += at(i);
  } else {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = at(j);
    int i = 8;
    for (; i < W - (W % 8); i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += at(i + j);
    }
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < W; ++i) s += at(i);
  }
  return s / W;
}

}  // namespace

// ------------------------------------------------------------------------------------
// Look-back
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void lookback_kernel(LookbackLaunch a) {
  __shared__ double sv[kBlock / 64];
  __shared__ int64_t si[kBlock / 64];
  const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = n < a.n;
  double wm = 0.0;
  if (live) {
    double x[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) x[j] = a.x_prev[j];
    const Input u = make_input(a.u_prev[0], a.u_prev[1]);
    const Tire t = load_tire(a.params, a.n, n);
    rk4_step(a.veh, t, x, u, a.Ts);                       // model.py:32-40, one RK4 step
    double s = 0.0;                                       // rt.py:349 mean over 4 states
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double e = x[j] - a.x_now[j];
      s += e * e;
    }
    const double err = s / 4;
    if (a.err_out) a.err_out[n] = err;
    a.ring[(int64_t)a.slot * a.n + n] = err;             // rt.py:352-353 without np.roll
    if (a.full) {
      const int o = (a.slot + 1 == a.W) ? 0 : a.slot + 1;   // oldest slot
      wm = window_mean(a.ring, a.n, n, o, a.W);           // rt.py:358
      if (a.wmean_out) a.wmean_out[n] = wm;
    }
  }
  if (!a.full) return;  // grid-uniform

  const int64_t gi = live ? a.goff + n : kNoIndex;
  // per-block argmin (rt.py:359)
  double v = live ? wm : (a.nan_first ? __builtin_inf() : __builtin_nan(""));
  int64_t i = gi;
  if (a.nan_first) block_min<1>(v, i, sv, si);
  else block_min<0>(v, i, sv, si);
  if (threadIdx.x == 0) {
    a.am_val[blockIdx.x] = v;
    a.am_idx[blockIdx.x] = i;
  }
  // per-block top-K in argsort order (rt.py:360): K rounds of "next larger key"
  const double mv = live ? wm : __builtin_nan("");
  double lv = 0.0;
  int64_t li = -1;
  for (int k = 0; k < a.K; ++k) {
    double cv = mv;
    int64_t ci = gi;
    if (li >= 0 && !less_nan_last(lv, li, mv, gi)) {
      cv = __builtin_nan("");
      ci = kNoIndex;
    }
    block_min<0>(cv, ci, sv, si);
    if (threadIdx.x == 0) {
      a.tk_val[(int64_t)blockIdx.x * a.K + k] = cv;
      a.tk_idx[(int64_t)blockIdx.x * a.K + k] = ci;
    }
    lv = cv;
    li = ci;
  }
}

// ------------------------------------------------------------------------------------
// Look-ahead
// ------------------------------------------------------------------------------------
// Dynamic LDS carve (16-B aligned offsets, cdna_hip_programming.md G17):
//   [0, 32)  sv[4] double  | [32, 64) si[4] int64 | [64, 80) sn[4] int32 | pad to 96
//   [96, 96 + 16(H+1))     xref as [k][2]
//   [.., + 16*C*H)         U as [k][c][2] when staged (consecutive c -> consecutive 16 B)
constexpr int kScratchBytes = 96;

template <int INTEG, bool STAGE>
__global__ __launch_bounds__(kBlock) void lookahead_kernel(LookaheadLaunch a, int G, int cpl) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* sv = reinterpret_cast<double*>(smem);
  int64_t* si = reinterpret_cast<int64_t*>(smem + 32);
  int32_t* sn = reinterpret_cast<int32_t*>(smem + 64);
  double* sx = reinterpret_cast<double*>(smem + kScratchBytes);
  double* su = sx + 2 * (a.H + 1);

  const int H = a.H, C = a.C;
  for (int e = threadIdx.x; e <= H; e += kBlock) {
    sx[2 * e] = a.xref[e];
    sx[2 * e + 1] = a.xref[(H + 1) + e];
  }
  if (STAGE) {
    for (int e = threadIdx.x; e < C * H; e += kBlock) {
      const int c = e / H, k = e - c * H;
      su[2 * (k * C + c)] = a.U[2 * e];
      su[2 * (k * C + c) + 1] = a.U[2 * e + 1];
    }
  }
  __syncthreads();

  const int g = threadIdx.x & (G - 1);
  const int64_t n = (int64_t)blockIdx.x * (kBlock / G) + threadIdx.x / G;
  const bool live = n < a.n;
  const CostK& q = a.cost;
  const double up0 = a.uprev[0], up1 = a.uprev[1];

  double bv = __builtin_nan("");
  int64_t bc = kNoIndex;
  int nf = 0;
  if (live) {
    const Tire t = load_tire(a.params, a.n, n);
    for (int j = 0; j < cpl; ++j) {
      const int c = g + j * G;
      if (c >= C) break;
      double x[6];
#pragma unroll
      for (int m = 0; m < 6; ++m) x[m] = a.x0[m];
      double track = 0.0, act = 0.0;
      double p0 = up0, p1 = up1;
      bool feas = true;
      for (int k = 0; k < H; ++k) {
        double ua, ud;
        if (STAGE) {
          ua = su[2 * (k * C + c)];
          ud = su[2 * (k * C + c) + 1];
        } else {
          ua = a.U[2 * ((int64_t)c * H + k)];
          ud = a.U[2 * ((int64_t)c * H + k) + 1];
        }
        const double d0 = ua - p0, d1 = ud - p1;          // nmpc.py:65-68
        if (q.enforce) {                                  // nmpc.py:102-105
          feas = feas && ua <= q.umax[0] && ua >= q.umin[0] && ud <= q.umax[1] &&
                 ud >= q.umin[1];
          if (q.dmax[0] >= 0) feas = feas && d0 <= q.dmax[0] && -d0 <= q.dmax[0];
          if (q.dmax[1] >= 0) feas = feas && d1 <= q.dmax[1] && -d1 <= q.dmax[1];
        }
        const Input u = make_input(ua, ud);
        step<INTEG>(a.veh, t, x, u, a.Ts);
        const double e0 = x[0] - sx[2 * (k + 1)], e1 = x[1] - sx[2 * (k + 1) + 1];
        track = track + (e0 * (q.Q[0] * e0 + q.Q[1] * e1) + e1 * (q.Q[2] * e0 + q.Q[3] * e1));
        act = act + (d0 * (q.R[0] * d0 + q.R[1] * d1) + d1 * (q.R[2] * d0 + q.R[3] * d1));
        p0 = ua;
        p1 = ud;
      }
      const double e0 = x[0] - sx[2 * H], e1 = x[1] - sx[2 * H + 1];   // nmpc.py:48
      const double term = e0 * (q.P[0] * e0 + q.P[1] * e1) + e1 * (q.P[2] * e0 + q.P[3] * e1);
      double J = (term + track) + act;                                // nmpc.py:111
      if (!feas) J = __builtin_inf();
      if (a.cost_out) a.cost_out[n * C + c] = J;
      nf += !isfinite(J);
      if (less_nan_last(J, c, bv, bc)) {
        bv = J;
        bc = c;
      }
    }
  }
  // per-model argmin over its candidates: xor-shuffles inside the G-lane group
  for (int off = G >> 1; off > 0; off >>= 1) {
    const double ov = __shfl_xor(bv, off, 64);
    const int64_t oc = __shfl_xor(bc, off, 64);
    if (less_nan_last(ov, oc, bv, bc)) {
      bv = ov;
      bc = oc;
    }
  }
  if (live && g == 0) {
    a.best_cand[n] = (int32_t)bc;
    a.best_cost[n] = bv;
  }
  // per-block argmin over (model, candidate) in flattened order (goff+n)*C + c
  int64_t key = (live && bc != kNoIndex) ? (a.goff + n) * C + bc : kNoIndex;
  double v = (key == kNoIndex) ? __builtin_nan("") : bv;
  block_min<0>(v, key, sv, si);
  const int nfs = block_sum(nf, sn);
  if (threadIdx.x == 0) {
    a.pv[blockIdx.x] = v;
    a.pidx[blockIdx.x] = key;
    a.pnf[blockIdx.x] = nfs;
  }
}

// ------------------------------------------------------------------------------------
// Select: merge per-block partials into the tick's llampc_plan_out
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void select_kernel(SelectLaunch a) {
  __shared__ double sv[kBlock / 64];
  __shared__ int64_t si[kBlock / 64];
  __shared__ int32_t sn[kBlock / 64];
  __shared__ int64_t s_top[LLAMPC_KMAX];
  __shared__ double s_topv[LLAMPC_KMAX];
  const int tid = threadIdx.x;
  const bool lb = a.do_lb && a.full;

  double lbv = __builtin_nan("");
  int64_t lbi = -1;
  if (lb) {
    double v = a.nan_first ? __builtin_inf() : __builtin_nan("");
    int64_t i = kNoIndex;
    for (int b = tid; b < a.lb_blocks; b += kBlock) {
      if (a.am_idx[b] == kNoIndex) continue;
      if (key_less(a.nan_first, a.am_val[b], a.am_idx[b], v, i)) {
        v = a.am_val[b];
        i = a.am_idx[b];
      }
    }
    if (a.nan_first) block_min<1>(v, i, sv, si);
    else block_min<0>(v, i, sv, si);
    if (i != kNoIndex) {
      lbv = v;
      lbi = i;
    }
    double lv = 0.0;
    int64_t li = -1;
    const int M = a.lb_blocks * a.K;
    for (int k = 0; k < a.K; ++k) {
      double cv = __builtin_nan("");
      int64_t ci = kNoIndex;
      for (int e = tid; e < M; e += kBlock) {
        const int64_t idx = a.tk_idx[e];
        if (idx == kNoIndex) continue;
        const double val = a.tk_val[e];
        if (li >= 0 && !less_nan_last(lv, li, val, idx)) continue;
        if (less_nan_last(val, idx, cv, ci)) {
          cv = val;
          ci = idx;
        }
      }
      block_min<0>(cv, ci, sv, si);
      if (tid == 0) {
        s_top[k] = ci;
        s_topv[k] = cv;
      }
      lv = cv;
      li = ci;
    }
  }

  double lav = __builtin_nan("");
  int64_t lai = kNoIndex;
  int nf = 0;
  if (a.do_la) {
    for (int b = tid; b < a.la_blocks; b += kBlock) {
      nf += a.pnf[b];
      if (a.pidx[b] == kNoIndex) continue;
      if (less_nan_last(a.pv[b], a.pidx[b], lav, lai)) {
        lav = a.pv[b];
        lai = a.pidx[b];
      }
    }
    block_min<0>(lav, lai, sv, si);
    nf = block_sum(nf, sn);
  }
  __syncthreads();

  if (tid != 0) return;
  llampc_plan_out* o = a.out;
  o->window_count = a.window_count;
  o->window_full = a.full;
  o->K = a.K;
  o->lb_best = lbi;
  o->lb_best_val = lbv;
  o->n_nonfinite = nf;
  o->reserved = 0;
  const int64_t sel = lb && lbi >= 0 ? lbi : a.current_model;
  const bool owned = sel >= a.goff && sel < a.goff + a.n;
  o->sel_model = sel;
  o->sel_owned = owned;
  o->sel_cand = (owned && a.do_la) ? a.best_cand[sel - a.goff] : -1;
  o->sel_cost = (owned && a.do_la) ? a.best_cost[sel - a.goff] : __builtin_nan("");
  if (a.do_la && lai != kNoIndex) {
    o->la_best_model = lai / a.C;
    o->la_best_cand = (int32_t)(lai % a.C);
    o->la_best_cost = lav;
  } else {
    o->la_best_model = -1;
    o->la_best_cand = -1;
    o->la_best_cost = __builtin_nan("");
  }
  for (int k = 0; k < LLAMPC_KMAX; ++k) {
    const bool have = lb && k < a.K && s_top[k] != kNoIndex;
    if (!have) {
      o->topk[k] = -1;
      o->topk_val[k] = o->topk_Df[k] = o->topk_Dr[k] = o->topk_cost[k] = __builtin_nan("");
      o->topk_cand[k] = -1;
      continue;
    }
    const int64_t gi = s_top[k], li = gi - a.goff;
    o->topk[k] = gi;
    o->topk_val[k] = s_topv[k];
    o->topk_Df[k] = a.params[2 * a.n + li];
    o->topk_Dr[k] = a.params[5 * a.n + li];
    o->topk_cand[k] = a.do_la ? a.best_cand[li] : -1;
    o->topk_cost[k] = a.do_la ? a.best_cost[li] : __builtin_nan("");
  }
}

__global__ void merge_kernel(const llampc_plan_out* parts, int32_t G, int32_t nan_first,
                             llampc_plan_out* merged) {
  if (threadIdx.x == 0 && blockIdx.x == 0) merge_plan_parts(parts, G, nan_first, merged);
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

int lookahead_group(int32_t C) {
  int G = 1;
  while (G < C && G < 64) G <<= 1;
  return G;
}

int lookahead_blocks(int64_t n, int32_t C) {
  const int mpb = kBlock / lookahead_group(C);
  return (int)((n + mpb - 1) / mpb);
}

constexpr size_t kStageLimit = 48 * 1024;

size_t lookahead_lds_bytes(int32_t C, int32_t H, bool* stage_u) {
  const size_t base = kScratchBytes + 16 * (size_t)(H + 1);
  const size_t ub = 16 * (size_t)C * H;
  *stage_u = base + ub <= kStageLimit;
  return *stage_u ? base + ub : base;
}

hipError_t launch_lookback(const LookbackLaunch& a, hipStream_t s) {
  const int nb = lookback_blocks(a.n);
  hipLaunchKernelGGL(lookback_kernel, dim3(nb), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <int INTEG>
static void launch_la_integ(const LookaheadLaunch& a, hipStream_t s, int nb, int G, int cpl,
                            bool stage, size_t lds) {
  if (stage)
    hipLaunchKernelGGL((lookahead_kernel<INTEG, true>), dim3(nb), dim3(kBlock), lds, s, a, G, cpl);
  else
    hipLaunchKernelGGL((lookahead_kernel<INTEG, false>), dim3(nb), dim3(kBlock), lds, s, a, G, cpl);
}

hipError_t launch_lookahead(const LookaheadLaunch& a, hipStream_t s) {
  const int G = lookahead_group(a.C);
  const int cpl = (a.C + G - 1) / G;
  const int nb = lookahead_blocks(a.n, a.C);
  bool stage = false;
  const size_t lds = lookahead_lds_bytes(a.C, a.H, &stage);
  switch (a.integrator) {
    case LLAMPC_RK4: launch_la_integ<0>(a, s, nb, G, cpl, stage, lds); break;
    case LLAMPC_EULER_NLP: launch_la_integ<1>(a, s, nb, G, cpl, stage, lds); break;
    case LLAMPC_RK6: launch_la_integ<2>(a, s, nb, G, cpl, stage, lds); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_select(const SelectLaunch& a, hipStream_t s) {
  hipLaunchKernelGGL(select_kernel, dim3(1), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_merge(const llampc_plan_out* parts, int32_t G, int32_t nan_first,
                        llampc_plan_out* merged, hipStream_t s) {
  hipLaunchKernelGGL(merge_kernel, dim3(1), dim3(64), 0, s, parts, G, nan_first, merged);
  return hipGetLastError();
}

hipError_t launch_dynamics(int32_t op, const double* x, const double* u, const double* params,
                           int64_t P, VehK veh, int64_t n, double* out, hipStream_t s) {
  const int nb = (int)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(dynamics_kernel, dim3(nb), dim3(kBlock), 0, s, op, x, u, params, P, veh, n, out);
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
