// merge.hpp — deterministic cross-shard merge of llampc_plan_out records.
// Compiled both for the device (llampc_merge_device, run after the RCCL all-gather) and
// for the host (llampc_merge), so the CPU tests exercise the exact code the GPUs run.
//
// Semantics = the unsharded reference on the concatenated bank:
//   lb_best  = np.argmin(avg_errors)          (rt.py:359; NaN-first under NAN_FIRST)
//   topk     = avg_errors.argsort()[:K]       (rt.py:360; NaN last; ties -> lower index)
//   la_best  = argmin over all (model, cand)  (NaN treated as +inf)
#pragma once
#include "dyn.hpp"
#include "llampc.h"

namespace llampc {

__device__ __host__ __forceinline__ bool la_less(double av, int64_t am, int32_t ac, double bv,
                                                 int64_t bm, int32_t bc) {
  const bool an = av != av, bn = bv != bv;
  if (an | bn) {
    if (!(an & bn)) return bn;
  } else if (av != bv) {
    return av < bv;
  }
  return (am < bm) || (am == bm && ac < bc);
}

__device__ __host__ inline void merge_plan_parts(const llampc_plan_out* parts, int G,
                                                 int nan_first, llampc_plan_out* m) {
  const llampc_plan_out& p0 = parts[0];
  m->window_count = p0.window_count;
  m->window_full = p0.window_full;
  m->K = p0.K;
  m->status = 0;
  for (int g = 0; g < G; ++g) m->status |= parts[g].status;

  // look-back argmin
  double bv = nan_first ? __builtin_inf() : __builtin_nan("");
  int64_t bi = kNoIndex;
  int owner = -1;
  for (int g = 0; g < G; ++g) {
    if (parts[g].lb_best < 0) continue;
    if (key_less(nan_first, parts[g].lb_best_val, parts[g].lb_best, bv, bi)) {
      bv = parts[g].lb_best_val;
      bi = parts[g].lb_best;
      owner = g;
    }
  }
  m->lb_best = owner >= 0 ? bi : -1;
  m->lb_best_val = owner >= 0 ? bv : __builtin_nan("");

  // selected model and its look-ahead choice
  if (m->window_full && owner >= 0) {
    m->sel_model = bi;
    m->sel_owned = parts[owner].sel_owned;
    m->sel_cand = parts[owner].sel_cand;
    m->sel_cost = parts[owner].sel_cost;
  } else {
    m->sel_model = p0.sel_model;
    m->sel_owned = 0;
    m->sel_cand = -1;
    m->sel_cost = __builtin_nan("");
    for (int g = 0; g < G; ++g) {
      if (parts[g].sel_owned) {
        m->sel_owned = 1;
        m->sel_cand = parts[g].sel_cand;
        m->sel_cost = parts[g].sel_cost;
        break;
      }
    }
  }

  // top-K: K rounds of "smallest key greater than the previous pick" (NaN last)
  const int K = p0.K;
  double lv = 0.0;
  int64_t li = -1;
  for (int k = 0; k < K; ++k) {
    double cv = __builtin_nan("");
    int64_t ci = kNoIndex;
    int cg = -1, cj = -1;
    for (int g = 0; g < G; ++g) {
      for (int j = 0; j < K; ++j) {
        const int64_t idx = parts[g].topk[j];
        if (idx < 0) continue;
        const double val = parts[g].topk_val[j];
        if (li >= 0 && !less_nan_last(lv, li, val, idx)) continue;
        if (less_nan_last(val, idx, cv, ci)) {
          cv = val;
          ci = idx;
          cg = g;
          cj = j;
        }
      }
    }
    if (cg < 0) {
      for (int r = k; r < K; ++r) {
        m->topk[r] = -1;
        m->topk_val[r] = __builtin_nan("");
        m->topk_Df[r] = m->topk_Dr[r] = m->topk_cost[r] = __builtin_nan("");
        m->topk_cand[r] = -1;
      }
      break;
    }
    m->topk[k] = ci;
    m->topk_val[k] = cv;
    m->topk_Df[k] = parts[cg].topk_Df[cj];
    m->topk_Dr[k] = parts[cg].topk_Dr[cj];
    m->topk_cand[k] = parts[cg].topk_cand[cj];
    m->topk_cost[k] = parts[cg].topk_cost[cj];
    lv = cv;
    li = ci;
  }
  for (int r = K; r < LLAMPC_KMAX; ++r) {
    m->topk[r] = -1;
    m->topk_val[r] = m->topk_Df[r] = m->topk_Dr[r] = m->topk_cost[r] = 0.0;
    m->topk_cand[r] = -1;
  }

  // global look-ahead best and non-finite count
  double av = __builtin_nan("");
  int64_t am = kNoIndex;
  int32_t ac = INT32_MAX;
  int nf = 0;
  for (int g = 0; g < G; ++g) {
    nf += parts[g].n_nonfinite;
    if (parts[g].la_best_model < 0) continue;
    if (la_less(parts[g].la_best_cost, parts[g].la_best_model, parts[g].la_best_cand, av, am, ac)) {
      av = parts[g].la_best_cost;
      am = parts[g].la_best_model;
      ac = parts[g].la_best_cand;
    }
  }
  m->la_best_model = am == kNoIndex ? -1 : am;
  m->la_best_cand = am == kNoIndex ? -1 : ac;
  m->la_best_cost = av;
  m->n_nonfinite = nf;
}

}  // namespace llampc
