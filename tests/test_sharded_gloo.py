"""N>1 path on CPU: world_size-2 gloo processes each produce their shard's llampc_plan_out
record (the oracle stands in for the GPU kernels here — test infrastructure), exchange
them with the product's ``gather_merge_host`` (one all-gather) and must reproduce the
unsharded look-back selection / top-K / look-ahead best on every rank."""
import datetime
import os
import shutil
import sys
import tempfile

import numpy as np
import pytest

from conftest import REPO, PKG_ROOT, golden

TS = 0.02


def _local_record(nat, p_all, lo, hi, states, inputs, W, K, U, xref, uprev):
    """Shard [lo, hi) record computed with the oracle (what the GPU kernels produce)."""
    from oracle import llampc_oracle as O
    pp = O.orca_params()
    shared = {k: pp[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
    p = p_all[:, lo:hi]
    win = O.LookbackWindow(hi - lo, W, K)
    for t in range(W):
        e = O.lookback_errors(O.evaluate_models_vectorized(shared, tuple(p), states[:, t], inputs[:, t], TS), states[:, t + 1])
        win.push(e)
    x_now = states[:, W]
    traj = O.rollout_rk4(shared, tuple(p), x_now, U, TS)
    C = U.shape[0]
    cost = O.mpc_cost(traj, U, xref, uprev, np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))).reshape(-1, C)
    o = nat.PlanOut()
    o.window_count, o.window_full, o.K = win.count, 1, K
    j = int(np.argmin(win.avg))
    o.lb_best, o.lb_best_val = lo + j, win.avg[j]
    bc = np.argmin(cost, axis=1)
    o.sel_model, o.sel_owned, o.sel_cand, o.sel_cost = lo + j, 1, int(bc[j]), cost[j, bc[j]]
    top = win.best_k
    for k in range(nat.KMAX):
        if k < K:
            i = top[k]
            o.topk[k], o.topk_val[k] = lo + i, win.avg[i]
            o.topk_Df[k], o.topk_Dr[k] = p[2, i], p[5, i]
            o.topk_cand[k], o.topk_cost[k] = int(bc[i]), cost[i, bc[i]]
        else:
            o.topk[k], o.topk_cand[k] = -1, -1
    f = int(np.argmin(cost.ravel()))
    o.la_best_model, o.la_best_cand, o.la_best_cost = lo + f // C, f % C, cost.ravel()[f]
    o.n_nonfinite = int((~np.isfinite(cost)).sum())
    return o, win, cost


def _worker(rank, world, store, q):
    try:
        for pth in (REPO, PKG_ROOT):
            sys.path.insert(0, pth)
        import torch.distributed as dist
        from llampc import _native as nat
        from llampc.mpc import generate_bank, shard_range
        from llampc.mpc.sharded import gather_merge_host
        dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=120))
        d = golden("dyn_slice.npz")
        N, W, K, H, C = 601, 10, 10, 20, 3
        p = generate_bank(N, seed=0)
        s, u = d["states"], d["inputs"]
        U = np.repeat(u[:, W:W + H].T[None], C, axis=0)
        U[:, :, 1] += np.array([-0.01, 0.0, 0.01])[:, None]
        xref = s[:2, W:W + H + 1] + 0.02
        lo, hi = shard_range(N, rank, world)
        local, _, _ = _local_record(nat, p, lo, hi, s, u, W, K, U, xref, u[:, W - 1])
        merged = nat.plan_out_to_dict(gather_merge_host(local))
        ref, win, cost = _local_record(nat, p, 0, N, s, u, W, K, U, xref, u[:, W - 1])
        ref = nat.plan_out_to_dict(ref)
        for k in ("lb_best", "sel_model", "sel_cand", "la_best_model", "la_best_cand", "n_nonfinite"):
            assert merged[k] == ref[k], (k, merged[k], ref[k])
        for k in ("topk", "topk_val", "topk_Df", "topk_Dr", "topk_cand", "topk_cost"):
            np.testing.assert_array_equal(merged[k], ref[k])
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


def run_gloo_ranks(target, world, timeout=240):
    """``target(rank, world, store, q)`` in `world` spawned processes meeting at a FileStore in a
    private temporary directory (no TCP port to race for); each puts (rank, "ok" | error) on q.
    Every rank process is reaped whatever happens."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    tmp = tempfile.mkdtemp(prefix="llampc_rdzv_")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, os.path.join(tmp, "store"), q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = []
    try:
        for _ in procs:
            res.append(q.get(timeout=timeout))
            if res[-1][1] != "ok":
                break
    finally:
        failed = any(msg != "ok" for _, msg in res)
        for pr in procs:
            pr.join(timeout=1 if failed else 60)
            if pr.is_alive():
                pr.terminate()
                pr.join(timeout=10)
        shutil.rmtree(tmp, ignore_errors=True)
    bad = [(rank, msg) for rank, msg in res if msg != "ok"]
    if bad:
        raise AssertionError(f"rank {bad[0][0]}: {bad[0][1]}")


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merge_gloo(world):
    run_gloo_ranks(_worker, world)


def _ctl_merge_worker(rank, world, store, q):
    """One rank of the sharded controller's selection (ctl.hpp "sharded controller"): its shard's
    window (the oracle stands in for the look-back kernel), its record — the sorted top-K and the
    argmin as (window mean, global index) — gathered over gloo and merged by the product's
    llampc_ctl_merge (the functions the device exchange runs): every rank must hold the
    unsharded argmin (np.argmin: first NaN) and top-K (stable argsort: NaN last, ties to the
    lower index), on a bank with exact ties across shards and NaN models."""
    try:
        for pth in (REPO, PKG_ROOT):
            sys.path.insert(0, pth)
        import torch.distributed as dist
        from llampc import _native as nat
        from llampc.mpc import generate_bank, shard_range
        from llampc.mpc.sharded import merge_ctl_records
        from oracle import llampc_oracle as O
        dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=120))
        d = golden("dyn_slice.npz")
        s, u = d["states"], d["inputs"]
        pp = O.orca_params()
        shared = {k: pp[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
        N, W, K = 907, 4, 10
        b0 = None
        for case in ("plain", "ties", "nan"):
            p = generate_bank(N, seed=31)
            if case == "ties":             # copies of the best model in every shard: equal means
                p[:, [c for c in (5, 300, 301, 620, 906) if c != b0]] = p[:, [b0]]
            elif case == "nan":            # NaN models in two shards: argmin = the first NaN
                p[2, [777, 150]] = np.nan
            with np.errstate(all="ignore"):
                errs = [O.lookback_errors(O.evaluate_models_vectorized(shared, tuple(p), s[:, t], u[:, t], TS), s[:, t + 1])
                        for t in range(W)]
            full = O.LookbackWindow(N, W, K)
            for e in errs:
                full.push(e)
            if case == "plain":
                b0 = full.current
            lo, hi = shard_range(N, rank, world)
            avg = full.avg[lo:hi]          # the shard's own window means (same values)
            order = np.argsort(avg, kind="stable")[:K]
            vals = np.full(K + 1, np.nan)
            gids = np.full(K + 1, -1, dtype=np.int64)
            vals[:order.size], gids[:order.size] = avg[order], order + lo
            vals[K], gids[K] = avg[int(np.argmin(avg))], int(np.argmin(avg)) + lo
            parts = [None] * world
            dist.all_gather_object(parts, (vals, gids))
            topk, tv, best, bv = merge_ctl_records(np.stack([a for a, _ in parts]), np.stack([b for _, b in parts]),
                                                   nat.NAN_FIRST)
            want = np.argsort(full.avg, kind="stable")[:K]
            np.testing.assert_array_equal(topk, want, err_msg=case)
            np.testing.assert_array_equal(tv, full.avg[want])
            assert best == int(np.argmin(full.avg)), (case, best)
            if case == "nan":
                assert best == 150 and np.isnan(bv)
            if case == "ties":             # the copies' equal means did meet in the merge
                assert np.sum(full.avg[topk] == full.avg[b0]) >= 5, topk
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_controller_merge_gloo(world):
    run_gloo_ranks(_ctl_merge_worker, world)
