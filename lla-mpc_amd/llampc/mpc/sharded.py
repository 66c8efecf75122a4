"""Model bank sharded over the GPUs of one node (one process per GPU).

The bank partitions into contiguous shards of independent models (bank.shard_range);
each rank runs the fused tick on its shard and contributes one fixed-size
``llampc_plan_out`` record (~1.1 KB: top-K with values, Df/Dr and each top-K model's best
look-ahead candidate, the local argmin, the selected model's choice, the look-ahead best).
ONE all-gather per tick (RCCL over xGMI with the "nccl" backend) moves the records, and
every rank runs the same deterministic merge (csrc/merge.hpp) on the device — so all ranks
hold the identical result of the unsharded computation.  There is no other data-path
collective.  With the "gloo" backend (CPU tests) the records travel as CPU tensors and the
same merge code runs on the host (llampc_merge).

Transports of the exchange (LLAMPC_EXCHANGE; the merged record is the same for all):
  peer  (default when it verifies) — no collective library: every rank's mailbox (uncached
        device memory) is mapped into every peer through HIP IPC, and the tick's own plan
        launch, once its record is complete, pushes it into all mailboxes over xGMI, polls its
        own until the tick's records have arrived and merges (llampc_plan_exchange: one launch
        per rank per tick; LLAMPC_PEER_SPLIT=1 runs the exchange as a second kernel).  Set up with one
        all_gather_object of the IPC handles on any backend (gloo included), then checked by a
        probe exchange against the host merge; on any failure every rank falls back together.
  rccl  — ncclAllGather on the tick stream over the library's own communicator (llampc_comm_*:
        ncclGetUniqueId on rank 0, shared through the process group, ncclCommInitRank on every
        rank; the RCCL the process already holds) + merge_kernel.
  c10d  — torch.distributed.all_gather_into_tensor + merge_kernel.
  host  — (gloo) records gathered on the host, merged by merge_kernel.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from llampc import _native as nat
from llampc.mpc.bank import ModelBank, shard_range
from llampc.mpc.plan import PlanResult, result_from_out


def _bytes_of(o: nat.PlanOut) -> np.ndarray:
    return np.frombuffer(C.string_at(C.addressof(o), nat.PLAN_OUT_BYTES), dtype=np.uint8).copy()


def _out_of(b: np.ndarray) -> nat.PlanOut:
    return nat.PlanOut.from_buffer_copy(np.ascontiguousarray(b, dtype=np.uint8).tobytes())


def _all_gather_obj(obj, group=None) -> list:
    import torch.distributed as dist
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def exchange_mode() -> str:
    """LLAMPC_EXCHANGE = auto (peer, else rccl/c10d/host) | peer (required) | rccl | c10d | host;
    LLAMPC_C10D_EXCHANGE=1 is the older spelling of c10d."""
    if os.environ.get("LLAMPC_C10D_EXCHANGE"):
        return "c10d"
    m = os.environ.get("LLAMPC_EXCHANGE", "auto")
    if m not in ("auto", "peer", "rccl", "c10d", "host"):
        raise ValueError(f"LLAMPC_EXCHANGE={m!r}: auto | peer | rccl | c10d | host")
    return m


def probe_record(rank: int, world: int, K: int = 10) -> nat.PlanOut:
    """A synthetic shard record for checking a transport: distinct global indices per rank,
    sorted top-K values, one NaN-free look-ahead best (deterministic in rank)."""
    rng = np.random.RandomState(7919 + rank)
    o = nat.PlanOut()
    o.window_count, o.window_full, o.K, o.sel_owned = 10, 1, K, int(rank == 0)
    vals = np.sort(rng.uniform(0.0, 1.0, K))
    for j in range(nat.KMAX):
        o.topk[j] = rank * 1000 + j if j < K else -1
        o.topk_val[j] = vals[j] if j < K else 0.0
        o.topk_Df[j] = o.topk_Dr[j] = o.topk_cost[j] = float(rank + j) if j < K else 0.0
        o.topk_cand[j] = j if j < K else -1
    o.lb_best, o.lb_best_val = rank * 1000, vals[0]
    o.sel_model, o.sel_cand, o.sel_cost = 0, 1, 0.5
    o.la_best_model, o.la_best_cand, o.la_best_cost = rank * 1000 + 3, rank, float(rng.uniform())
    o.n_nonfinite, o.status = rank, 0
    return o


def merge_ctl_records(vals, gids, nan_policy=nat.NAN_FIRST):
    """The sharded controller's merge on the host (llampc_ctl_merge: the functions the device
    exchange runs).  vals / gids [G, K+1]: each shard's sorted top-K (global index -1: none) and,
    last, its argmin.  -> (topk [K] (-1 padded), topk_val [K], best, best_val)."""
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    gids = np.ascontiguousarray(gids, dtype=np.int64)
    G, K1 = vals.shape
    K = K1 - 1
    topk = np.empty(K, dtype=np.int64)
    tv = np.empty(K)
    best, bv = C.c_int64(), C.c_double()
    nat.check(nat.load().llampc_ctl_merge(nat.dptr(vals), gids.ctypes.data, G, K, int(nan_policy), topk.ctypes.data,
                                          nat.dptr(tv), C.byref(best), C.byref(bv)))
    return topk, tv, best.value, bv.value


def records_equal(a: nat.PlanOut, b: nat.PlanOut) -> bool:
    A, B = nat.plan_out_to_dict(a), nat.plan_out_to_dict(b)
    for k in B:
        x, y = np.asarray(A[k]), np.asarray(B[k])
        if x.shape != y.shape or not np.array_equal(x, y, equal_nan=x.dtype.kind == "f"):
            return False
    return True


def gather_merge_host(local: nat.PlanOut, group=None, nan_policy=nat.NAN_FIRST) -> nat.PlanOut:
    """All-gather the shard records over a CPU (gloo) group and merge on the host."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.from_numpy(_bytes_of(local))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return nat.merge([_out_of(p.numpy()) for p in parts], nan_policy)


class ShardedBank:
    """This rank's shard of a global bank, plus the per-tick exchange."""

    def __init__(self, params_global, rank: int, world: int, device: int, W: int = 10,
                 group=None, shared=None):
        import torch
        import torch.distributed as dist
        params_global = np.ascontiguousarray(params_global, dtype=np.float64)
        self.params_global = params_global     # the sharded controller's replicated table
        self.n_global = params_global.shape[1]
        self.rank, self.world, self.device, self.group = rank, world, device, group
        lo, hi = shard_range(self.n_global, rank, world)
        self.lo, self.hi = lo, hi
        self.bank = ModelBank(params_global[:, lo:hi], shared=shared, W=W, device=device, global_offset=lo)
        self.backend = dist.get_backend(group) if (dist.is_available() and dist.is_initialized()) else None
        dev = torch.device("cuda", device)
        B = nat.PLAN_OUT_BYTES
        self._torch = torch
        self.d_local = torch.empty(B, dtype=torch.uint8, device=dev)
        self.d_all = torch.empty(B * world, dtype=torch.uint8, device=dev)
        # one shard: its record IS the result (no gather, no merge launch).
        # LLAMPC_FORCE_EXCHANGE=1 runs the exchange anyway (a 1-rank group): measures the
        # collective + merge cost per tick on one GPU (diagnostic)
        import os
        self.exchange = world > 1 or (self.backend is not None and bool(os.environ.get("LLAMPC_FORCE_EXCHANGE")))
        self.d_merged = torch.empty(B, dtype=torch.uint8, device=dev) if self.exchange else self.d_local
        self.h_merged = torch.empty(B, dtype=torch.uint8).pin_memory()
        self._inputs = None
        # every stage of the tick (input upload, plan, all-gather, merge, read-back) runs on
        # ONE stream, which is also the bank's: torch's default stream has handle 0, which the
        # C ABI reads as "the bank's own stream", so it is never used to launch a tick.  A
        # torch stream, not the bank's own wrapped as an ExternalStream: torch's caching
        # allocator keeps using the streams its blocks were used on after the shard is closed
        # (the self-spawned 2-rank bench crashed at the end with the bank's stream destroyed)
        self.stream = torch.cuda.Stream(device=dev)
        self.bank.set_stream(self.stream.cuda_stream)
        # native exchange: the all-gather is issued by llampc_exchange_rccl straight on the
        # tick's stream over the library's own RCCL communicator — no c10d stream hand-off,
        # ~1 us of host time per tick.  LLAMPC_C10D_EXCHANGE=1 keeps the c10d call.
        self._comm = None
        self._mailbox = None
        self.transport = None
        self.fallback_reason = None        # why a preferred transport was not taken (reported)
        if self.exchange:
            mode = exchange_mode()
            if mode in ("auto", "peer"):
                self._setup_peer_exchange(dev, required=mode == "peer")
            if self._mailbox is None and ((self.backend == "nccl" and mode == "auto") or mode == "rccl"):
                self._setup_native_exchange(dev)
            self.transport = self._decide_transport()

    def _decide_transport(self) -> str:
        """The exchange the ticks use, from what the collective setup left: the peer mailboxes,
        else the native RCCL all-gather, else c10d's (nccl), else the host gather (gloo)."""
        return ("peer" if self._mailbox is not None else "rccl" if self._comm is not None
                else "c10d" if self.backend == "nccl" else "host")

    def _setup_peer_exchange(self, dev, required=False):
        """Map every rank's mailbox (collective: all ranks take the same decision)."""
        import sys
        import torch
        lib = nat.load()
        mb = C.c_void_p()
        err, handle = None, b""
        try:
            nat.check(lib.llampc_mailbox_create(self.world, self.rank, self.device, C.byref(mb)))
            h = (C.c_ubyte * 64)()
            nat.check(lib.llampc_mailbox_ipc_handle(mb, h))
            handle = bytes(h)
        except Exception as e:                     # noqa: BLE001 — decided collectively below
            err = e
        handles = _all_gather_obj(handle, self.group)
        if err is None and all(handles):
            try:
                for g, hg in enumerate(handles):
                    if g != self.rank:
                        nat.check(lib.llampc_mailbox_open_peer(mb, g, (C.c_ubyte * 64).from_buffer_copy(hg)))
            except Exception as e:                 # noqa: BLE001
                err = e
        ok = all(_all_gather_obj(err is None, self.group))
        if ok:                                     # probe exchange vs the host merge
            rec = probe_record(self.rank, self.world)
            parts = [_out_of(np.frombuffer(b, dtype=np.uint8))
                     for b in _all_gather_obj(_bytes_of(rec).tobytes(), self.group)]
            want = nat.merge(parts, nat.NAN_FIRST)
            d_in = torch.from_numpy(_bytes_of(rec)).to(dev)
            d_out = torch.zeros_like(d_in)
            torch.cuda.current_stream(dev).synchronize()   # the fill above ran on torch's stream
            try:
                nat.check(lib.llampc_exchange_peer(mb, d_in.data_ptr(), d_out.data_ptr(), nat.NAN_FIRST,
                                                   self.stream.cuda_stream))
                self.stream.synchronize()
                got = _out_of(d_out.cpu().numpy())
                if got.status != 0 or not records_equal(got, want):
                    err = nat.NativeError(f"probe exchange differs from the host merge (status {got.status})")
            except Exception as e:                 # noqa: BLE001
                err = e
            ok = all(_all_gather_obj(err is None, self.group))
        if not ok:
            if mb.value:
                lib.llampc_mailbox_destroy(mb)
            msg = f"llampc: peer exchange unavailable ({err or 'failed on another rank'})"
            if required:
                raise nat.NativeError(msg)
            print(msg + "; falling back", file=sys.stderr)
            self.fallback_reason = f"peer: {err or 'failed on another rank'}"
            return
        self._mailbox = mb

    def _setup_native_exchange(self, dev):
        """The library's RCCL communicator (llampc_comm_*, rccl.h): every rank checks that RCCL
        loads and makes an id, rank 0's id is shared through the process group (any backend),
        then every rank joins (ncclCommInitRank).  Each step is decided collectively, so no rank
        waits in an init the others never enter; on failure all keep the c10d / host gather."""
        import sys
        lib = nat.load()
        err, uid = None, b""
        try:
            buf = (C.c_ubyte * 128)()
            nat.check(lib.llampc_comm_unique_id(buf))
            uid = bytes(buf)
        except Exception as e:                     # noqa: BLE001 — decided collectively below
            err = e
        ok = all(_all_gather_obj(err is None, self.group))
        comm = C.c_void_p()
        if ok:
            uids = _all_gather_obj(uid if self.rank == 0 else b"", self.group)
            try:
                nat.check(lib.llampc_comm_create((C.c_ubyte * 128).from_buffer_copy(uids[0]), self.world, self.rank,
                                                 self.device, C.byref(comm)))
            except Exception as e:                 # noqa: BLE001
                err = e
            ok = all(_all_gather_obj(err is None, self.group))
        if not ok:
            if comm.value:
                lib.llampc_comm_destroy(comm)
            msg = f"{err or 'failed on another rank'}"
            print(f"llampc: native RCCL exchange unavailable ({msg}); using the c10d / host gather", file=sys.stderr)
            self.fallback_reason = ((self.fallback_reason + "; ") if self.fallback_reason else "") + f"rccl: {msg}"
            return
        self._comm = comm

    @property
    def comm(self):
        """This rank's RCCL communicator (llampc_comm*) when the exchange uses it, else None."""
        return self._comm

    def gather_words(self, words: np.ndarray) -> np.ndarray:
        """All-gather a fixed-size uint64 record of every rank, in rank order, over the process
        group: the host-carried transport of the sharded controller (llampc_ctl_resume)."""
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(words, dtype=np.uint64).view(np.int64))
        if self.backend == "nccl":
            d = t.to(self.d_local.device)
            out = torch.empty(self.world * t.numel(), dtype=torch.int64, device=d.device)
            dist.all_gather_into_tensor(out, d, group=self.group)
            return out.cpu().numpy().view(np.uint64)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return torch.cat(parts).numpy().view(np.uint64)

    def stage(self, x_prev, u_prev, x_now, U, xref, uprev) -> dict:
        """Upload one tick's inputs into a device pack (kept resident by the caller)."""
        torch = self._torch
        U = np.asarray(U, dtype=np.float64)
        if U.ndim == 2:
            U = U[None]
        C_, H = U.shape[0], U.shape[1]
        pack = np.concatenate([np.asarray(x_prev, dtype=np.float64).ravel(),
                               np.asarray(u_prev, dtype=np.float64).ravel(),
                               np.asarray(x_now, dtype=np.float64).ravel(),
                               np.asarray(uprev, dtype=np.float64).ravel(),
                               np.asarray(xref, dtype=np.float64).ravel(), U.ravel()])
        with torch.cuda.stream(self.stream):
            d = torch.from_numpy(pack).to(torch.device("cuda", self.device))
        return dict(pack=d, C=C_, H=H, U=U)

    def tick_stream(self, stream=None):
        """The stream a tick runs on: ``stream`` if it is a non-default torch stream, else
        this shard's own stream (self.stream)."""
        if stream is None or stream.cuda_stream == 0:
            return self.stream
        return stream

    def make_plan_in(self, pack, C_, H, Ts=0.02, K=10, integrator="rk4", current_model=0,
                     do_lookback=True, nan_policy=nat.NAN_FIRST, cost=None) -> nat.PlanIn:
        """A PlanIn whose pointers address a device pack laid out as
        [x_prev 6 | u_prev 2 | x_now 6 | uprev 2 | xref 2(H+1) | U 2CH] (float64)."""
        base = pack.data_ptr()
        pin = nat.PlanIn()
        dp = lambda off: base + 8 * off
        pin.x_prev, pin.u_prev, pin.x_now, pin.uprev = dp(0), dp(6), dp(8), dp(14)
        pin.xref, pin.U = dp(16), dp(16 + 2 * (H + 1))
        pin.C, pin.H, pin.K = C_, H, K
        pin.integrator = nat.INTEGRATORS[integrator]
        pin.do_lookback, pin.do_lookahead = int(bool(do_lookback)), 1
        pin.nan_policy = nan_policy
        pin.current_model = current_model
        pin.Ts = Ts
        pin.cost = cost if cost is not None else nat.default_cost()
        pin._pack = pack                   # keep the device buffer alive
        self._nan_policy = nan_policy
        return pin

    def launch(self, pin: nat.PlanIn, stream=None, exchange_events=None):
        """Enqueue one tick on ``tick_stream(stream)``: fused plan on this shard, then (world
        > 1) ONE all-gather of the shard records and the on-device merge, all stream-ordered.
        The merged record is left in ``self.d_merged``; nothing synchronises.
        exchange_events = (start, stop) torch events: this tick runs the exchange as its own
        kernel(s) after the plan launch (the peer transport's split form, llampc_plan_device +
        llampc_exchange_peer: the same protocol and tick number as the fused launch) and the
        events bracket the exchange alone — the bench's per-tick split of plan and exchange."""
        torch = self._torch
        s = self.tick_stream(stream)
        lib = nat.load()
        if self._mailbox is not None and exchange_events is None:   # peer: the plan launch pushes, polls, merges
            nat.check(lib.llampc_plan_exchange(self.bank.handle, C.byref(pin), self.d_local.data_ptr(),
                                               self.d_merged.data_ptr(), self._mailbox, s.cuda_stream))
            return s
        nat.check(lib.llampc_plan_device(self.bank.handle, C.byref(pin), self.d_local.data_ptr(),
                                         None, None, None, s.cuda_stream))
        if exchange_events is not None and self.exchange:
            exchange_events[0].record(s)
        if self._mailbox is not None:
            nat.check(lib.llampc_exchange_peer(self._mailbox, self.d_local.data_ptr(), self.d_merged.data_ptr(),
                                               pin.nan_policy, s.cuda_stream))
            exchange_events[1].record(s)
            return s
        if self._comm is not None:           # native: all-gather + merge on stream s
            nat.check(lib.llampc_exchange_rccl(self._comm, self.d_local.data_ptr(), self.d_all.data_ptr(),
                                               self.d_merged.data_ptr(), pin.nan_policy, s.cuda_stream))
        elif self.exchange:
            import torch.distributed as dist
            if self.backend == "nccl":
                with torch.cuda.stream(s):
                    dist.all_gather_into_tensor(self.d_all, self.d_local, group=self.group)
            else:                          # gloo (CPU rehearsal): gather on the host
                s.synchronize()
                parts = [torch.empty(nat.PLAN_OUT_BYTES, dtype=torch.uint8) for _ in range(self.world)]
                dist.all_gather(parts, self.d_local.cpu(), group=self.group)
                with torch.cuda.stream(s):
                    self.d_all.copy_(torch.cat(parts).to(self.d_all.device), non_blocking=False)
            nat.check(lib.llampc_merge_device(self.d_all.data_ptr(), self.world, pin.nan_policy,
                                              self.d_merged.data_ptr(), self.device, s.cuda_stream))
        if exchange_events is not None and self.exchange:
            exchange_events[1].record(s)
        return s

    def plan_device(self, staged: dict, stream=None, **kw):
        pin = self.make_plan_in(staged["pack"], staged["C"], staged["H"], **kw)
        return self.launch(pin, stream)

    @property
    def mailbox(self):
        """This rank's peer mailbox (llampc_mailbox*), or None when the peer transport is not in
        use (world 1, or a fallback transport)."""
        return self._mailbox

    def close(self):
        if self._mailbox is not None:        # after this rank's last exchange (it synchronises)
            nat.load().llampc_mailbox_destroy(self._mailbox)
            self._mailbox = None
        if self._comm is not None:
            self.stream.synchronize()
            nat.load().llampc_comm_destroy(self._comm)
            self._comm = None
        self.bank.close()

    def fetch(self, stream=None, U=None) -> PlanResult:
        torch = self._torch
        s = self.tick_stream(stream)
        with torch.cuda.stream(s):
            self.h_merged.copy_(self.d_merged, non_blocking=True)
        s.synchronize()
        return result_from_out(_out_of(self.h_merged.numpy()), U)

    def plan(self, x_prev, u_prev, x_now, U, xref, uprev, **kw) -> PlanResult:
        staged = self.stage(x_prev, u_prev, x_now, U, xref, uprev)
        s = self.plan_device(staged, **kw)
        return self.fetch(s, staged["U"])
