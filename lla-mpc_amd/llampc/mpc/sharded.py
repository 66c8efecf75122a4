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


def _rccl_allgather_addr() -> int:
    """Address of ncclAllGather in the RCCL this process already loaded (torch's), found in
    /proc/self/maps: llampc_exchange_device calls it, so no second RCCL is loaded."""
    path = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "librccl" in line:
                path = line.split()[-1]
                break
    if path is None:
        raise nat.NativeError("no RCCL library loaded in this process")
    return C.cast(C.CDLL(path).ncclAllGather, C.c_void_p).value


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
        params_global = np.asarray(params_global, dtype=np.float64)
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
        # C ABI reads as "the bank's own stream", so it is never used to launch a tick
        self.stream = torch.cuda.Stream(device=dev)
        self.bank.set_stream(self.stream.cuda_stream)
        # native exchange (nccl): the all-gather is issued by llampc_exchange_device straight
        # on the tick's stream, over the communicator of a group of its own — no c10d stream
        # hand-off, ~1 us of host time per tick.  LLAMPC_C10D_EXCHANGE=1 keeps the c10d call.
        self._comm = None
        if self.exchange and self.backend == "nccl" and not os.environ.get("LLAMPC_C10D_EXCHANGE"):
            self._setup_native_exchange(dev)

    def _setup_native_exchange(self, dev):
        import sys
        import torch
        import torch.distributed as dist
        xg = dist.new_group(backend="nccl")        # collective: every rank builds its shard
        # one c10d collective creates the group's communicator before its raw use
        dist.all_gather_into_tensor(self.d_all, self.d_local, group=xg)
        torch.cuda.synchronize(dev)
        try:
            comm = xg._get_backend(dev)._comm_ptr()
            fn = _rccl_allgather_addr()
        except Exception as e:                     # transport only: results are the same
            print(f"llampc: native exchange unavailable ({e}); using the c10d all-gather",
                  file=sys.stderr)
            return
        if comm:
            self._xgroup, self._comm, self._allgather = xg, comm, fn

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

    def launch(self, pin: nat.PlanIn, stream=None):
        """Enqueue one tick on ``tick_stream(stream)``: fused plan on this shard, then (world
        > 1) ONE all-gather of the shard records and the on-device merge, all stream-ordered.
        The merged record is left in ``self.d_merged``; nothing synchronises."""
        torch = self._torch
        s = self.tick_stream(stream)
        lib = nat.load()
        nat.check(lib.llampc_plan_device(self.bank.handle, C.byref(pin), self.d_local.data_ptr(),
                                         None, None, None, s.cuda_stream))
        if self._comm is not None:           # native: all-gather + merge on stream s
            nat.check(lib.llampc_exchange_device(self.d_local.data_ptr(), self.d_all.data_ptr(), self.world,
                                                 self.d_merged.data_ptr(), pin.nan_policy, self._comm,
                                                 self._allgather, self.device, s.cuda_stream))
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
        return s

    def plan_device(self, staged: dict, stream=None, **kw):
        pin = self.make_plan_in(staged["pack"], staged["C"], staged["H"], **kw)
        return self.launch(pin, stream)

    def close(self):
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
