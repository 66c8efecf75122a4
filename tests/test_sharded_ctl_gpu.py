"""The sharded controller (BASELINE config 5's real loop across GPUs): world 2, 3 and 8 ranks —
self-spawned processes sharing cuda:0, each ticking LLAMPC (device mode) on its contiguous shard
with the per-tick exchange, over each transport the ShardedBank can take:
  peer  llampc_ctl_set_exchange: inside the tick's launch (push of the shard's top-K and argmin
        into every peer's IPC-mapped mailbox, poll, merge); launched, and armed ("peer-armed":
        every rank's launch enqueued during the previous tick, rung with x_t, the exchange after
        its doorbell — with rank 0 cancelling its arming for one tick mid-run);
  host  llampc_ctl_set_gather without a communicator: two launches, the records carried by the
        process group (gloo) between them (llampc_ctl_shard_record / llampc_ctl_resume);
  rccl  llampc_ctl_set_gather with the library's RCCL communicator: ncclAllGather between the two
        launches on the bank's stream — at world 1 (RCCL refuses two ranks on one device, and
        this box has one; the merge of several records is the host transport's, same kernel).
Every rank rolls out the merged selection's K + 1 models from the replicated global table.  In
closed loop with
the RK6 plant (the oracle's, on the host: every rank applies the same control), every rank's
llampc_ctl_out record must equal the UNSHARDED controller's, bitwise, tick after tick —
through the warm-up (no exchange), the first full window and the ticks after it.  One case has
NaN models in two shards (np.argmin's first NaN must win across the shards)."""
import datetime
import os
import shutil
import sys
import tempfile

import numpy as np
import pytest

from conftest import REPO, PKG_ROOT, golden

pytestmark = pytest.mark.gpu

H, C, K, W, T, TS = 40, 64, 10, 5, 12, 0.02


def _bank(n, case):
    from llampc.mpc import generate_bank
    p = generate_bank(n, seed=4)
    if case == "nan":                      # NaN models in the first and the last shard
        p[2, [n - 7, 11]] = np.nan
    return p


def _loop(ctl, x0, ticks, before=None):
    """Closed loop: tick, apply u_seq[0] to the RK6 plant (friction dropping 1/260 per tick);
    before(t) runs ahead of tick t."""
    from oracle import llampc_oracle as O
    from llampc import _native as nat
    plant = O.Vehicle.from_params(O.orca_params())
    x = x0.copy()
    recs = []
    for t in range(ticks):
        if before is not None:
            before(t)
        r = ctl.tick(x)
        recs.append(np.frombuffer(bytes(r.raw), dtype=np.uint8).copy())
        u = np.array(r.raw.u_seq[0][:])
        plant.Df *= 1 - 1 / 260.0
        plant.Dr *= 1 - 1 / 260.0
        xn, _ = O.sim_continuous(plant, x, u.reshape(2, 1), [0, TS])
        x = xn[:, -1]
    assert recs[0].size == C_OUT_BYTES(nat)
    return np.stack(recs)


def C_OUT_BYTES(nat):
    import ctypes
    return ctypes.sizeof(nat.CtlOut)


def _worker(rank, world, store, q, n, case, transport):
    try:
        armed = transport == "peer-armed"
        transport = "peer" if armed else transport
        os.environ["LLAMPC_EXCHANGE"] = transport
        if world == 1:
            os.environ["LLAMPC_FORCE_EXCHANGE"] = "1"     # the exchange path on a one-rank group
        for pth in (REPO, PKG_ROOT):
            if pth not in sys.path:
                sys.path.insert(0, pth)
        import torch
        import torch.distributed as dist
        from llampc.mpc import LLAMPC
        from llampc.mpc.sharded import ShardedBank
        from llampc.tracks import ETHZ
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        sb = ShardedBank(_bank(n, case), rank, world, 0, W=W)
        assert sb.exchange and sb.transport == transport, (sb.transport, sb.fallback_reason)
        sb.bank.set_concurrency(world)     # every rank on this one device: its share of the CUs
        ctl = LLAMPC(sb, ETHZ('optimal', True), H=H, C=C, K=K, mode="device", prelaunch=armed)
        assert ctl._ctl.transport == transport and ctl._ctl.prelaunch == armed
        before = None
        if armed and rank == 0:            # a cancel mid-run on one rank only: its tick 8 launches
            def before(t):                 # while the other ranks' armed launches are rung
                if t == 8:
                    ctl.set_prelaunch(False)
                elif t == 9:
                    ctl.set_prelaunch(True)
        recs = _loop(ctl, golden("dyn_slice.npz")["states"][:, 0], T, before)
        ctl.close()
        dist.barrier()
        sb.close()
        dist.destroy_process_group()
        q.put((rank, recs, None))
    except Exception:                      # report, do not hang the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def _run_ranks(world, n, case, transport="peer"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    tmp = tempfile.mkdtemp(prefix="llampc_rdzv_")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, os.path.join(tmp, "store"), q, n, case, transport))
             for r in range(world)]
    for p in procs:
        p.start()
    got, errs = {}, []
    try:
        for _ in range(world):
            rank, recs, err = q.get(timeout=150)
            if err is not None:
                errs.append((rank, err))
                break
            got[rank] = recs
    finally:
        for p in procs:
            p.join(timeout=30 if not errs else 1)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
        shutil.rmtree(tmp, ignore_errors=True)
    if errs:
        raise AssertionError(f"rank {errs[0][0]}:\n{errs[0][1]}")
    return got


@pytest.mark.parametrize("world,n,case,transport", [(2, 4000, "plain", "peer"), (3, 4001, "plain", "peer"),
                                                    (8, 8000, "plain", "peer"), (3, 3001, "nan", "peer"),
                                                    (2, 4000, "plain", "peer-armed"),
                                                    (3, 4001, "plain", "peer-armed"),
                                                    (8, 8000, "plain", "peer-armed"),
                                                    (3, 3001, "nan", "peer-armed"),
                                                    (2, 4000, "plain", "host"), (3, 4001, "plain", "host"),
                                                    (3, 3001, "nan", "host"),
                                                    (1, 4000, "plain", "rccl"), (1, 3001, "nan", "rccl")])
def test_sharded_controller_equals_unsharded(world, n, case, transport):
    from llampc import _native as nat
    from llampc.mpc import LLAMPC, ModelBank
    from llampc.tracks import ETHZ
    nat.load()
    if nat.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    got = _run_ranks(world, n, case, transport)
    # the unsharded controller, launched (prelaunch=False): armed ticks equal launched ones
    with ModelBank(_bank(n, case), W=W, device=0) as b, \
            LLAMPC(b, ETHZ('optimal', True), H=H, C=C, K=K, prelaunch=False) as ctl:
        ref = _loop(ctl, golden("dyn_slice.npz")["states"][:, 0], T)
    dt = np.dtype(nat.CtlOut)
    for rank in range(world):
        for t in range(T):
            if np.array_equal(got[rank][t], ref[t]):
                continue
            a, b = got[rank][t].view(dt)[0], ref[t].view(dt)[0]
            diff = [f for f in dt.names if not np.array_equal(np.asarray(a[f]).view(np.uint8),
                                                                np.asarray(b[f]).view(np.uint8))]
            raise AssertionError(f"rank {rank} tick {t}: record fields differ: {diff}")
    # the case did select across shards after the warm-up
    last = ref[-1].view(dt)[0]
    assert last["warm"] == 0 and last["plan"]["window_full"] == 1
    if case == "nan":
        assert last["plan"]["lb_best"] == 11
