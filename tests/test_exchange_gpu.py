"""GPU test of the N > 1 tick path on one device: a 1-rank RCCL group with the exchange
forced on (LLAMPC_FORCE_EXCHANGE=1), so each tick runs plan -> all-gather -> merge_kernel
exactly as a rank of the 8-GPU job does.  Every tick's merged record must equal the plain
single-bank tick on the same inputs, for each transport: the peer mailbox (llampc_exchange_peer:
push over IPC-mapped memory, poll, merge — one kernel), RCCL issued natively
(llampc_exchange_rccl over the library's RCCL communicator, on the tick's stream) and c10d.
No per-tick synchronisation: the stream order alone must make the records right."""
import os
import tempfile

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist
    from llampc import _native
    _native.load()
    if _native.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    torch.cuda.set_device(0)
    with tempfile.TemporaryDirectory(prefix="llampc_rdzv_") as tmp:   # a FileStore: no port to race for
        dist.init_process_group("nccl", init_method=f"file://{os.path.join(tmp, 'store')}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        yield
        dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["peer", "peer-ticket", "peer-split", "rccl", "c10d"])
def test_exchange_tick_equals_plain_tick(nccl_world1, transport, monkeypatch):
    import torch
    from llampc import _native as nat
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank, _out_of
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    N, H, C, W, K, T = 4000, 20, 2, 4, 6, 12
    rng = np.random.RandomState(5)
    bank = generate_bank(N, seed=6)
    if transport == "peer-split":            # the plan launch, then peer_exchange_kernel
        monkeypatch.setenv("LLAMPC_PEER_SPLIT", "1")
        transport = "peer"
    if transport == "peer-ticket":           # fused exchange after the ticket completion
        monkeypatch.setenv("LLAMPC_NO_POLL", "1")
        transport = "peer"
    env = {"LLAMPC_FORCE_EXCHANGE": "1", "LLAMPC_EXCHANGE": transport}
    os.environ.update(env)
    try:
        sx = ShardedBank(bank, 0, 1, 0, W=W)
    finally:
        for k in env:
            del os.environ[k]
    sp = ShardedBank(bank, 0, 1, 0, W=W)
    try:
        assert sx.exchange and not sp.exchange
        assert sx.transport == transport
        staged = []
        for t in range(1, T + 1):
            U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
            U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
            staged.append((s[:, t - 1], u[:, t - 1], s[:, t], U, s[:2, t:t + H + 1], u[:, t - 1]))
        px = [sx.make_plan_in(sx.stage(*a)["pack"], C, H, K=K, current_model=3) for a in staged]
        pp = [sp.make_plan_in(sp.stage(*a)["pack"], C, H, K=K, current_model=3) for a in staged]
        torch.cuda.synchronize()
        recs_x, recs_p = [], []
        for i in range(T):
            sx.launch(px[i])                 # no synchronisation between the ticks
            sp.launch(pp[i])
            hx = torch.empty_like(sx.h_merged)
            hp = torch.empty_like(sp.h_merged)
            with torch.cuda.stream(sx.stream):
                hx.copy_(sx.d_merged, non_blocking=True)
            with torch.cuda.stream(sp.stream):
                hp.copy_(sp.d_merged, non_blocking=True)
            recs_x.append(hx)
            recs_p.append(hp)
        torch.cuda.synchronize()
        for i in range(T):
            A = nat.plan_out_to_dict(_out_of(recs_x[i].numpy()))
            B = nat.plan_out_to_dict(_out_of(recs_p[i].numpy()))
            assert A["status"] == 0 and B["status"] == 0
            for k in B:
                if isinstance(B[k], np.ndarray):
                    np.testing.assert_array_equal(A[k], B[k], err_msg=f"tick {i} {k}")
                else:
                    assert A[k] == B[k] or (A[k] != A[k] and B[k] != B[k]), (i, k, A[k], B[k])
        assert recs_p[-1].numpy().any()
    finally:
        sx.close()
        sp.close()


def _mailboxes(G, bound=None):
    import ctypes as C
    from llampc import _native as nat
    lib = nat.load()
    mbs = []
    for r in range(G):
        mb = C.c_void_p()
        nat.check(lib.llampc_mailbox_create(G, r, 0, C.byref(mb)))
        if bound is not None:
            nat.check(lib.llampc_mailbox_set_bound(mb, bound))
        mbs.append(mb)
    for r in range(G):
        for g in range(G):
            if g != r:
                nat.check(lib.llampc_mailbox_link(mbs[r], g, mbs[g]))
    return lib, mbs


def test_peer_exchange_missing_rank_times_out():
    """A rank whose peer never pushes gives up after the poll bound with status
    LLAMPC_STATUS_POLL_TIMEOUT (the host path raises on it) instead of hanging."""
    import time
    import torch
    from llampc import _native as nat
    from llampc.mpc.sharded import _bytes_of, _out_of, probe_record
    lib, mbs = _mailboxes(2, bound=0.05)
    try:
        d_in = torch.from_numpy(_bytes_of(probe_record(0, 2))).cuda()
        d_out = torch.zeros_like(d_in)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nat.check(lib.llampc_exchange_peer(mbs[0], d_in.data_ptr(), d_out.data_ptr(), nat.NAN_FIRST, None))
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 5.0
        assert _out_of(d_out.cpu().numpy()).status == 1
    finally:
        for mb in mbs:
            lib.llampc_mailbox_destroy(mb)
