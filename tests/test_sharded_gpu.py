"""The N > 1 flow of the product (ShardedBank: per-shard plan kernel, exchange of the
records, merge) with world_size 2, 3 and 4 on ONE GPU: the ranks share cuda:0 (RCCL refuses two
ranks on one device; test_exchange_gpu.py covers the RCCL transport on a 1-rank group).
Transports: "peer" (each rank's mailbox mapped into the other processes through HIP IPC; the
plan launch itself pushes, polls and merges — "peer-split": a second kernel does — with the
ticks enqueued back to back with no synchronisation, so the mailbox's two slots are reused
under load) and "host" (gloo gather,
merge_kernel).  Every rank's merged record, tick after tick, must equal the unsharded tick of
the whole bank on the same inputs."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO, PKG_ROOT, golden

pytestmark = pytest.mark.gpu

N, H, C, W, K, T = 3001, 20, 3, 3, 7, 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ticks():
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    rng = np.random.RandomState(8)
    out = []
    for t in range(1, T + 1):
        U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
        U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
        out.append((s[:, t - 1], u[:, t - 1], s[:, t], U, s[:2, t:t + H + 1], u[:, t - 1]))
    return out


def _worker(rank, world, port, q, transport):
    try:
        if transport == "peer-split":
            os.environ["LLAMPC_PEER_SPLIT"] = "1"
            transport = "peer"
        os.environ["LLAMPC_EXCHANGE"] = transport
        for pth in (REPO, PKG_ROOT):
            if pth not in sys.path:
                sys.path.insert(0, pth)
        import torch
        import torch.distributed as dist
        from llampc import _native as nat
        from llampc.mpc import generate_bank
        from llampc.mpc.sharded import ShardedBank, _bytes_of
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        sb = ShardedBank(generate_bank(N, seed=12), rank, world, 0, W=W)
        assert sb.transport == transport, (sb.transport, transport)
        pins = [sb.make_plan_in(sb.stage(*a)["pack"], C, H, K=K, current_model=5) for a in _ticks()]
        torch.cuda.synchronize()
        outs = []
        for pin in pins:                        # back to back: no synchronisation between ticks
            s_ = sb.launch(pin)
            o = torch.empty_like(sb.d_merged)
            with torch.cuda.stream(s_):
                o.copy_(sb.d_merged)
            outs.append(o)
        torch.cuda.synchronize()
        recs = [o.cpu().numpy() for o in outs]
        sb.close()
        dist.destroy_process_group()
        q.put((rank, np.stack(recs), None))
    except Exception as e:                      # report, do not hang the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("transport", ["peer", "peer-split", "host"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_tick_equals_unsharded_on_gpu(world, transport):
    import torch.multiprocessing as mp
    from llampc import _native as nat
    from llampc.mpc import ModelBank, generate_bank
    from llampc.mpc.sharded import _out_of
    nat.load()
    if nat.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, transport)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, recs, err = q.get(timeout=100)
        assert err is None, f"rank {rank}:\n{err}"
        got[rank] = recs
    for p in procs:
        p.join(timeout=30)
    ref = []
    with ModelBank(generate_bank(N, seed=12), W=W, device=0) as b:
        for a in _ticks():
            ref.append(nat.plan_out_to_dict(b.plan_raw(*a, K=K, current_model=5)[0]))
    for rank in range(world):
        for t in range(T):
            A = nat.plan_out_to_dict(_out_of(got[rank][t]))
            B = ref[t]
            assert A["status"] == 0
            for k in B:
                if isinstance(B[k], np.ndarray):
                    np.testing.assert_array_equal(A[k], B[k], err_msg=f"rank {rank} tick {t} {k}")
                else:
                    assert A[k] == B[k] or (A[k] != A[k] and B[k] != B[k]), (rank, t, k, A[k], B[k])
