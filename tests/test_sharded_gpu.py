"""The N > 1 flow of the product (ShardedBank: per-shard plan kernel, exchange of the
records, merge) with world_size 2, 3, 4 and 8 on ONE GPU: the ranks share cuda:0 (RCCL refuses two
ranks on one device; test_exchange_gpu.py covers the RCCL transport on a 1-rank group).
Transports: "peer" (each rank's mailbox mapped into the other processes through HIP IPC; the
plan launch itself pushes, polls and merges — "peer-split": a second kernel does — with the
ticks enqueued back to back with no synchronisation, so the mailbox's two slots are reused
under load) and "host" (gloo gather,
merge_kernel).  Every rank's merged record, tick after tick, must equal the unsharded tick of
the whole bank on the same inputs."""
import datetime
import os
import shutil
import sys
import tempfile

import numpy as np
import pytest

from conftest import REPO, PKG_ROOT, golden

pytestmark = pytest.mark.gpu

H, W, K, T = 20, 3, 7, 6


def n_models(world, C=3):
    """3001 models (ragged shards) up to world 4; BASELINE config 4's 8 x 10^4 at world 8;
    6001 at C = 64 (each shard's look-ahead then runs the work-queue layout)."""
    return 6001 if C == 64 else (80000 if world == 8 else 3001)


def _ticks(C=3):
    d = golden("dyn_slice.npz")
    s, u = d["states"], d["inputs"]
    rng = np.random.RandomState(8)
    out = []
    for t in range(1, T + 1):
        U = np.repeat(u[:, t:t + H].T[None], C, axis=0)
        U[1:] += rng.uniform(-0.02, 0.02, U[1:].shape)
        out.append((s[:, t - 1], u[:, t - 1], s[:, t], U, s[:2, t:t + H + 1], u[:, t - 1]))
    return out


def _worker(rank, world, store, q, transport, C=3):
    try:
        if transport.endswith("-wq8"):         # the 8-wave work-queue layout at this size
            os.environ["LLAMPC_WQ_WAVES"] = "8"
            transport = transport[:-4]
        if transport == "peer-split":
            os.environ["LLAMPC_PEER_SPLIT"] = "1"
            transport = "peer"
        elif transport == "peer-ticket":       # ticket completion: lb_final in another block
            os.environ["LLAMPC_NO_POLL"] = "1"
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
        dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        sb = ShardedBank(generate_bank(n_models(world, C), seed=12), rank, world, 0, W=W)
        assert sb.transport == transport, (sb.transport, transport)
        pins = [sb.make_plan_in(sb.stage(*a)["pack"], C, H, K=K, current_model=5) for a in _ticks(C)]
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


def _run_ranks(world, transport, C):
    """The ranks in spawned processes, meeting at a FileStore in a private temporary directory
    (no TCP port: nothing another process can take between a probe and the bind); every rank
    process is reaped whatever happens (a rank left waiting on its rendezvous would keep the
    test runner from exiting)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    tmp = tempfile.mkdtemp(prefix="llampc_rdzv_")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, os.path.join(tmp, "store"), q, transport, C))
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


CASES = ([(w, "peer", 3) for w in (2, 3, 4, 8)] + [(w, "host", 3) for w in (2, 3, 8)] +
         [(w, "peer-split", 3) for w in (2, 4)] + [(w, "peer-ticket", 3) for w in (2, 3, 8)] +
         [(2, "peer", 64), (3, "peer-ticket", 64), (2, "peer-wq8", 64), (3, "peer-ticket-wq8", 64)])


@pytest.mark.parametrize("world,transport,C", CASES)
def test_sharded_tick_equals_unsharded_on_gpu(world, transport, C):
    """peer-ticket: LLAMPC_NO_POLL=1, so the record's look-back half is written by lb_final in
    another block than the one that pushes it to the peers (the sc1 hand-off of peer_finish)."""
    from llampc import _native as nat
    from llampc.mpc import ModelBank, generate_bank
    from llampc.mpc.sharded import _out_of
    nat.load()
    if nat.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X")
    got = _run_ranks(world, transport, C)
    ref = []
    with ModelBank(generate_bank(n_models(world, C), seed=12), W=W, device=0) as b:
        for a in _ticks(C):
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


@pytest.mark.parametrize("exchange", ["peer", "host"])
def test_bench_spawns_its_own_ranks(exchange):
    """`python bench.py --gpus 2` with no launcher (no RANK in the environment) starts its two
    rank processes itself (the parent never touches the GPU) and rank 0 prints ONE JSON line
    for the whole job — rehearsed on one GPU (LLAMPC_SAME_DEVICE=1, gloo for the host-side
    collectives; the records travel through the peer mailboxes, or with LLAMPC_EXCHANGE=host
    through the process group: the transport a node without peer access falls back to) —
    extras included: C = 64 ticks, BASELINE config 5 (two tracks) sharded over both ranks and
    the sharded controller."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                              "MASTER_ADDR", "MASTER_PORT")}
    env.update(LLAMPC_DIST_BACKEND="gloo", LLAMPC_SAME_DEVICE="1", LLAMPC_EXCHANGE=exchange)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "40",
                        "--warmup", "5", "--ticks", "4", "--n-per-gpu", "2000",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["N_models_total"] == 4000
    assert rec["config"]["transport"] == exchange and rec["config"]["transport_fallback"] is None
    assert rec["value"] > 0 and rec["plan_call_us"]["p50"] > 0
    # the extras run on every rank: C = 64 ticks and BASELINE config 5 sharded over the ranks
    assert rec["C64"]["ms_per_step"] > 0
    c5 = rec["config5"]
    assert c5["N_per_track"] == 4000 and c5["transport"] == [exchange] * 2 and c5["p99_us"] > 0
    # the sharded controller (config 5's real loop): both tracks' controllers over both ranks
    ct = rec["controller_tick_us"]
    assert ct["N_per_track"] == 4000 and ct["transport"] == [exchange] * 2 and 0 < ct["p50"] <= ct["p99"]
