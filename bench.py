#!/usr/bin/env python3
"""bench.py — LLA-MPC model-bank tick on MI355X (BASELINE.json metric).

One *step* = one LLA-MPC control tick of the hot path over the whole bank:
look-back (score every model on the newest transition, slide the W-window, argmin +
top-K) + look-ahead (H-step RK4 rollout + MPC cost of every (model, candidate)) +
selection, i.e. ``llampc_plan_device`` (ONE kernel launch).  With --gpus N > 1 each rank owns a
contiguous shard of N_per_gpu models (weak scaling; config 4 = 8 x 10^4) and every tick
adds ONE exchange of the 1.5 KB shard records plus the on-device merge: by default one
kernel that pushes the record into every peer's IPC-mapped mailbox over xGMI and merges
(llampc_exchange_peer), else an RCCL all-gather + merge_kernel (LLAMPC_EXCHANGE).

Workload (BASELINE.json configs[1]): ETHZ track, N_models = 10^4 per GPU, H = 20, C = 1
candidate, W = 10, K = 10, Ts = 0.02, gradual friction change.  Tick inputs are
synthetic-but-physical: states from the device RK6 plant (Dynamic.sim_continuous)
driven by the recorded ETHZ controls (llampc/tracks/data/dyn_slice.npz) under the gradual
friction decay D <- D(1 - 1/2600) per tick (rt.py:125-130), xref from ConstantSpeed on the
packaged ETHZ raceline library.  All tick inputs are resident in HBM before timing.

value = (N_total * C * H + N_total) / (ms_per_step / 1e3)  [model-rollout-steps / s].
"""
import argparse
import ctypes
import json
import os
import sys
import time

# kernel arguments in device memory (the default of this ROCm; kept explicit: host-memory
# kernargs cost the tick 5 us) — set before anything initialises HIP
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "lla-mpc_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X fp64 vector spec
# ONE HIP-event pair brackets the whole timed loop (stride = --steps): each event record costs
# ~5 us of stream time (kernel trace, profiles/r03/s3_ramp: a 10.2 us gap at every group
# boundary), so the old groups of 8 added ~1.3 us to every timed tick
TIMING_SAMPLE = 64              # with the exchange: one plan launch in 64 bracketed alone (each pair ~10 us of stream time)
FLOPS_PER_MODEL_STEP = 264 + 7  # RK4 step + cost accumulation (excl. transcendentals)
# Issue roofline: instructions per rollout step of the fast look-ahead loop, per lane, by lane
# split (tools/diag/isa_counts.py on the current sources), and the chip's fp64 VALU issue
# capacity: 1,024 SIMDs x 16 lanes per clock x 2.4 GHz (MI355X_MICROARCH.md max clock).
ISSUE_INSTR_PER_STEP = {4: 456, 2: 568, 1: 809}   # tools/diag/isa_counts.py, 8-term cores (LPM 1: work queue)
ISSUE_PEAK_LANE_INSTR = 1024 * 16 * 2.4e9
# the controller's and the NLP search's rollout steps (tools/diag/isa_counts.py): the
# controller's LPM-4 step with its staged input terms, the NLP's LPM-4 Euler step with staged terms
CTL_INSTR_PER_STEP = 453
NLP_INSTR_PER_STEP = 159
LOOKBACK_INSTR_PER_MODEL = ISSUE_INSTR_PER_STEP[1]   # one LPM-1 RK4 step + error + ring per model (upper bound)


EXCHANGE_DESC = {
    "peer": "peer mailboxes over xGMI (HIP IPC): the plan launch pushes its record, polls and merges (llampc_plan_exchange)",
    "rccl": "ncclAllGather on the tick stream over the library's own RCCL communicator (llampc_exchange_rccl) + merge_kernel",
    "c10d": "c10d all_gather_into_tensor (nccl) + merge_kernel",
    "host": "gloo all-gather on the host + merge_kernel",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--n-per-gpu", type=int, default=10000)
    ap.add_argument("--H", type=int, default=20)
    ap.add_argument("--C", type=int, default=1)
    ap.add_argument("--W", type=int, default=10)
    ap.add_argument("--K", type=int, default=10)
    ap.add_argument("--track", default="ETHZ", choices=["ETHZ", "ETHZMobil"])
    ap.add_argument("--scenario", default=None, choices=["gradual", "sudden"],
                    help="friction change of the tick inputs (default: gradual on ETHZ, sudden on "
                         "ETHZMobil, BASELINE configs 2/3)")
    ap.add_argument("--ticks", type=int, default=64, help="distinct resident tick inputs")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C=64 and latency extras")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--no-call-latency", action="store_true", help="skip the per-plan() H2D+tick+D2H latency")
    return ap.parse_args()


def make_ticks(args, T, seed=0):
    """T ticks of (x_prev, u_prev, x_now, uprev, xref, U) of the config's friction scenario
    (llampc.mpc.scenarios: config 2 gradual on ETHZ, config 3 sudden on ETHZMobil)."""
    from llampc.mpc.scenarios import scenario_ticks
    return scenario_ticks(args.track, args.H, args.C, T, getattr(args, "scenario", None), device=torch_device_index())


_DEV = [0]


def max_over_ranks(x: float) -> float:
    """MAX of a host scalar over the process group (device tensor under nccl, host under gloo)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", _DEV[0]) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def torch_device_index():
    return _DEV[0]


def cpu_model_name() -> str:
    """The host CPU's model name (what `lscpu` prints as "Model name"), from /proc/cpuinfo."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """CPUs this process may run on (the box's CPU share, not the whole machine's count)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


_CPU_SHARD = {}


def _cpu_shard_init(N, lo, hi, W, K, seed, ticks):
    """Worker of the sharded NumPy baseline: its contiguous shard [lo, hi) of the seeded bank
    and its own look-back window (the reference state per rank of SURVEY.md §8(e))."""
    for p in (REPO, os.path.join(REPO, "lla-mpc_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from llampc.mpc import generate_bank
    from oracle import llampc_oracle as O
    p = O.orca_params()
    _CPU_SHARD.update(
        O=O, bank=generate_bank(N, seed=seed)[:, lo:hi], lo=lo, ticks=ticks,
        win=O.LookbackWindow(hi - lo, W, K),
        shared={k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")})


def _cpu_shard_tick(i, C, H):
    """One tick of the oracle plan_cpu on this worker's shard; returns the shard record the
    merge needs: the window's top-K (values, global indices) and the look-ahead best."""
    S = _CPU_SHARD
    O, pk = S["O"], S["ticks"][i % len(S["ticks"])]
    xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
    U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))
    _, best_k, cost = O.plan_cpu(S["shared"], S["bank"], S["win"], pk[0:6], pk[6:8], pk[8:14], U, xref,
                                 pk[14:16], 0.02, Q, R, P)
    flat = cost.ravel()
    j = int(np.argmin(np.where(np.isnan(flat), np.inf, flat)))
    if best_k is None:
        return None, None, float(flat[j]), S["lo"] * C + j
    return S["win"].avg[best_k], best_k + S["lo"], float(flat[j]), S["lo"] * C + j


def cpu_baseline(args, seconds):
    """The oracle (NumPy restatement of the reference path) on the same workload shape:
    look-back + window/argmin/argsort + H-step RK4 rollout + cost.  Two legs: one process
    (the reference runs single-threaded) and the bank split over P worker
    processes (SURVEY.md §8(d) "n-process sharded NumPy variant": contiguous shards, each with
    its own window, merged per tick like the GPU shards)."""
    from llampc.mpc import generate_bank
    from oracle import llampc_oracle as O
    ticks = make_ticks(args, 4)
    N, H, C = args.n_per_gpu, args.H, args.C
    seed = 0 if args.track == "ETHZ" else 1
    bank = generate_bank(N, seed=seed)
    p = O.orca_params()
    shared = {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
    win = O.LookbackWindow(N, args.W, args.K)
    Q, R, P = np.eye(2), np.diag([5e-3, 1]), np.zeros((2, 2))

    def one(i):
        pk = ticks[i % len(ticks)]
        xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
        U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
        O.plan_cpu(shared, bank, win, pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], 0.02, Q, R, P)

    def timed(fn, budget):
        fn(0)
        reps, t0 = 0, time.perf_counter()
        while True:
            fn(reps + 1)
            reps += 1
            el = time.perf_counter() - t0
            if (el >= budget and reps >= 2) or reps >= 1000:
                return reps, el

    reps, el = timed(one, seconds)
    per = el / reps
    model = cpu_model_name()
    out = {"value": (N * C * H + N) / per, "unit": "model-rollout-steps/s", "cores": 1, "kind": "port",
           "ms_per_step": per * 1e3, "cpu_model": model, "host_cores_visible": host_cores(),
           "sample": f"{reps} plan() ticks of the oracle NumPy restatement (oracle/llampc_oracle.py "
                     f"plan_cpu = reference evaluate_models_vectorized + rt.py window logic + H x "
                     f"_integrate_batch + nmpc.py cost) at N={N}, H={H}, C={C} on 1 core of "
                     f"{host_cores()} visible ({model}; the sharded leg uses the box share of 16), {el:.1f} s"}
    nproc = min(16, host_cores())
    if nproc > 1:
        out["sharded"] = cpu_baseline_sharded(args, ticks, nproc, seconds, seed)
    return out


def cpu_baseline_sharded(args, ticks, nproc, seconds, seed):
    """The sharded NumPy leg: nproc worker processes (spawned: fresh interpreters, no GPU
    state), each ticking plan_cpu on its contiguous shard; per tick the parent gathers the
    shard records and merges them (top-K by value, ties to the lower index; look-ahead best)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    N, H, C, W, K = args.n_per_gpu, args.H, args.C, args.W, args.K
    pools = []
    try:
        for r in range(nproc):
            lo, hi = (r * N) // nproc, ((r + 1) * N) // nproc
            pools.append(ProcessPoolExecutor(1, mp_context=mp.get_context("spawn"), initializer=_cpu_shard_init,
                                             initargs=(N, lo, hi, W, K, seed, ticks)))

        def one(i):
            parts = [f.result() for f in [p.submit(_cpu_shard_tick, i, C, H) for p in pools]]
            if parts[0][0] is not None:
                vals = np.concatenate([q[0] for q in parts])
                idx = np.concatenate([q[1] for q in parts])
                order = np.lexsort((idx, vals))[:K]
                _ = idx[order]
            return min((q[2], q[3]) for q in parts)

        one(0)                                  # start the workers (imports) outside the clock
        reps, t0 = 0, time.perf_counter()
        while True:
            one(reps + 1)
            reps += 1
            el = time.perf_counter() - t0
            if (el >= seconds and reps >= 2) or reps >= 1000:
                break
    finally:
        for p in pools:
            p.shutdown(wait=True, cancel_futures=True)
    per = el / reps
    return {"value": (N * C * H + N) / per, "unit": "model-rollout-steps/s", "cores": nproc, "kind": "port",
            "ms_per_step": per * 1e3,
            "sample": f"{reps} plan() ticks, bank split into {nproc} contiguous shards, one NumPy process "
                      f"each (own window), records merged per tick; N={N}, H={H}, C={C}, {el:.1f} s"}


def spawn_ranks(n: int, cmd=None) -> int:
    """`bench.py --gpus N` (N > 1) started WITHOUT a launcher (no RANK in the environment):
    start N rank processes of this same command line, one per GPU, with the environment
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
    MASTER_ADDR=127.0.0.1) and, for the rendezvous, LLAMPC_INIT_FILE: a FileStore path in a
    private temporary directory (no TCP port to probe and then lose to another process), and
    return their exit status.  This parent never touches the GPU — no torch import, no HIP call,
    no exec — it starts, watches and, if one rank fails, stops its own children by PID so the
    rest do not wait in a rendezvous."""
    import shutil
    import signal
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp(prefix="llampc_rdzv_")
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", LLAMPC_INIT_FILE=os.path.join(tmp, "store"))
        env.pop("MASTER_PORT", None)
        procs.append(subprocess.Popen(cmd, env=env))
    rc, live = 0, list(procs)
    try:
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c          # killed by signal -c
                    print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for q in procs:                                   # only reached with live ranks on error
            if q.poll() is None:
                q.kill()
                q.wait()
        shutil.rmtree(tmp, ignore_errors=True)
    return rc


def init_group(backend, rank, world, device=None):
    """torch.distributed rendezvous: the FileStore of a self-spawned job (LLAMPC_INIT_FILE,
    spawn_ranks), else env:// (torch.distributed.run's MASTER_ADDR / MASTER_PORT)."""
    import torch.distributed as dist
    kw = {"device_id": device} if device is not None else {}
    path = os.environ.get("LLAMPC_INIT_FILE")
    if path:
        dist.init_process_group(backend, init_method=f"file://{path}", rank=rank, world_size=world, **kw)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = int(os.environ.get("WORLD_SIZE", "1"))
    import torch
    import torch.distributed as dist
    # LLAMPC_DIST_BACKEND=gloo + LLAMPC_SAME_DEVICE=1: rehearsal of the N-rank flow on a
    # one-GPU box (records gathered over gloo on the host, merged by the same device kernel)
    backend = os.environ.get("LLAMPC_DIST_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("LLAMPC_SAME_DEVICE") else local
    torch.cuda.set_device(dev_index)
    _DEV[0] = dev_index
    local = dev_index
    # LLAMPC_FORCE_EXCHANGE=1 (diagnostic, under torch.distributed.run with one rank): the
    # tick runs the collective + device merge of the N > 1 path on a 1-rank group
    if world > 1 or os.environ.get("LLAMPC_FORCE_EXCHANGE"):
        init_group(backend, rank, world, torch.device("cuda", local) if backend == "nccl" else None)
    from llampc import _native as nat
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank

    N_local, H, C, K, W = args.n_per_gpu, args.H, args.C, args.K, args.W
    N_total = N_local * world
    T = max(args.ticks, 1)
    ticks = make_ticks(args, T)
    dev = torch.device("cuda", local)
    packs = torch.from_numpy(ticks).to(dev)                 # resident tick inputs [T, L]
    torch.cuda.synchronize()
    bank_global = generate_bank(N_total, seed=0 if args.track == "ETHZ" else 1)
    sb = ShardedBank(bank_global, rank, world, local, W=W)
    stream = sb.stream                  # plan, all-gather and merge: one stream (the bank's)
    pins = [sb.make_plan_in(packs[i], C, H, K=K, current_model=0) for i in range(T)]
    lib = nat.load()

    def step(i, ex=None):
        sb.launch(pins[i % T], stream, exchange_events=ex)

    # with the exchange: the ticks whose plan launch the bank's sampled event pair brackets (one
    # in TIMING_SAMPLE) run the exchange as its own kernel, bracketed by a second event pair, so
    # the line splits a tick into plan and exchange (peer: the split form of the same protocol)
    ex_events = []
    if sb.exchange and not args.no_timing:
        ex_events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in range(args.steps // TIMING_SAMPLE + 1)]

    avg = (ctypes.c_double * 3)()
    cnt = (ctypes.c_int64 * 3)()
    if not args.no_timing:
        # events created (and the stream synchronised) before the warmup, so the gap between
        # the warmup and the timed loop is the synchronize alone; one event pair brackets all K consecutive launches of the timed loop: the kernel's
        # mean duration measured live (back-to-back launches: the trace shows no gap between
        # them, so elapsed / K is the mean duration), the events' own cost spread over K.
        # With the exchange, a group would also hold the all-gathers and merges in between,
        # so ONE plan launch in every TIMING_SAMPLE gets its own pair (negative stride =
        # sampling; the bracketed launch reads ~2 us high, the events' own cost, and only
        # 1/TIMING_SAMPLE of the timed ticks carry events: measured 0.8 us/tick of event
        # cost at 1 in 8 on a forced 1-rank exchange, ~2 us with a pair on every tick)
        stride = -TIMING_SAMPLE if sb.exchange else max(args.steps, 1)
        nat.check(lib.llampc_bank_timing(sb.bank.handle, stride, args.steps // abs(stride) + 8))
    if world > 1:                       # every rank's exchange waits for the others' records
        dist.barrier()
    # every timed tick runs the stated workload, the full-window look-back (window mean, top-K,
    # lb_final; rt.py:354-360): at least W ticks run before the timed loop, whatever --warmup
    # says (a tick with a partial window skips the selection)
    fill = max(args.warmup, W)
    for i in range(fill):
        step(i)
    if not args.no_timing:              # restart the count: the warmup launches are not timed
        nat.check(lib.llampc_bank_timing_read(sb.bank.handle, avg, cnt))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    count_before = sb.bank.window_count         # host state: the window before the first timed tick
    for i in range(args.steps):
        step(fill + i, ex_events[i // TIMING_SAMPLE] if ex_events and i % TIMING_SAMPLE == 0 else None)
    t_issue = time.perf_counter() - t0       # host time to enqueue the K ticks
    torch.cuda.synchronize()
    if world > 1:                            # (at world 1 there is no barrier to re-synchronise after)
        dist.barrier()
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el)
    ms = el / args.steps * 1e3

    if not args.no_timing:
        nat.check(lib.llampc_bank_timing_read(sb.bank.handle, avg, cnt))
        nat.check(lib.llampc_bank_timing(sb.bank.handle, 0, 1))
    plan_ms = avg[0]
    exch_ms = float(np.mean([a.elapsed_time(b) for a, b in ex_events])) if ex_events else None
    if world > 1 and exch_ms is not None:
        exch_ms = max_over_ranks(exch_ms)
        plan_ms = max_over_ranks(plan_ms)

    merged = sb.fetch(stream)          # result of the last tick (all ranks identical)

    # SURVEY §8(d)'s per-plan() wall time: the same tick with its inputs coming from host
    # memory and its record going back (every rank; the exchange included when world > 1)
    call = None if args.no_call_latency else plan_call_latency(args, sb, stream, ticks, world)

    extra = {}
    if not args.no_extra:              # every rank: the C=64 extra ticks run the collective
        extra = extras(args, sb, stream, world, rank)

    if rank == 0:
        steps_per_tick = N_total * C * H + N_total
        value = steps_per_tick / (ms / 1e3)
        # algorithmic HBM bytes of one fused plan-kernel launch (the dominant kernel), SURVEY
        # §8(d): per model params 48 B + ring read 8W + ring write 8 + look-ahead result 12;
        # per launch candidates 16*C*H + xref 16*(H+1) + states/inputs 64
        plan_bytes = N_local * (48 + 8 * W + 8 + 12) + 16 * C * H + 16 * (H + 1) + 64
        achieved = plan_bytes / (plan_ms * 1e-3) / 1e9 if plan_ms > 0 else None
        traffic = pmc_traffic(args)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                "kernel": "plan_kernel<RK4> (the whole tick: look-back + look-ahead + selection)",
                "kernel_avg_us": plan_ms * 1e3,
                "bytes_per_launch": plan_bytes,
                "note": "binding resource is fp64 VALU/latency, not HBM (see valu)"}
        valu_gf = (N_local * C * H + N_local) * FLOPS_PER_MODEL_STEP / (plan_ms * 1e-3) / 1e9 if plan_ms > 0 else None
        line = {
            "metric": "model-rollouts/sec (N_models x H steps) per control tick; wall-clock per plan() call",
            "value": value, "unit": "model-rollout-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (RK6-plant states under the friction change of config.workload, recorded ETHZ controls, "
                    "ConstantSpeed xref; seeded Pacejka bank)",
            "config": {"workload": f"{args.track} LLA-MPC tick: look-back W={W} K={K} + look-ahead H={H} "
                                   f"C={C}, {args.scenario or ('sudden' if args.track == 'ETHZMobil' else 'gradual')} friction",
                       "N_models_total": N_total,
                       "N_models_per_gpu": N_local, "H": H, "C": C, "W": W, "K": K, "Ts": 0.02,
                       "track": args.track, "parallelism": f"bank-shard x{world}" + (f" + 1 exchange/tick ({sb.transport})" if sb.exchange else ""),
                       "transport": sb.transport, "transport_fallback": sb.fallback_reason},
            "value_basis": "resident inputs: ms_per_step = wall time per tick of llampc_plan_device (ONE launch"
                           + (" + the exchange" if sb.exchange else "") + ") on tick inputs already in HBM, "
                           "K ticks back to back; plan_call_us is the same tick with H2D of its inputs and "
                           "D2H of its record, timed alone",
            "plan_call_us": call,
            "roofline": roof,
            "valu": {"bound": "fp64-valu", "achieved_gflops": valu_gf, "peak_tflops": FP64_VALU_PEAK_TFLOPS,
                     "frac": valu_gf / (FP64_VALU_PEAK_TFLOPS * 1e3) if valu_gf else None,
                     "flops_per_model_step": FLOPS_PER_MODEL_STEP,
                     "note": "plain flops only; the 29 fp64 transcendentals per RK4 step are excluded"},
            "issue": issue_roofline(N_local, C, H, lpm_of(N_local, C), plan_ms),
            "kernel_us": {"plan": plan_ms * 1e3, "events": int(cnt[0]),
                          "exchange": exch_ms * 1e3 if exch_ms is not None else None,
                          "bracket": (f"one tick in every {TIMING_SAMPLE}: its plan launch and its exchange (run as its "
                                      "own kernel on that tick) each bracketed by an event pair; max over ranks")
                                     if sb.exchange else
                                     f"one event pair around all {args.steps} timed plan launches: stream time per "
                                     "launch (includes any gap between launches; rocprof's kernel average beside it "
                                     "in profiles/ is the per-dispatch duration)"},
            "exchange": EXCHANGE_DESC[sb.transport] if sb.exchange else None,
            # the event pair measures stream time: if the host enqueued the launches barely faster
            # than they ran, gaps between launches would count as kernel time
            "kernel_time_host_bound_suspect": bool(plan_ms > 0 and t_issue / args.steps * 1e3 > 0.8 * plan_ms),
            "host_issue_us_per_step": t_issue / args.steps * 1e6,
            "lpm": lpm_of(N_local, C),
            "result_check": {"sel_model": merged.best_model, "window_full": merged.window_full,
                             "window_full_every_timed_tick": bool(count_before >= W),
                             "untimed_ticks_before": fill,
                             "sel_cand": merged.best_cand, "n_nonfinite": merged.n_nonfinite},
            "cpu_baseline": None,
        }
        line.update(extra)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    sb.close()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def plan_call_latency(args, sb, stream, ticks, world, n=1000, warm=50):
    """Per-plan() wall time as SURVEY.md §8(d) defines it: HIP events on the tick's stream
    around [H2D of the tick's input pack from pinned host memory -> the tick (one launch; with
    world > 1 the exchange too) -> D2H of the (merged) record into pinned host memory], one
    tick at a time (each waited for), p50/p99 over n ticks after `warm`; max over ranks."""
    import torch
    from llampc import _native as nat
    dev = torch.device("cuda", sb.device)
    T = len(ticks)
    h_in = [torch.from_numpy(np.ascontiguousarray(t)).pin_memory() for t in ticks]
    d_in = torch.empty(ticks.shape[1], dtype=torch.float64, device=dev)
    h_out = torch.empty(nat.PLAN_OUT_BYTES, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize(dev)
    pin = sb.make_plan_in(d_in, args.C, args.H, K=args.K)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lat = []
    for i in range(n + warm):
        with torch.cuda.stream(stream):
            e0.record(stream)
            d_in.copy_(h_in[i % T], non_blocking=True)
            sb.launch(pin, stream)
            h_out.copy_(sb.d_merged, non_blocking=True)
            e1.record(stream)
        e1.synchronize()
        if i >= warm:
            lat.append(e0.elapsed_time(e1) * 1e3)
    lat = np.array(lat)
    p50, p99 = float(np.percentile(lat, 50)), float(np.percentile(lat, 99))
    if world > 1:
        p50, p99 = max_over_ranks(p50), max_over_ranks(p99)
    return {"p50": p50, "p99": p99, "ticks": int(lat.size),
            "rollout_steps_per_s_at_p50": (args.n_per_gpu * world * (args.C * args.H + 1)) / (p50 * 1e-6),
            "note": "hipEvent-timed on the tick stream: H2D input pack + plan launch"
                    + (" + exchange" if world > 1 else "") + " + D2H record, one tick at a time"}


def extras(args, sb, stream, world, rank=0):
    """Extras reported by rank 0: C=64 throughput on the same bank (run on EVERY rank — each
    tick includes the exchange); at world 1, synchronous per-tick latency through the
    host-pointer API and BASELINE config 5 with host pointers (PCIe-inclusive); at world > 1,
    BASELINE config 5 sharded over the ranks.  Never the headline value."""
    import torch
    out = {}
    H = args.H
    a2 = argparse.Namespace(**vars(args))
    a2.C = 64
    t64 = make_ticks(a2, 8)
    p64 = torch.from_numpy(t64).to(torch.device("cuda", sb.device))
    torch.cuda.synchronize()
    pins = [sb.make_plan_in(p64[i], 64, H, K=args.K) for i in range(8)]
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    for i in range(5):
        sb.launch(pins[i % 8], stream)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for i in range(n):
        sb.launch(pins[i % 8], stream)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / n * 1e3
    Nt = args.n_per_gpu * world
    if world > 1:
        ms = max_over_ranks(ms)
    out["C64"] = {"ms_per_step": ms, "value": (Nt * 64 * H + Nt) / (ms / 1e3),
                  "issue": issue_roofline(args.n_per_gpu, 64, H, lpm_of(args.n_per_gpu, 64), ms)}
    if world == 1:
        pk = make_ticks(args, 1)[0]
        C = args.C
        xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
        U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
        lat = []
        for i in range(1050):                 # >= 1000 ticks after 50 warm-up
            t0 = time.perf_counter()
            sb.bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=args.K)
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat[50:]) * 1e6
        out["sync_plan_latency_us"] = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                       "ticks": int(lat.size),
                                       "note": "host-pointer llampc_plan from Python: inputs as kernel arguments, record via pinned host memory + completion-tag spin"}
        # the same call paced at the controller's period (rt.py: Ts = 0.02 s simulated, a 1 kHz
        # loop in BASELINE config 5): the GPU idles ~0.96 ms between ticks, so every tick runs
        # in the cold-clock regime that back-to-back ticks leave after ~600 launches
        period = 1e-3
        lat = []
        nxt = time.perf_counter() + period
        for i in range(1050):
            while time.perf_counter() < nxt:
                pass
            nxt += period
            t0 = time.perf_counter()
            sb.bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=args.K)
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat[50:]) * 1e6
        out["paced_plan_latency_us"] = {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                        "max": float(lat.max()), "ticks": int(lat.size), "period_us": period * 1e6,
                                        "note": "sync_plan_latency's call, one tick per 1 ms period (busy-wait pacing)"}
        # (one process: an extra that fails is reported in the line, not fatal to the headline)
        for key, fn in (("config5", concurrent_tracks), ("config3", config3), ("controller_tick_us", controller_ticks),
                        ("solve_us", solve_latency)):
            try:
                out[key] = fn(args)
            except Exception as e:          # noqa: BLE001
                out[key] = {"error": f"{type(e).__name__}: {e}"}
    else:
        # every rank runs each extra (they exchange every tick); a failure on any rank is
        # reported in the line, decided over the ranks, and never costs the headline
        for key, fn in (("config5", concurrent_tracks_sharded), ("controller_tick_us", controller_ticks_sharded)):
            val, err = None, None
            try:
                val = fn(args, world, rank, sb.device)
            except Exception as e:          # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
                print(f"bench.py: rank {rank}: extra {key} failed: {err}", file=sys.stderr, flush=True)
            failed = max_over_ranks(1.0 if err is not None else 0.0) > 0
            out[key] = val if not failed else {"error": err or "failed on another rank"}
    return out


def controller_ticks_sharded(args, world, rank, dev_index, ticks=1000, warm=60, period=1e-3, H=40, C=64):
    """BASELINE config 5's real loop across the ranks: LLAMPC.tick (device mode) on an ETHZ and an
    ETHZMobil bank of N_per_gpu x world models each, every bank sharded over the ranks (each
    tick exchanges the shards' top-K + argmin over the ShardedBank's transport, every rank merges
    and rolls out the merged selection's K + 1 models), both tracks ticked concurrently
    (tick_begin on both, then tick_end), paced at 1 kHz; p50/p99/max of the step, max over ranks.
    The plant (the host oracle's RK6 would cost ms; the device RK6) advances each car between
    steps, outside the timed region — every rank applies the same control."""
    import torch.distributed as dist
    from llampc.models import Dynamic
    from llampc.mpc import LLAMPC, generate_bank
    from llampc.mpc.sharded import ShardedBank
    from llampc.params import ORCA
    from llampc.tracks import ETHZ, ETHZMobil, dyn_slice
    p = ORCA()
    setups = []
    try:
        for seed, tr in ((0, ETHZ('optimal', True)), (1, ETHZMobil('optimal', True))):
            sb = ShardedBank(generate_bank(args.n_per_gpu * world, seed=seed), rank, world, dev_index, W=args.W)
            # the controllers ticked together on this device: two tracks, times the ranks when a
            # one-GPU rehearsal puts every rank on it (LLAMPC_SAME_DEVICE) — an armed launch's
            # blocks must all be resident (llampc_bank_set_concurrency sizes its spec blocks)
            sb.bank.set_concurrency(2 * (world if os.environ.get("LLAMPC_SAME_DEVICE") else 1))
            ctl = LLAMPC(sb, tr, H=H, C=C, K=args.K, mode="device")
            plant = Dynamic(**p, device=dev_index)
            if tr.name == "ETHZ":
                x = dyn_slice()["states"][:, 0].copy()
            else:
                x = np.array([tr.x_init, tr.y_init, tr.psi_init, 1.0, 0.0, 0.0])
            setups.append([sb, ctl, plant, x])
        dist.barrier()
        lat, devt = [], []
        # every rank's step starts at the same instant (one x_t for the whole node, as from one
        # sensor): the ranks pace to a common CLOCK_MONOTONIC epoch (one clock per host), so a
        # step's latency holds no skew between the ranks' own timers
        nxt = max_over_ranks(time.monotonic() + 0.005)
        for i in range(ticks + warm):
            nxt = pace(nxt, period, time.monotonic)
            t0 = time.perf_counter()
            for s in setups:
                s[1].tick_begin(s[3])
            res = [s[1].tick_end() for s in setups]
            lat.append(time.perf_counter() - t0)
            devt.append([s[1].device_us() for s in setups])
            for s, r in zip(setups, res):
                pl = s[2]
                pl.Df -= pl.Df / 2600.
                pl.Dr -= pl.Dr / 2600.
                xn, _ = pl.sim_continuous(s[3], r.u_seq[:, 0].reshape(2, 1), [0, 0.02])
                s[3] = xn[:, -1]
        sel = [int(r.best_model) for r in res]
        transports = [s[1]._ctl.transport for s in setups]
    finally:
        for s in setups:
            s[1].close()
        dist.barrier()
        for s in setups:
            s[0].close()
    q = pctl(np.array(lat[warm:]) * 1e6)
    p50, p99, mx = max_over_ranks(q["p50"]), max_over_ranks(q["p99"]), max_over_ranks(q["max"])
    dv = np.array(devt[warm:], dtype=np.float64).ravel()
    dv = dv[np.isfinite(dv)]
    device_us = {"p50": max_over_ranks(float(np.percentile(dv, 50))), "p99": max_over_ranks(float(np.percentile(dv, 99))),
                 "note": "llampc_ctl_device_us per tick and track (x_t on the device -> the record's stores issued, "
                         "the exchange included), max over ranks"} if dv.size else None
    N, K = args.n_per_gpu, args.K
    steps_tick = N * world + (K + 1) * C * H
    return {"p50": p50, "p99": p99, "max": mx, "ticks": q["ticks"], "period_us": period * 1e6, "budget_us": 1000.0,
            "device_us": device_us, "armed": [bool(s[1]._ctl.prelaunch) for s in setups],
            "paced": "every rank to a common CLOCK_MONOTONIC epoch (the same step start on all ranks)",
            "met": p99 < 1000.0, "tracks": ["ETHZ", "ETHZMobil"], "N_per_track": N * world, "N_per_track_per_gpu": N,
            "H": H, "C": C, "K": K, "W": args.W, "sel_models": sel, "transport": transports,
            "rollout_steps_per_tick": steps_tick, "rollout_steps_per_s_at_p50": 2 * steps_tick / (p50 * 1e-6),
            "note": "LLAMPC.tick (device mode) on banks sharded over the ranks: the selection exchanged every "
                    "tick over `transport` (peer: inside the tick's one launch, llampc_ctl_set_exchange; rccl: "
                    "ncclAllGather between the tick's two launches; host/c10d: the records carried by the "
                    "process group between them, llampc_ctl_set_gather), two tracks concurrently, paced at "
                    "1 ms; max over ranks"}


def concurrent_tracks_sharded(args, world, rank, dev_index, ticks=1000, warm=50):
    """BASELINE config 5 across the ranks: an ETHZ bank (seed 0) and an ETHZMobil bank (seed
    1) of N_per_gpu x world models each, H = 40, both sharded over the ranks (each with its own
    exchange); every control step ticks BOTH — one launch each on its own stream, device-resident
    inputs — and reads both merged records back into pinned host memory; p50/p99 of the step
    (max over ranks) against the 1 ms budget (1 kHz control loop)."""
    import torch
    import torch.distributed as dist
    from llampc import _native as nat
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank
    H = 40
    dev = torch.device("cuda", dev_index)
    sbs, pins, hbuf = [], [], []
    try:
        for seed, track in ((0, "ETHZ"), (1, "ETHZMobil")):
            a = argparse.Namespace(**vars(args))
            a.track, a.H, a.C, a.scenario = track, H, 1, None
            t = make_ticks(a, 8)
            sb = ShardedBank(generate_bank(args.n_per_gpu * world, seed=seed), rank, world, dev_index, W=args.W)
            sb.bank.set_concurrency(2)    # the two tracks' launches share each GPU
            sbs.append(sb)
            packs = torch.from_numpy(t).to(dev)
            torch.cuda.synchronize(dev)
            pins.append([sb.make_plan_in(packs[i], 1, H, K=args.K) for i in range(len(t))])
            hbuf.append(torch.empty(nat.PLAN_OUT_BYTES, dtype=torch.uint8).pin_memory())
        dist.barrier()
        lat = []
        for i in range(ticks + warm):
            t0 = time.perf_counter()
            for sb, pl, hb in zip(sbs, pins, hbuf):
                s = sb.launch(pl[i % len(pl)], sb.stream)
                with torch.cuda.stream(s):
                    hb.copy_(sb.d_merged, non_blocking=True)
            for sb in sbs:
                sb.stream.synchronize()
            lat.append(time.perf_counter() - t0)
        sel = [int(nat.PlanOut.from_buffer_copy(hb.numpy().tobytes()).sel_model) for hb in hbuf]
        transports = [sb.transport for sb in sbs]
    finally:
        for sb in sbs:
            sb.close()
    lat = np.array(lat[warm:]) * 1e6
    p50, p99 = float(np.percentile(lat, 50)), float(np.percentile(lat, 99))
    p50, p99 = max_over_ranks(p50), max_over_ranks(p99)
    return {"p50_us": p50, "p99_us": p99, "ticks": int(lat.size), "budget_us": 1000.0, "met": p99 <= 1000.0,
            "N_per_track": args.n_per_gpu * world, "N_per_track_per_gpu": args.n_per_gpu, "H": H,
            "sel_models": sel, "transport": transports,
            "note": "two sharded plan() instances per control step (ETHZ + ETHZMobil), each one launch with "
                    "its own exchange on its own stream, device-resident inputs, both merged records read back"}


def pace(nxt, period, clock=time.perf_counter):
    """Busy-wait to the next period boundary (the 1 kHz control loop); returns the next one."""
    while clock() < nxt:
        pass
    return nxt + period


def pctl(lat_us):
    lat = np.asarray(lat_us)
    return {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)), "max": float(lat.max()),
            "ticks": int(lat.size)}


def concurrent_tracks(args, ticks=1000, warm=50, period=1e-3):
    """BASELINE config 5 on one GPU: ETHZ and ETHZMobil banks (N_per_gpu each, H=40) ticked
    concurrently every control step — llampc_plan_async on both, then llampc_plan_wait on
    both (host pointers: inputs as kernel arguments, the record through pinned host memory) —
    PACED at the 1 kHz control period (each step starts on a period boundary, the GPU idles in
    between, as in the real loop), p50/p99/max of the per-step latency against the 1 ms budget;
    the same steps back to back are reported beside it."""
    from llampc.mpc import ModelBank, generate_bank
    H, W, K = 40, args.W, args.K
    banks, inputs = [], []
    for seed, track in ((0, "ETHZ"), (1, "ETHZMobil")):
        a = argparse.Namespace(**vars(args))
        a.track, a.H, a.C = track, H, 1
        t = make_ticks(a, 8)
        banks.append(ModelBank(generate_bank(args.n_per_gpu, seed=seed), W=W, device=torch_device_index()))
        banks[-1].set_concurrency(2)      # two launches share the chip (llampc_bank_set_concurrency)
        inputs.append(t)

    def step(i):
        t0 = time.perf_counter()
        for b, t in zip(banks, inputs):
            pk = t[i % len(t)]
            b.plan_async(pk[0:6], pk[6:8], pk[8:14], pk[16 + 2 * (H + 1):].reshape(1, H, 2),
                         pk[16:16 + 2 * (H + 1)].reshape(2, H + 1), pk[14:16], K=K)
        outs = [b.plan_wait() for b in banks]
        return time.perf_counter() - t0, outs

    paced, b2b = [], []
    try:
        nxt = time.perf_counter() + period
        for i in range(ticks + warm):
            nxt = pace(nxt, period)
            dt, outs = step(i)
            paced.append(dt)
        for i in range(ticks // 2 + warm):
            dt, outs = step(i)
            b2b.append(dt)
    finally:
        for b in banks:
            b.close()
    p = pctl(np.array(paced[warm:]) * 1e6)
    q = pctl(np.array(b2b[warm:]) * 1e6)
    return {"p50_us": p["p50"], "p99_us": p["p99"], "max_us": p["max"], "ticks": p["ticks"], "period_us": period * 1e6,
            "budget_us": 1000.0, "met": p["p99"] <= 1000.0, "N_per_track": args.n_per_gpu, "H": H, "C": 1,
            "back_to_back": q,
            "sel_models": [int(o.sel_model) for o in outs],
            "note": "two independent plan() instances per control step (ETHZ + ETHZMobil), async on two streams, "
                    "host pointers in and the record read back, each bank sized for half the chip "
                    "(set_concurrency(2)); paced: one step per 1 ms period (busy-wait)"}


def config3(args, steps=200, warmup=20):
    """BASELINE config 3 in the driver's line: ETHZMobil, N_per_gpu models, H = 40, C = 1, the
    sudden friction drop — K ticks of llampc_plan_device on resident inputs (the headline's
    method: one HIP-event pair around the timed loop for the kernel time)."""
    import torch
    from llampc import _native as nat
    from llampc.mpc import generate_bank
    from llampc.mpc.sharded import ShardedBank
    a = argparse.Namespace(**vars(args))
    a.track, a.H, a.C, a.scenario = "ETHZMobil", 40, 1, "sudden"
    ticks = make_ticks(a, 64)
    dev = torch.device("cuda", torch_device_index())
    packs = torch.from_numpy(ticks).to(dev)
    torch.cuda.synchronize()
    sb = ShardedBank(generate_bank(args.n_per_gpu, seed=1), 0, 1, torch_device_index(), W=args.W)
    lib = nat.load()
    try:
        pins = [sb.make_plan_in(packs[i], 1, 40, K=args.K, current_model=0) for i in range(len(ticks))]
        nat.check(lib.llampc_bank_timing(sb.bank.handle, steps, 4))
        for i in range(warmup):
            sb.launch(pins[i % len(pins)], sb.stream)
        avg = (ctypes.c_double * 3)()
        cnt = (ctypes.c_int64 * 3)()
        nat.check(lib.llampc_bank_timing_read(sb.bank.handle, avg, cnt))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            sb.launch(pins[(warmup + i) % len(pins)], sb.stream)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        nat.check(lib.llampc_bank_timing_read(sb.bank.handle, avg, cnt))
        res = sb.fetch(sb.stream)
    finally:
        sb.close()
    N = args.n_per_gpu
    return {"ms_per_step": ms, "value": (N * 40 + N) / (ms / 1e3), "kernel_us": avg[0] * 1e3, "steps": steps,
            "warmup": warmup, "N": N, "H": 40, "C": 1, "track": "ETHZMobil", "scenario": "sudden",
            "sel_model": res.best_model,
            "note": "llampc_plan_device on resident inputs, one event pair around the timed loop"}


def controller_ticks(args, ticks=1000, warm=60, period=1e-3, H=40, C=64):
    """The real control loop (verdict r03 #1): LLAMPC.tick in device mode — ONE launch per
    step computing the ConstantSpeed reference with mu-hat, the candidates, the look-back and
    selection, the look-ahead of the selected and top-K models, mu-hat and the controller state
    — for an ETHZ and an ETHZMobil controller CONCURRENTLY (tick_begin on both, then
    tick_end), H = 40, C = 64, N_per_gpu models each, paced at 1 kHz; p50/p99/max of the step
    (both ticks + the Python results) against the 1 ms budget.  The plant (the device RK6,
    Dynamic.sim_continuous under the gradual friction decay) advances each car between
    steps, outside the timed region."""
    from llampc import _native as nat
    from llampc.models import Dynamic
    from llampc.mpc import LLAMPC, ModelBank, generate_bank
    from llampc.params import ORCA
    from llampc.tracks import ETHZ, ETHZMobil, dyn_slice
    dev = torch_device_index()
    p = ORCA()
    setups = []
    for seed, tr in ((0, ETHZ('optimal', True)), (1, ETHZMobil('optimal', True))):
        b = ModelBank(generate_bank(args.n_per_gpu, seed=seed), W=args.W, device=dev)
        b.set_concurrency(2)                # two controllers tick together: a hardware queue each
        ctl = LLAMPC(b, tr, H=H, C=C, K=args.K, mode="device")
        plant = Dynamic(**p, device=dev)
        if tr.name == "ETHZ":
            x = dyn_slice()["states"][:, 0].copy()
        else:
            x = np.array([tr.x_init, tr.y_init, tr.psi_init, 1.0, 0.0, 0.0])
        setups.append([b, ctl, plant, x])
    lat, kern, split, devt = [], [], [], []
    lib = nat.load()
    ev_ticks = 100                          # after the timed steps: per-launch event pairs for
    try:                                    # the kernel time (their cost stays out of lat)
        nxt = time.perf_counter() + period
        for i in range(ticks + warm + ev_ticks):
            if i == warm + ticks:             # launched ticks: an armed launch's events hold its wait
                for s in setups:
                    s[1].set_prelaunch(False)
                    nat.check(lib.llampc_bank_timing(s[0].handle, 1, ev_ticks + 8))
            nxt = pace(nxt, period)
            t0 = time.perf_counter()
            for s in setups:
                s[1].tick_begin(s[3])
            t1 = time.perf_counter()
            res = [s[1].tick_end() for s in setups]
            t2 = time.perf_counter()
            lat.append(t2 - t0)
            split.append((t1 - t0, t2 - t1))
            devt.append([s[1].device_us() for s in setups])
            for s, r in zip(setups, res):     # the plant (outside the timed step)
                pl = s[2]
                pl.Df -= pl.Df / 2600.
                pl.Dr -= pl.Dr / 2600.
                xn, _ = pl.sim_continuous(s[3], r.u_seq[:, 0].reshape(2, 1), [0, 0.02])
                s[3] = xn[:, -1]
        avg = (ctypes.c_double * 3)()
        cnt = (ctypes.c_int64 * 3)()
        for s in setups:
            nat.check(lib.llampc_bank_timing_read(s[0].handle, avg, cnt))
            kern.append(avg[0] * 1e3)
        laps = [int(s[1].projidx) for s in setups]
        sel = [int(r.best_model) for r in res]
    finally:
        for s in setups:
            s[1].close()
            s[0].close()
    q = pctl(np.array(lat[warm:warm + ticks]) * 1e6)
    dv = np.array(devt, dtype=np.float64)
    def dpct(a):
        a = a[np.isfinite(a)]
        return {"p50": float(np.percentile(a, 50)), "p99": float(np.percentile(a, 99)), "max": float(a.max())} if a.size else None
    device_us = {"armed": dpct(dv[warm:warm + ticks].ravel()), "launched": dpct(dv[warm + ticks + 8:].ravel()),
                 "note": "llampc_ctl_device_us per tick and track: x_t on the device (armed: block 0 sees the "
                         "doorbell; launched: block 0 starts) to the record's stores issued, by the GPU's 100 MHz "
                         "clock; armed = the timed steps, launched = the event-timed steps after them"}
    N, K, W = args.n_per_gpu, args.K, args.W
    steps_tick = N + (K + 1) * C * H              # look-back steps + the (K+1) x C rollouts' steps
    # algorithmic HBM bytes of one controller launch: the look-back's params + ring read/write per
    # model, the rolled-out models' params, the raceline tables one block stages (knots + two
    # speed profiles), the candidates' variates read and the next tick's written, the state and
    # the record
    m = 700                                       # raceline knots (ETHZ 700, Mobil 500: upper)
    ctl_bytes = N * (48 + 8 * W + 8) + (K + 1) * 48 + 8 * m + 64 * (m - 1) + 2 * 16 * C * H + 2 * 1024 + 2048
    lane_instr = (K + 1) * C * H * 4 * CTL_INSTR_PER_STEP + N * LOOKBACK_INSTR_PER_MODEL
    kmean = float(np.mean(kern)) if kern else 0.0
    issue = None
    if kmean > 0:
        ach = lane_instr / (kmean * 1e-6)
        issue = {"bound": "fp64-valu-issue", "achieved": ach, "peak": ISSUE_PEAK_LANE_INSTR,
                 "unit": "lane-instructions/s", "frac": ach / ISSUE_PEAK_LANE_INSTR, "lane_instr_per_launch": lane_instr,
                 "pmc": pmc_issue("ctl_kernel", kmean),
                 "note": f"static count: (K+1) C H rollout steps x 4 lanes x {CTL_INSTR_PER_STEP} + N x "
                         f"{LOOKBACK_INSTR_PER_MODEL} (look-back, upper bound) over the mean launch; pmc: "
                         "SQ_INSTS_VALU x 64 of the committed PMC pass over the same launch time"}
    extra_ctl = {"rollout_steps_per_tick": steps_tick,
                 "spec_models": 32,
                 "spec_note": "armed ticks also roll out the 32 best models by the window mean without x_t from the "
                              "doorbell on (CtlLaunch.n_spec; 32 C H further steps per tick, not counted above): the "
                              "selected ones are not rolled out again",
                 "rollout_steps_per_s_at_p50": 2 * steps_tick / (q["p50"] * 1e-6),
                 "bytes_per_launch": ctl_bytes,
                 "hbm_frac": (ctl_bytes / (kmean * 1e-6) / 1e9 / HBM_PEAK_GBS) if kmean > 0 else None,
                 "issue": issue}
    return {"p50": q["p50"], "p99": q["p99"], "max": q["max"], "ticks": q["ticks"], "period_us": period * 1e6,
            "budget_us": 1000.0, "met": q["p99"] < 1000.0, "tracks": ["ETHZ", "ETHZMobil"],
            "N_per_track": args.n_per_gpu, "H": H, "C": C, "K": args.K, "W": args.W,
            "kernel_us_avg": kern, "device_us": device_us, "sel_models": sel, "projidx": laps, **extra_ctl,
            "host_split_us_p50": {"begin": float(np.median([a for a, _ in split[warm:warm + ticks]]) * 1e6),
                                  "end": float(np.median([b for _, b in split[warm:warm + ticks]]) * 1e6)},
            "note": "LLAMPC.tick (device mode, llampc_ctl_tick_async/wait: one launch per track per step, armed "
                    "during the previous step and rung with x_t — llampc_ctl_set_prelaunch) for two tracks "
                    "concurrently, paced at 1 ms; kernel_us_avg = per-launch HIP events of each bank's "
                    "controller launch over 100 further LAUNCHED steps (the timed steps carry no events)"}


def solve_latency(args, n=200, warm=10, H=20):
    """The setupNLP.solve drop-in (llampc_nlp_solve: the selected model's NMPC, nmpc.py:161-203,
    minimised on the device by the cross-entropy search — 1,024 samples x 8 rounds, elite 32 —
    with ONE copy back) called from Python per control step on successive DYN-slice states,
    p50/p99/max; the reference's published figure for its whole control step with IPOPT is
    0.03 s (results/table1.png)."""
    from llampc.models import Dynamic
    from llampc.mpc.nmpc import setupNLP
    from llampc.mpc.planner import ConstantSpeed
    from llampc.params import ORCA
    from llampc.tracks import ETHZ
    from llampc.tracks import dyn_slice
    d = dyn_slice()
    s, u = d["states"], d["inputs"]
    tr = ETHZ('optimal', True)
    p = ORCA(control="pwm")
    nlp = setupNLP(H, 0.02, np.eye(2), np.zeros((2, 2)), np.diag([5e-3, 1]), p, Dynamic(**p, device=torch_device_index()),
                   tr, device=torch_device_index())
    cases, projidx = [], 0
    for t in range(10, 10 + 40):
        xref, projidx, _ = ConstantSpeed(s[:2, t], s[3, t], tr, H, 0.02, projidx)
        cases.append((s[:, t].copy(), xref, u[:, t - 1].copy()))
    lat, fv = [], []
    from llampc import _native as nat
    lib = nat.load()
    avg = (ctypes.c_double * 3)()
    cnt = (ctypes.c_int64 * 3)()
    try:
        for i in range(n + warm):               # the latency: no per-launch events
            x0, xref, up = cases[i % len(cases)]
            t0 = time.perf_counter()
            _, fval, _, _ = nlp.solve(x0, xref, up)
            lat.append(time.perf_counter() - t0)
            fv.append(fval)
        # then the kernel's own duration: per-launch HIP events on the solver's bank, a pass of
        # its own (the events' records are host work inside the call)
        nat.check(lib.llampc_bank_timing(nlp._bank.handle, 1, n + 8))
        for i in range(n):
            x0, xref, up = cases[i % len(cases)]
            nlp.solve(x0, xref, up)
        nat.check(lib.llampc_bank_timing_read(nlp._bank.handle, avg, cnt))
    finally:
        nlp.close()
    q = pctl(np.array(lat[warm:]) * 1e6)
    kus = avg[0] * 1e3
    steps = nlp.samples * nlp.iters * H
    lane_instr = steps * 4 * NLP_INSTR_PER_STEP
    nlp_bytes = nlp.iters * (nlp.samples * (16 * H + 16 * H + 16)) + 16 * (H + 1) + 48 * H + 6 * 8 * (H + 1)
    issue = None
    if kus > 0:
        ach = lane_instr / (kus * 1e-6)
        issue = {"bound": "fp64-valu-issue", "achieved": ach, "peak": ISSUE_PEAK_LANE_INSTR,
                 "unit": "lane-instructions/s", "frac": ach / ISSUE_PEAK_LANE_INSTR, "lane_instr_per_launch": lane_instr,
                 "pmc": pmc_issue("nlp_kernel", kus),
                 "note": f"static count: samples x rounds x H steps x 4 lanes x {NLP_INSTR_PER_STEP} over the "
                         "launch (all rounds in one launch); pmc: SQ_INSTS_VALU x 64 of the committed PMC pass"}
    return {"p50": q["p50"], "p99": q["p99"], "max": q["max"], "solves": q["ticks"], "H": H,
            "samples": nlp.samples, "rounds": nlp.iters, "elite": nlp.elite,
            "kernel_us_avg": kus, "launches_timed": int(cnt[0]), "rollout_steps_per_solve": steps,
            "rollout_steps_per_s_at_p50": steps / (q["p50"] * 1e-6), "bytes_per_launch": nlp_bytes,
            "issue": issue,
            "reference_s_per_control_step": 0.03, "fval_p50": float(np.median(fv)),
            "note": "setupNLP(...).solve from Python: the CEM rounds back to back on the GPU + the Euler "
                    "trajectory + one copy back (the latency pass without per-launch events; kernel_us_avg "
                    "from a second pass with them); the reference's 0.03 s is its whole tick incl. IPOPT "
                    "(unstated hardware)"}


def issue_roofline(n, C, H, lpm, ms):
    """fp64 VALU issue roofline of the plan kernel: lane-instructions of the look-ahead
    rollouts (+ the look-back's one LPM-1 step per model) per launch / the launch's mean
    duration, against the chip's issue capacity.  The binding resource of this kernel."""
    if not ms or ms <= 0:
        return None
    lane_instr = n * C * H * lpm * ISSUE_INSTR_PER_STEP[lpm] + n * ISSUE_INSTR_PER_STEP[1]
    achieved = lane_instr / (ms * 1e-3)
    return {"bound": "fp64-valu-issue", "achieved": achieved, "peak": ISSUE_PEAK_LANE_INSTR,
            "unit": "lane-instructions/s", "frac": achieved / ISSUE_PEAK_LANE_INSTR,
            "instr_per_step_per_lane": ISSUE_INSTR_PER_STEP[lpm], "lanes_per_rollout": lpm,
            "note": "a tick at C=1 is one rollout's instruction stream long (628 of 1,024 SIMDs "
                    "busy at LPM 4, ~4.75 cycles per instruction); C=64 fills the chip"}


def lpm_of(n, C):
    """Lanes per rollout the library picks (mirror of kernels.hip lookahead_lpm)."""
    G = 1
    while G < C and G < 256:
        G <<= 1
    env = os.environ.get("LLAMPC_LPM")
    if env == "1" or (env == "2" and G <= 128) or (env == "4" and G <= 64):
        return int(env)
    if n * G <= 16384 and G <= 64:
        return 4
    return 2 if (n * G <= 32768 and G <= 128) else 1


def pmc_issue(kernel: str, kernel_us: float):
    """Issue fraction of `kernel` from the committed PMC summary (profiles/r06/pmc_kernels.json,
    tools/pmc_kernels.py): SQ_INSTS_VALU wave-instructions per dispatch x 64 lanes / kernel_us /
    the chip's issue capacity; None when no pass is committed for the kernel."""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "r06", "pmc_kernels.json")))
    except (OSError, ValueError):
        return None
    v = d.get(kernel)
    if not v or not kernel_us:
        return None
    lane = v["SQ_INSTS_VALU"] * 64
    return {"lane_instr_per_launch": lane, "frac": lane / (kernel_us * 1e-6) / ISSUE_PEAK_LANE_INSTR,
            "source": "profiles/r06/pmc_kernels.json"}


def pmc_traffic(args):
    """HBM bytes per look-ahead launch from a committed rocprofv3 --pmc summary (None if
    absent for this config): profiles/pmc_lookahead.json written by tools/pmc_summary.py."""
    path = os.path.join(REPO, "profiles", "pmc_lookahead.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    key = f"{args.track}_N{args.n_per_gpu}_H{args.H}_C{args.C}"
    v = d.get(key)
    return None if v is None else v.get("hbm_bytes_per_launch")


if __name__ == "__main__":
    main()
