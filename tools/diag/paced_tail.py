"""Diagnostic: where the paced tick's tail comes from (verdict r03 #2).  Mode "run": the
headline workload's host-pointer tick (bank.plan_raw: inputs as kernel arguments, record via
pinned host memory — bench.py's paced_plan_latency_us call) at a 1 ms period, n ticks, the
wall time of every call saved to <out>.npy; run it under rocprofv3 --kernel-trace.  Mode
"split": matches the calls with the trace's plan-kernel dispatches (one per call, in order)
and splits every call into the kernel's duration and the rest (launch + completion trip +
Python), then shows the slowest 1 % of calls.
usage: python tools/diag/paced_tail.py run <out> [n] | split <out> <kernel_trace.csv>"""
import csv
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]


def run(out, n):
    import bench
    from llampc.mpc import ModelBank, generate_bank
    sys.argv = sys.argv[:1]
    args = bench.parse()
    pk = bench.make_ticks(args, 1)[0]
    H, C = args.H, args.C
    xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
    U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
    bank = ModelBank(generate_bank(args.n_per_gpu, seed=0), W=args.W, device=0)
    lat = []
    period = 1e-3
    nxt = time.perf_counter() + period
    for i in range(n):
        while time.perf_counter() < nxt:
            pass
        nxt += period
        t0 = time.perf_counter()
        bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=args.K)
        lat.append(time.perf_counter() - t0)
    bank.close()
    np.save(out, np.array(lat) * 1e6)
    q = np.array(lat[50:]) * 1e6
    print(f"paced host-pointer tick: p50 {np.median(q):.1f} p99 {np.percentile(q, 99):.1f} max {q.max():.1f} us")


def split(out, trace):
    lat = np.load(out + ".npy")
    rows = [r for r in csv.DictReader(open(trace)) if "plan_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.float64) / 1e3
    en = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.float64) / 1e3
    dur = (en - st)[-len(lat):]                 # the paced calls are the last dispatches
    gap = np.diff(st[-len(lat):], prepend=np.nan)
    lat, dur, gap = lat[50:], dur[50:], gap[50:]
    rest = lat - dur
    q = lambda v: f"p50 {np.median(v):.1f} p99 {np.percentile(v, 99):.1f} max {np.max(v):.1f}"  # noqa: E731
    print(f"calls {len(lat)}: wall {q(lat)} | kernel {q(dur)} | rest (launch + completion + Python) {q(rest)}")
    print(f"dispatch-to-dispatch period: p50 {np.nanmedian(gap):.1f} p99 {np.nanpercentile(gap, 99):.1f} us")
    idx = np.argsort(lat)[::-1][:max(1, len(lat) // 100)]
    print("slowest 1 %: wall / kernel / rest (us)")
    for i in idx:
        print(f"  call {i + 50:5d}: {lat[i]:7.1f} / {dur[i]:6.1f} / {rest[i]:7.1f}")
    k_share = np.corrcoef(lat, dur)[0, 1]
    print(f"correlation(wall, kernel) {k_share:.2f}; correlation(wall, rest) {np.corrcoef(lat, rest)[0, 1]:.2f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2000)
    else:
        split(sys.argv[2], sys.argv[3])
