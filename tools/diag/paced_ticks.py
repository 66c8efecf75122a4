"""Host-pointer ticks at a fixed period (diagnostic for the controller's 1 kHz regime): run
under rocprofv3 --kernel-trace to see the plan kernel's duration when the GPU idles between
ticks.  usage: python tools/diag/paced_ticks.py [period_us] [ticks]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "lla-mpc_amd"))
import bench  # noqa: E402  (tick inputs of the headline workload)


def main():
    period = float(sys.argv[1]) * 1e-6 if len(sys.argv) > 1 else 1e-3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    from llampc.mpc import ModelBank, generate_bank
    sys.argv = sys.argv[:1]
    args = bench.parse()                # the headline workload's defaults
    pk = bench.make_ticks(args, 1)[0]
    H, C = args.H, args.C
    xref = pk[16:16 + 2 * (H + 1)].reshape(2, H + 1)
    U = pk[16 + 2 * (H + 1):].reshape(C, H, 2)
    bank = ModelBank(generate_bank(args.n_per_gpu, seed=0), W=args.W, device=0)
    lat = []
    nxt = time.perf_counter() + period
    for i in range(n):
        while time.perf_counter() < nxt:
            pass
        nxt += period
        t0 = time.perf_counter()
        bank.plan_raw(pk[0:6], pk[6:8], pk[8:14], U, xref, pk[14:16], K=args.K)
        lat.append(time.perf_counter() - t0)
    lat = np.array(lat[20:]) * 1e6
    print(f"period {period * 1e6:.0f} us, {lat.size} ticks: p50 {np.percentile(lat, 50):.1f} "
          f"p99 {np.percentile(lat, 99):.1f} us")
    bank.close()


if __name__ == "__main__":
    main()
