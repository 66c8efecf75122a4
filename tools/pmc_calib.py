"""Calibration kernel for the rocprofv3 HBM counters (MI355X_MICROARCH.md §HBM: 8-B-per-lane
access widths are uncalibrated): llampc_math_batch fn 9 (math_kernel, a[i] / 6) streams
n doubles in and n doubles out, 8 B per lane, coalesced — the access shape of the plan
kernel's params/ring/cost traffic.  n = 2^26 (512 MB each way, beyond the 256 MB Infinity
Cache).  tools/pmc_traffic.py divides FETCH_SIZE/WRITE_SIZE of this dispatch by 8n."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
a = np.random.RandomState(0).standard_normal(n)
out = np.empty_like(a)
lib = nat.load()
nat.check(lib.llampc_math_batch(9, a.ctypes.data, None, n, out.ctypes.data, 0))
assert np.array_equal(out[:1000], a[:1000] / 6.0)
print(f"calibration dispatch: n={n} bytes_in={8 * n} bytes_out={8 * n}")
