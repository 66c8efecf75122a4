"""Diagnostic (not product): phase stamps of select_kernel from libllampc_hip_stamps.so."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["LLAMPC_HIP_LIB"] = os.path.join(REPO, "lla-mpc_amd/llampc/_lib/libllampc_hip_stamps.so")
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat
from llampc.mpc import ModelBank, generate_bank
lib = nat.load()
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N, H = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 20
b = ModelBank(generate_bank(N, 0), W=10, device=0)
xref = s[:2, :H + 1]
U = np.tile(u[:, 0], (H, 1))[None]
for t in range(1, 40):
    b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
st = (ctypes.c_ulonglong * (64 * 8 * 2))()
nl = ctypes.c_uint()
fn = lib.llampc_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
fn(st, ctypes.byref(nl))
a = np.frombuffer(st, dtype=np.uint64).reshape(64, 8, 2).astype(np.int64)
print("launches", nl.value)
for l in list(range(5, 12)) + [30, 38]:
    mt, rt = a[l, :6, 0], a[l, :6, 1]
    # slots 0-2: lb_final (stage+argmin, tree merge); 3-5: final_select; lb_final may be skipped
    print(f"launch {l:2d}: lb_final {mt[1]-mt[0]}, {mt[2]-mt[1]} cyc | final {mt[4]-mt[3]}, {mt[5]-mt[4]} cyc "
          f"= {(rt[5]-rt[3])*10/1000:.2f} us | lb_final end -> final start {(rt[3]-rt[2])*10/1000:.2f} us")
