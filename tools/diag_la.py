"""Diagnostic (not product): phase stamps of the first 8 look-ahead blocks (stamps build)."""
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
for t in range(1, 30):
    b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1])
st = (ctypes.c_ulonglong * (8 * 8 * 2))()
fn = lib.llampc_debug_la_stamps
fn.argtypes = [ctypes.c_void_p]
fn(st)
a = np.frombuffer(st, dtype=np.uint64).reshape(8, 8, 2).astype(np.int64)
t0 = a[:, 0, 1].min()
for blk in range(8):
    mt, rt = a[blk, :4, 0], a[blk, :4, 1]
    clk = (mt[3] - mt[0]) / max(1, rt[3] - rt[0]) * 100       # s_memrealtime ticks at 100 MHz
    print(f"la block {blk}: start +{(rt[0]-t0)/100:.2f}us | cycles: staging {mt[1]-mt[0]}, rollout {mt[2]-mt[1]} "
          f"({(mt[2]-mt[1])/20:.0f}/step), reduce {mt[3]-mt[2]} | {(rt[3]-rt[0])/100:.2f}us  clock {clk:.0f} MHz")
