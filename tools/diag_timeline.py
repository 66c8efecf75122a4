"""Diagnostic (not product): one tick's timeline from the stamps build — look-ahead blocks
(first 8: start, end of staging, end of rollout, end of reduction) and the completion stages
(lb_final, final_select) on the same s_memrealtime (100 MHz) clock."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LLAMPC_HIP_LIB", os.path.join(REPO, "lla-mpc_amd/llampc/_lib/libllampc_hip_stamps.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from llampc import _native as nat
from llampc.mpc import ModelBank, generate_bank
lib = nat.load()
d = np.load(os.path.join(REPO, "tests/golden/dyn_slice.npz"))
s, u = d["states"], d["inputs"]
N, H = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 20
LB_ONLY = len(sys.argv) > 2 and sys.argv[2] == "lb"
b = ModelBank(generate_bank(N, 0), W=10, device=0)
xref = s[:2, :H + 1]
U = np.tile(u[:, 0], (H, 1))[None]
kw = {}
if os.environ.get("RACELINE"):                # xref_mode RACELINE (per-model ConstantSpeed)
    from llampc.mpc.planner import raceline_start
    from llampc.tracks import ETHZ
    tr = ETHZ('optimal', True)
    b.set_raceline(tr)
    kw = dict(raceline_start=(raceline_start(s[:, 1], tr, 0)[0], float(s[3, 1]), 0.9))
for t in range(1, 30):
    b.plan_raw(s[:, t - 1], u[:, t - 1], s[:, t], U, xref, u[:, t - 1], do_lookahead=not LB_ONLY, **kw)
la = (ctypes.c_ulonglong * (8 * 8 * 2))()
lib.llampc_debug_la_stamps.argtypes = [ctypes.c_void_p]
lib.llampc_debug_la_stamps(la)
fs = (ctypes.c_ulonglong * (64 * 8 * 2))()
nl = ctypes.c_uint()
lib.llampc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
lib.llampc_debug_stamps(fs, ctypes.byref(nl))
A = np.frombuffer(la, dtype=np.uint64).reshape(8, 8, 2).astype(np.int64)[:, :4, 1]
lb = (ctypes.c_ulonglong * (8 * 8 * 2))()
lib.llampc_debug_lb_stamps.argtypes = [ctypes.c_void_p]
lib.llampc_debug_lb_stamps(lb)
B = np.frombuffer(lb, dtype=np.uint64).reshape(8, 8, 2).astype(np.int64)
F = np.frombuffer(fs, dtype=np.uint64).reshape(64, 8, 2).astype(np.int64)
l = (nl.value - 1) & 63
R = F[l, :6, 1]
B0 = np.frombuffer(lb, dtype=np.uint64).reshape(8, 8, 2).astype(np.int64)
t0 = B0[:, 0, 1].min() if LB_ONLY else A[:, 0].min()
us = lambda x: (x - t0) / 100.0
print(f"launches {nl.value}; times in us from the first look-ahead block start")
print(f"look-ahead blocks: start {us(A[:,0].min()):.2f}..{us(A[:,0].max()):.2f}, staging end ..{us(A[:,1].max()):.2f}, "
      f"rollout end {us(A[:,2].min()):.2f}..{us(A[:,2].max()):.2f}, reduce end ..{us(A[:,3].max()):.2f}")
for k in range(8):
    print(f"look-back block {k}: start {us(B[k,0,1]):.2f}, step+ring+mean end {us(B[k,1,1]):.2f}, "
          f"argmin end {us(B[k,2,1]):.2f}, top-K end {us(B[k,3,1]):.2f}  "
          f"(cycles {B[k,1,0]-B[k,0,0]}, {B[k,2,0]-B[k,1,0]}, {B[k,3,0]-B[k,2,0]})")
ALL = (ctypes.c_ulonglong * (1024 * 4 * 2))()
lib.llampc_debug_la_all.argtypes = [ctypes.c_void_p]
lib.llampc_debug_la_all(ALL)
Z = np.frombuffer(ALL, dtype=np.uint64).reshape(1024, 4, 2).astype(np.int64)
nla = int((Z[:, 3, 1] >= A[:, 0].min()).sum())
Z = Z[:nla]
q = lambda v: f"{np.min(v):.2f}/{np.median(v):.2f}/{np.max(v):.2f}"
print(f"all {nla} look-ahead blocks (min/median/max): start {q(us(Z[:,0,1]))}, staged {q(us(Z[:,1,1]))}, "
      f"rolled out {q(us(Z[:,2,1]))}, reduced {q(us(Z[:,3,1]))}")
cyc = Z[:, 2, 0] - Z[:, 1, 0]
rt = (Z[:, 2, 1] - Z[:, 1, 1]) / 100.0
print(f"rollout per block: {q(rt)} us, {q(cyc)} shader cycles, clock {np.median(cyc / rt) / 1e3:.2f} GHz")
R8 = F[l, :8, 1]
print(f"lb_final: {us(R[0]):.2f} (loads) -> {us(R[1]):.2f} (head ranks) -> {us(R8[6]):.2f} (candidates) -> "
      f"{us(R8[7]):.2f} (ranks, argmin) -> {us(R[2]):.2f}")
print(f"final_select: {us(R[3]):.2f} -> {us(R[4]):.2f} -> {us(R[5]):.2f}")

WV = (ctypes.c_ulonglong * (1024 * 4))()
if hasattr(lib, "llampc_debug_la_wave"):
    lib.llampc_debug_la_wave.argtypes = [ctypes.c_void_p]
    lib.llampc_debug_la_wave(WV)
    V = np.frombuffer(WV, dtype=np.uint64).reshape(1024, 4).astype(np.int64)[:nla]
    sk = (V.max(axis=1) - V.min(axis=1)) / 100.0
    w0 = (V - V.min(axis=1, keepdims=True)) / 100.0
    print(f"wave rollout-end skew per block (us): {q(sk)}; mean offset of waves 0..3 from the block's first: "
          + ", ".join(f"{x:.2f}" for x in w0.mean(axis=0)))

if os.environ.get("RACELINE") and hasattr(lib, "llampc_debug_rl"):
    RD = (ctypes.c_double * 8)()
    lib.llampc_debug_rl.argtypes = [ctypes.c_void_p]
    lib.llampc_debug_rl(RD)
    print("raceline window: need %.1f cap %.0f adv %.3f s0 %.3f L %.3f vmax %.3f" % tuple(RD[:6]))

if os.environ.get("RACELINE") and hasattr(lib, "llampc_debug_rl_ph"):
    PH = (ctypes.c_ulonglong * (1024 * 4))()
    lib.llampc_debug_rl_ph.argtypes = [ctypes.c_void_p]
    lib.llampc_debug_rl_ph(PH)
    P = np.frombuffer(PH, dtype=np.uint64).reshape(1024, 4).astype(np.int64)[:nla]
    st = Z[:, 0, 1]
    print("raceline prologue (us after block start, min/median/max): tables " + q((P[:, 0] - st) / 100.0)
          + ", window " + q((P[:, 1] - st) / 100.0) + ", walkers " + q((P[:, 2] - st) / 100.0)
          + ", fence " + q((P[:, 3] - st) / 100.0))
