"""Diagnostic (build-time): VALU+SALU instructions per H-step of the fast look-ahead rollout
loop for each lane split (LPM 1/2/4) of plan_kernel<RK4, staged, LPM, xref shared> and of the
controller tick's ctl_kernel<LPM> (candidates in LDS, input terms staged: the shortest loop), from hipcc -S listings of the
translation units that hold them.  bench.py's ISSUE_INSTR_PER_STEP holds the plan numbers.
usage: python tools/diag/isa_counts.py [extra hipcc flags, e.g. -DLLAMPC_LEAN_TERMS=7]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tmp = tempfile.mkdtemp()


def listing(tu):
    out = f"{tmp}/{tu}.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm",
                    "-disable-machine-licm", *sys.argv[1:], f"-I{REPO}/include", f"-I{REPO}/lla-mpc_amd/csrc", "--cuda-device-only",
                    "-S", f"{REPO}/lla-mpc_amd/csrc/{tu}.hip", "-o", out], cwd=tmp, check=True, stderr=subprocess.DEVNULL)
    return open(out).read().split("\n")


def loop_of(asm, pattern, fmin=150, rcp=1):
    s = next(i for i, l in enumerate(asm) if re.match(pattern, l))
    e = next(i for i in range(s, len(asm)) if "s_endpgm" in asm[i])
    body = asm[s:e]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            n = sum(1 for x in seg if re.match(r"^\s+(v_|s_)", x))
            f = sum(1 for x in seg if re.match(r"^\s+v_\w+_f64", x))
            # the rollout step: the innermost loop with the division and most fp64 work
            if sum("v_rcp_f64" in x for x in seg) >= rcp and 200 < n < 2000 and f > fmin and (best is None or n < best[0]):
                best = (n, seg)
    return best


def report(name, best):
    if best is None:
        print(f"{name}: no rollout loop found")
        return
    n, seg = best
    ops = collections.Counter(re.match(r"^\s+(\S+)", x).group(1) for x in seg if re.match(r"^\s+(v_|s_|ds_|global_|flat_|buffer_|scratch_)", x))
    fp64 = sum(v for k, v in ops.items() if k.endswith("_f64"))
    spill = sum(v for k, v in ops.items() if k.startswith(("v_readlane", "v_writelane", "scratch_")))
    mem = sum(v for k, v in ops.items() if k.startswith(("ds_", "global_", "flat_", "buffer_")))
    print(f"{name}: {n} VALU+SALU per step (fp64 {fp64}, lane moves/spill {spill}, memory {mem})")


asm4 = listing("plan_rk4_l4")
report("plan LPM 4 (staged)", loop_of(asm4, r"^_ZN6llampc11plan_kernelILi0ELb1ELi4ELi0ELb0ELi0E\S+:"))
asm2 = listing("plan_rk4_l2")
report("plan LPM 2 (staged)", loop_of(asm2, r"^_ZN6llampc11plan_kernelILi0ELb1ELi2ELi0ELb0ELi0E\S+:"))
asm1 = listing("plan_rk4_l1")
report("plan LPM 1 (staged)", loop_of(asm1, r"^_ZN6llampc11plan_kernelILi0ELb1ELi1ELi0ELb0ELi0E\S+:"))
report("plan LPM 1 (work queue, 8 waves)", loop_of(asm1, r"^_ZN6llampc11plan_kernelILi0ELb1ELi1ELi0ELb0ELi2E\S+:"))
asmc = listing("ctl")
for lpm in (4, 2, 1):
    # a whole RK4 step: 4 stages x 2 chains' divisions (the look-back's and the walker's loops
    # divide too)
    report(f"ctl LPM {lpm} (staged inputs)", loop_of(asmc, rf"^_ZN6llampc10ctl_kernelILi{lpm}ELb0EEEvNS_9CtlLaunchE:", 300, 8))
