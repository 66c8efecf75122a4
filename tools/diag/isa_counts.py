"""Diagnostic (build-time): VALU+SALU instructions per H-step of the fast look-ahead rollout
loop for each lane split (LPM 1/2/4) of plan_kernel<RK4, staged, LPM, xref shared>, from a
hipcc -S listing.  bench.py's ISSUE_INSTR_PER_STEP holds these numbers.
usage: python tools/diag/isa_counts.py"""
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tmp = tempfile.mkdtemp()
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm",
                "-disable-machine-licm", f"-I{REPO}/include", f"-I{REPO}/lla-mpc_amd/csrc", "-c",
                f"{REPO}/lla-mpc_amd/csrc/kernels.hip", "-save-temps", "-o", f"{tmp}/k.o"],
               cwd=tmp, check=True, stderr=subprocess.DEVNULL)
asm = open(f"{tmp}/kernels-hip-amdgcn-amd-amdhsa-gfx950.s").read().split("\n")
# (lpm, work-queue layout): the headline C = 1 kernel is LPM 4; C >= 64 runs LPM 1 in the
# work-queue layout (last template flag WQ = 1)
for lpm, wq in ((4, 0), (2, 0), (1, 0), (1, 1)):
    s = next(i for i, l in enumerate(asm) if re.match(rf"^_ZN6llampc11plan_kernelILi0ELb1ELi{lpm}ELi0ELb0ELb{wq}E\S+:", l))
    e = next(i for i in range(s, len(asm)) if "s_endpgm" in asm[i])
    body = asm[s:e]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            n = sum(1 for x in seg if re.match(r"^\s+(v_|s_)", x))
            if any("v_rcp_f64" in x for x in seg) and 200 < n < 1500 and (best is None or n < best):
                best = n
    print(f"LPM {lpm}{' work queue' if wq else ''}: {best} instructions per rollout step")
