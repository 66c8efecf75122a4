"""ISA statistics of the plan kernels (build-time diagnostic): instruction mix and the
largest loop body (the H-step rollout loop).  Usage: python tools/isa_stats.py [regex]"""
import os, re, subprocess, sys, tempfile
from collections import Counter
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else r"plan_kernelILi0ELb1ELi[124]E"
extra = sys.argv[2].split() if len(sys.argv) > 2 else []
tmp = tempfile.mkdtemp()
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                f"-I{REPO}/include", f"-I{REPO}/lla-mpc_amd/csrc", "-c",
                f"{REPO}/lla-mpc_amd/csrc/kernels.hip", "-save-temps", "-o", f"{tmp}/k.o"] + extra,
               cwd=tmp, check=True, stderr=subprocess.DEVNULL)
asm = open(f"{tmp}/kernels-hip-amdgcn-amd-amdhsa-gfx950.s").read().split("\n")
starts = [i for i, l in enumerate(asm) if re.match(r"^_Z\S+:", l)]
for si, s in enumerate(starts):
    name = asm[s].split(":")[0]
    if not re.search(pat, name):
        continue
    end = next(i for i in range(s, len(asm)) if "s_endpgm" in asm[i])
    body = asm[s:end + 1]
    ins = [l.split()[0] for l in body if re.match(r"^\s+[vs]_", l)]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    best = 0
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            n = sum(1 for x in body[labels[m.group(1)]:i + 1] if re.match(r"^\s+[vs]_", x))
            best = max(best, n)
    meta = "\n".join(asm[end:end + 400])
    vg = re.search(r"\.vgpr_count:\s+(\d+)", meta)
    c = Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name[:60]}: instrs {len(ins)} valu {valu} loop {best} readlane {c['v_readlane_b32']} "
          f"vmov64 {c['v_mov_b64_e32']} trig_preop {c['v_trig_preop_f64']} vgpr {vg.group(1) if vg else '?'}")
