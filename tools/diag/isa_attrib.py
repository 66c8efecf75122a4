"""Diagnostic (build-time): per-source-function accounting of the instructions in one rollout
step of the LPM-1 work-queue loop (plan_kernel<RK4, staged, LPM 1, ..., layout 2>), from a
hipcc -g -S listing: every instruction in the loop body is attributed to the source line of
its .loc (inlined code keeps its own file/line), lines to the enclosing function by the
nearest preceding definition.  usage: python tools/diag/isa_attrib.py [tu] [kernel-regex]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
tu = sys.argv[1] if len(sys.argv) > 1 else "plan_rk4_l1"
kre = sys.argv[2] if len(sys.argv) > 2 else r"^_ZN6llampc11plan_kernelILi0ELb1ELi1ELi0ELb0ELi2E\S+:"
tmp = tempfile.mkdtemp()
out = f"{tmp}/{tu}.s"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-g", "-std=c++17", "-mllvm",
                "-disable-machine-licm", f"-I{REPO}/include", f"-I{REPO}/lla-mpc_amd/csrc", "--cuda-device-only",
                "-S", f"{REPO}/lla-mpc_amd/csrc/{tu}.hip", "-o", out], cwd=tmp, check=True, stderr=subprocess.DEVNULL)
files, body, on = {}, [], False
with open(out) as f:
    for l in f:
        m = re.match(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = os.path.join(m.group(2), m.group(3))
            continue
        if re.match(kre, l):
            on = True
        if on:
            if "s_endpgm" in l:
                break
            if l.startswith(("\t.loc", "\t.", "\ts_", "\tv_", "\tds_", "\tglobal_", ".LBB")) or re.match(r"^\s+[sv]_|^\s+ds_|^\s+global_", l):
                body.append(l.rstrip("\n"))
labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
best = None
for i, l in enumerate(body):
    m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        seg = body[labels[m.group(1)]:i + 1]
        n = sum(1 for x in seg if re.match(r"^\s+(v_|s_)", x))
        if any("v_rcp_f64" in x for x in seg) and 200 < n < 2000 and (best is None or n < best[0]):
            best = (n, labels[m.group(1)], seg)
n, start, seg = best
# the .loc in force at the loop head: the last one before it
loc = None
for l in body[:start][::-1]:
    m = re.match(r"^\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = (int(m.group(1)), int(m.group(2)))
        break
src_cache = {}


def func_of(fi, line):
    path = files.get(fi, "?")
    if path not in src_cache:
        try:
            src_cache[path] = open(path).read().split("\n")
        except OSError:
            src_cache[path] = []
    src = src_cache[path]
    for j in range(min(line, len(src)) - 1, -1, -1):
        m = re.search(r"(?:__device__|__host__)[^;{]*?\b([A-Za-z_][\w:]*)\s*\(", src[j])
        if m and "return" not in src[j]:
            return f"{os.path.basename(path)}:{m.group(1)}"
    return f"{os.path.basename(path)}:?"


per_fn, per_line = collections.Counter(), collections.Counter()
fp64 = collections.Counter()
ours = lambda fi: "/lla-mpc_amd/" in files.get(fi, "")  # noqa: E731
for l in seg:
    m = re.match(r"^\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        # a .loc inside a system header (fma, fabs ... wrappers) keeps the caller's line
        if ours(int(m.group(1))) or loc is None:
            loc = (int(m.group(1)), int(m.group(2)))
        continue
    m = re.match(r"^\s+((?:v_|s_)\S+)", l)
    if not m:
        continue
    key = func_of(*loc) if loc else "?"
    per_fn[key] += 1
    per_line[(os.path.basename(files.get(loc[0], "?")), loc[1]) if loc else "?"] += 1
    if m.group(1).endswith("_f64") or "_f64_" in m.group(1):
        fp64[key] += 1
print(f"{tu}: {n} VALU+SALU instructions per step")
print(f"{'function':48s} {'instr':>6s} {'fp64':>5s}")
for k, v in per_fn.most_common():
    print(f"{k:48s} {v:6d} {fp64[k]:5d}")
print("\ntop source lines:")
for k, v in per_line.most_common(25):
    print(f"  {k}: {v}")
