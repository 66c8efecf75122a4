"""Instruction mix of the innermost loop(s) containing a marker instruction in one kernel
of a hipcc -S listing (diagnostic).  usage: isa_loop.py file.s kernel_substr marker"""
import collections
import os
import re
import sys

src, kname, marker = sys.argv[1], sys.argv[2], sys.argv[3]
s = open(src).read()
starts = [m.start() for m in re.finditer(r'^(_Z\S+):', s, re.M)]
for st in starts:
    name = s[st:s.index(':', st)]
    if kname not in name:
        continue
    end = s.index('.Lfunc_end', st)
    lines = s[st:end].split('\n')
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        m = re.match(r'\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            body = lines[labels[m.group(1)]:i + 1]
            if any(marker in b for b in body):
                loops.append((labels[m.group(1)], i, body))
    loops.sort(key=lambda t: t[1] - t[0])
    print(name[:90], 'loops with marker:', len(loops))
    dump = os.environ.get("ISA_DUMP")
    if dump and loops:
        open(dump, "w").write("\n".join(loops[0][2]))
    for lo, hi, body in loops[:3]:
        ins = [b.strip().split()[0] for b in body if b.startswith('\t') and not b.strip().startswith(('.', ';'))]
        c = collections.Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        salu = sum(v for k, v in c.items() if k.startswith('s_'))
        print(f'  lines {lo}-{hi}: {len(ins)} instrs, VALU {valu}, SALU {salu}')
        print('   ', ', '.join(f'{k} {v}' for k, v in c.most_common(28)))
