#!/usr/bin/env python3
"""Find the largest loop (backward branch) in a disassembled kernel (isa_mix.py dump) and print its
instruction mix: python3 tools/isa_loop.py dump.s [top]"""
import collections
import re
import sys

lines = [l for l in open(sys.argv[1]).read().split("\n")[1:] if l.strip()]
addr, ins = [], []
for l in lines:
    m = re.search(r"//\s*([0-9A-Fa-f]+):", l)
    if not m:
        continue
    addr.append(int(m.group(1), 16))
    ins.append(l.split("//")[0].strip())
base = addr[0]
best = None
for i, s in enumerate(ins):
    m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", lines[i]) if False else None
for i, l in enumerate(lines):
    pass
# branch targets are printed as <sym+0xOFF>
full = [l for l in lines if re.search(r"//\s*[0-9A-Fa-f]+:", l)]
for i, l in enumerate(full):
    if "branch" in ins[i]:
        m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
        if m:
            tgt = base + int(m.group(1), 16)
            if tgt < addr[i]:
                j = addr.index(tgt) if tgt in addr else None
                if j is not None and (best is None or i - j > best[1] - best[0]):
                    best = (j, i)
j, i = best
body = ins[j:i + 1]
print(f"loop: {i - j + 1} instructions")
c = collections.Counter(s.split()[0] for s in body)
for k, v in c.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
    print(f"  {k:30s}{v}")
open("/tmp/loop_body.s", "w").write("\n".join(body))
