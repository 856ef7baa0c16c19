#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc object (gfx950): python3 tools/isa_mix.py obj kernel_substr"""
import collections
import os
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj, pat = sys.argv[1], sys.argv[2]
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", f"--input={fat}", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    txt = subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], text=True)
blocks = txt.split("\n\n")
for b in blocks:
    head = b.strip().split("\n")[0]
    if pat in head:
        lines = [l.strip() for l in b.strip().split("\n")[1:] if l.strip() and not l.strip().startswith(";")]
        ops = collections.Counter(l.split()[0] for l in lines)
        print(head, len(lines))
        for k, v in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
            print(f"  {k:30s}{v}")
        if len(sys.argv) > 4:
            open(sys.argv[4], "w").write(b)
