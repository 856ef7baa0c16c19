#!/usr/bin/env python3
"""Disassemble one kernel of a hipcc object (gfx950) to stdout: python3 tools/isa_dump.py obj kernel_substr
(feed the output to tools/isa_loop.py for the step loop's instruction mix)."""
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
for b in txt.split("\n\n"):
    if pat in b.strip().split("\n")[0]:
        print(b)
        break
