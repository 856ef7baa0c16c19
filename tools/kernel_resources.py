#!/usr/bin/env python3
"""Print VGPR / SGPR / scratch / spill counts of the gfx950 kernels inside hipcc object files."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", f"--input={fat}", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
    for b in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
        m = re.search(r"\.name:\s+(\S+)", b)
        if not m:
            continue

        def g(k):
            mm = re.search(r"\." + k + r":\s+(\S+)", b)
            return mm.group(1) if mm else "?"
        yield m.group(1), g("vgpr_count"), g("sgpr_count"), g("private_segment_fixed_size"), g("vgpr_spill_count")


if __name__ == "__main__":
    for obj in sys.argv[1:]:
        for name, v, s, scr, sp in kernels(obj):
            print(f"{name:48s} vgpr={v:>4} sgpr={s:>4} scratch={scr:>6} vgpr_spill={sp}")
