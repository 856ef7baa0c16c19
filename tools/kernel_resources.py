#!/usr/bin/env python3
"""VGPR / SGPR / scratch / spill counts of the gfx950 kernels inside hipcc object files or the linked
libqcart.so: every clang offload bundle of the .hip_fatbin section (a linked library holds one per
translation unit) is split out and its code-object metadata notes are read with llvm-readelf.
python3 tools/kernel_resources.py <file.o | libqcart.so> ..."""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    """The gfx950 code objects (bytes) of every offload bundle in the file's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(d, "x")])
        data = open(fat, "rb").read()
    pos = data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                yield data[pos + off:pos + off + size]
        pos = data.find(MAGIC, pos + 1)


def kernels(path):
    """(name, vgpr_count, sgpr_count, private_segment_fixed_size, vgpr_spill_count, sgpr_spill_count) per kernel,
    as strings. sgpr_spill_count: SGPRs the allocator spilled (into VGPR lanes: v_writelane / v_readlane on the VALU,
    or to scratch when no lane is free)."""
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", f.name], text=True)
        for b in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
            m = re.search(r"\.name:\s+(\S+)", b)
            if not m:
                continue

            def g(k):
                mm = re.search(r"\." + k + r":\s+(\S+)", b)
                return mm.group(1) if mm else "?"
            yield (m.group(1), g("vgpr_count"), g("sgpr_count"), g("private_segment_fixed_size"), g("vgpr_spill_count"),
                   g("sgpr_spill_count"))


if __name__ == "__main__":
    for obj in sys.argv[1:]:
        for name, v, s, scr, sp, ssp in kernels(obj):
            print(f"{name:48s} vgpr={v:>4} sgpr={s:>4} scratch={scr:>6} vgpr_spill={sp} sgpr_spill={ssp}")
