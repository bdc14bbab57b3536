#!/usr/bin/env python3
"""VGPRs, spilled VGPRs and scratch bytes per lane of every kernel of a built
libpsn_lk.so, from the gfx950 code objects' metadata (no GPU): the .hip_fatbin
section's offload bundles, each code object through llvm-readelf --notes.
Usage: tools/kernel_resources.py [lib] [kernel-regex]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x.so")],
                       check=True)
        data = open(fb, "rb").read()
    pos = 0
    while True:
        b = data.find(MAGIC, pos)
        if b < 0:
            return
        n = struct.unpack_from("<Q", data, b + 24)[0]
        p = b + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                yield data[b + off:b + off + size]
        pos = b + len(MAGIC)


def kernels(lib):
    out = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
        for blk in re.split(r"\n\s+- \.agpr_count", txt)[1:]:
            def g(k):
                m = re.search(r"\." + k + r":\s+(\S+)", blk)
                return m.group(1) if m else "?"
            out[g("name")] = {"vgpr": g("vgpr_count"), "vgpr_spill": g("vgpr_spill_count"),
                              "scratch": g("private_segment_fixed_size"), "lds": g("group_segment_fixed_size")}
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "mcmtt_opticalflow_amd/lib/libpsn_lk.so"
    rx = sys.argv[2] if len(sys.argv) > 2 else "lk_kernel"
    for n, r in sorted(kernels(lib).items()):
        if re.search(rx, n):
            print(f"{n:56s} vgpr {r['vgpr']:>4s} spill {r['vgpr_spill']:>3s} scratch {r['scratch']:>4s}")
