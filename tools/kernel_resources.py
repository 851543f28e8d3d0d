#!/usr/bin/env python
"""Per-kernel register / LDS / scratch usage of the gfx950 code object inside a
built library (no GPU needed).

Extracts the clang offload bundle from the library's .hip_fatbin section, takes
the amdgcn code object and prints, for every kernel whose name matches the
pattern, the AMDGPU metadata fields .vgpr_count, .agpr_count, .sgpr_count,
.group_segment_fixed_size (LDS), .private_segment_fixed_size (scratch).

  python3 tools/kernel_resources.py adversarial-collaborative-filtering_amd/lib/libacf_apr.so k_stream
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib: str):
    data = open(lib, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(magic))[0]
        p = pos + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                yield data[pos + off:pos + off + size]
        pos = data.find(magic, pos + 1)


def main():
    lib, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
        out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], capture_output=True,
                             text=True).stdout
        os.unlink(f.name)
        for block in out.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", block)
            if not name or not pat.search(name.group(1)):
                continue
            fields = {k: re.search(rf"\.{k}:\s+(\S+)", block) for k in
                      ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
                       "private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count")}
            agpr = block.split("\n", 1)[0].strip(": ")
            dem = subprocess.run(["c++filt"], input=name.group(1), capture_output=True,
                                 text=True).stdout.strip()
            print(dem[:90], "agpr", agpr, " ".join(f"{k}={v.group(1)}" for k, v in fields.items() if v))


if __name__ == "__main__":
    main()
