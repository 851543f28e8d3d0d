"""Build the in-tree HIP libraries with ``hipcc --offload-arch=gfx950``:
``lib/libacf_apr.so`` (APR path, C-ABI of ``include/acf_apr.h``) and
``lib/libacf_neumf.so`` (NeuMF path, ``include/acf_neumf.h``).  They land inside
the repository so that ``gpurun`` ships them to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
HIP_SRC = os.path.join(PKG_DIR, "csrc", "acf_apr.hip")
HIP_LIB = os.path.join(PKG_DIR, "lib", "libacf_apr.so")
HEADER = os.path.join(REPO, "include", "acf_apr.h")
NEUMF_SRC = os.path.join(PKG_DIR, "csrc", "acf_neumf.hip")
NEUMF_LIB = os.path.join(PKG_DIR, "lib", "libacf_neumf.so")
NEUMF_HEADER = os.path.join(REPO, "include", "acf_neumf.h")
TARGETS = [(HIP_SRC, HIP_LIB, [HEADER]), (NEUMF_SRC, NEUMF_LIB, [HEADER, NEUMF_HEADER])]

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-result",
]


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources if os.path.exists(s))


def build_hip(force: bool = False, verbose: bool = True) -> str:
    for src, lib, headers in TARGETS:
        if force or _stale(lib, [src, *headers, __file__]):
            os.makedirs(os.path.dirname(lib), exist_ok=True)
            hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
            tmp = lib + ".tmp"
            cmd = [hipcc, *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), src, "-o", tmp]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(tmp, lib)
    return HIP_LIB


def main(argv: list[str]) -> int:
    force = "--force" in argv
    build_hip(force)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
