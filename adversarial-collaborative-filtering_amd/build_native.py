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
OPS_SRC = os.path.join(PKG_DIR, "csrc", "acf_ops.hip")
ROWS_H = os.path.join(PKG_DIR, "csrc", "acf_rows.h")
HIP_LIB = os.path.join(PKG_DIR, "lib", "libacf_apr.so")
HEADER = os.path.join(REPO, "include", "acf_apr.h")
NEUMF_SRC = os.path.join(PKG_DIR, "csrc", "acf_neumf.hip")
NEUMF_LIB = os.path.join(PKG_DIR, "lib", "libacf_neumf.so")
NEUMF_HEADER = os.path.join(REPO, "include", "acf_neumf.h")
# (sources, library, headers it depends on)
TARGETS = [([HIP_SRC, OPS_SRC], HIP_LIB, [HEADER, ROWS_H]), ([NEUMF_SRC], NEUMF_LIB, [HEADER, NEUMF_HEADER])]

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
    for srcs, lib, headers in TARGETS:
        if force or _stale(lib, [*srcs, *headers, __file__]):
            os.makedirs(os.path.dirname(lib), exist_ok=True)
            hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
            tmp = lib + ".tmp"
            cmd = [hipcc, *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), *srcs, "-o", tmp]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(tmp, lib)
    return HIP_LIB


TORCH_SRC = os.path.join(PKG_DIR, "csrc", "acf_torch.cpp")
TORCH_LIB = os.path.join(PKG_DIR, "lib", "libacf_torch.so")


def build_torch_ops(force: bool = False, verbose: bool = True) -> str:
    """lib/libacf_torch.so: the TORCH_LIBRARY(acf, m) custom ops over libacf_apr.so
    (host code only: g++ against the installed torch's headers and libraries)."""
    import torch

    if not (force or _stale(TORCH_LIB, [TORCH_SRC, HEADER, HIP_LIB, __file__])):
        return TORCH_LIB
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = TORCH_LIB + ".tmp"
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-I", os.path.join(tdir, "include"), "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           "-I", "/opt/rocm/include", "-I", os.path.join(REPO, "include"), TORCH_SRC, "-o", tmp,
           "-L", os.path.join(tdir, "lib"), "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip",
           "-L", os.path.dirname(HIP_LIB), "-lacf_apr", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, TORCH_LIB)
    return TORCH_LIB


def main(argv: list[str]) -> int:
    force = "--force" in argv
    build_hip(force)
    build_torch_ops(force)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
