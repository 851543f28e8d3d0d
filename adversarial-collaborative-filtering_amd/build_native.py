"""Build the in-tree native libraries.

- ``lib/libacf_apr.so``: the HIP kernels + C-ABI (``include/acf_apr.h``), built
  with ``hipcc --offload-arch=gfx950``.  This is the product.
- ``oracle/_build/liboracle_apr.so``: the CPU restatement used only by tests and
  by ``bench.py``'s ``cpu_baseline`` leg (built with gcc).

Both land inside the repository so that ``gpurun`` ships them to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
HIP_SRC = os.path.join(PKG_DIR, "csrc", "acf_apr.hip")
HIP_LIB = os.path.join(PKG_DIR, "lib", "libacf_apr.so")
ORACLE_SRC = os.path.join(REPO, "oracle", "apr_oracle.c")
ORACLE_LIB = os.path.join(REPO, "oracle", "_build", "liboracle_apr.so")
HEADER = os.path.join(REPO, "include", "acf_apr.h")

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
    if force or _stale(HIP_LIB, [HIP_SRC, HEADER, __file__]):
        os.makedirs(os.path.dirname(HIP_LIB), exist_ok=True)
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        tmp = HIP_LIB + ".tmp"
        cmd = [hipcc, *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), HIP_SRC, "-o", tmp]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_oracle(force: bool = False, verbose: bool = True) -> str:
    if force or _stale(ORACLE_LIB, [ORACLE_SRC, __file__]):
        os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
        tmp = ORACLE_LIB + ".tmp"
        cmd = ["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fPIC", "-shared",
               "-Wall", ORACLE_SRC, "-o", tmp, "-lm"]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def main(argv: list[str]) -> int:
    force = "--force" in argv
    build_hip(force)
    if os.path.exists(ORACLE_SRC):
        build_oracle(force)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
