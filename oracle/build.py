"""Build recipe for the oracle's C restatement (test infrastructure only).

Output: oracle/_build/liboracle_apr.so (git-ignored; ships to the GPU box with
the snapshot so tests and bench.py's cpu_baseline leg can load it there).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "apr_oracle.c")
LIB = os.path.join(HERE, "_build", "liboracle_apr.so")


def build(force: bool = False, verbose: bool = True) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(SRC) > os.path.getmtime(LIB):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        tmp = LIB + ".tmp"
        # -fopenmp: oracle_apr_train_mt (the threaded CPU baseline); the other
        # functions have no OpenMP pragmas and run on the calling thread
        cmd = ["gcc", "-O3", "-std=c11", "-ffp-contract=off", "-fopenmp", "-fPIC", "-shared", "-Wall", SRC, "-o",
               tmp, "-lm"]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build("--force" in sys.argv)
