"""bench.py with another build of libacf_apr.so (A/B; diagnostic builds included),
bypassing the build-hash check: ACF_LARGE_LINE_LIB=path python3 tools/bench_alt.py [bench args]"""
import ctypes
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

alt = os.environ.get("ACF_LARGE_LINE_LIB")
if alt:
    nat = importlib.import_module(bench.PKG + "._native")
    lib = ctypes.CDLL(alt)
    for fname, (res, args) in nat.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res, args
    nat._lib = lib
sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
