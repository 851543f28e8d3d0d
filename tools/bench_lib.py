"""bench.py over another build of libacf_apr.so (same-box A/Bs of the headline
line): ACF_ALT_LIB=path loads that library in place of the package's, bypassing
the build-hash check (as tools/large_line.py does); every other argument goes to
bench.py unchanged.  Without ACF_ALT_LIB it is bench.py itself."""
import ctypes
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

alt = os.environ.get("ACF_ALT_LIB")
if alt:
    nat = importlib.import_module(bench.PKG + "._native")
    lib = ctypes.CDLL(alt)
    for fname, (res, args) in nat.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res, args
    nat._lib = lib
sys.argv = [bench.__file__] + sys.argv[1:]
bench.main()
