"""The split-step bench lines alone (world 1), for rocprofv3 --kernel-trace --stats:
   rocprofv3 --kernel-trace --stats -d gpurun_out/prof_shard -- python3 tools/shard_profile.py"""
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
acf = importlib.import_module(bench.PKG)
ops = importlib.import_module(bench.PKG + ".ops")
alt = os.environ.get("ACF_LARGE_LINE_LIB")  # another build of libacf_apr.so (A/B; see tools/large_line.py)
if alt:
    import ctypes
    nat = importlib.import_module(bench.PKG + "._native")
    lib = ctypes.CDLL(alt)
    for fname, (res, args) in nat.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res, args
    nat._lib = lib
if "--per-step-plans" in sys.argv:  # A/B: r05's one-batch plan beside every step
    sys.argv.remove("--per-step-plans")
    importlib.import_module(bench.PKG + ".distributed").HipLocal.chunk_planned = False
if "--chunk-min" in sys.argv:  # A/B: chunk plans from this local batch size up
    k = sys.argv.index("--chunk-min")
    importlib.import_module(bench.PKG + ".distributed").HipLocal.chunk_min = int(sys.argv[k + 1])
    del sys.argv[k:k + 2]
big = acf.synthetic_large(device=dev)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
print(json.dumps(bench.sharded_lines(acf, ops, dev, None, 1, 0, big, steps)))
