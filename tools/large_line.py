"""configs[4] line(s) alone (bench.large_batch_roofline) for same-box A/B runs:
python3 tools/large_line.py [d[:eager] ...] -> one JSON line per entry
(eager: chunks launched without hipGraph).  ACF_LARGE_LINE_LIB=path loads another
build of libacf_apr.so (an older commit's, tools/build_at.sh) in place of the
package's, bypassing the build-hash check (tools/gpu_ab_large.sh)."""
import ctypes
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

acf = importlib.import_module(bench.PKG)
ops = importlib.import_module(bench.PKG + ".ops")
alt = os.environ.get("ACF_LARGE_LINE_LIB")
if alt:
    nat = importlib.import_module(bench.PKG + "._native")
    lib = ctypes.CDLL(alt)
    for fname, (res, args) in nat.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res, args
    nat._lib = lib
dev = torch.device("cuda", 0)
big = acf.synthetic_large(device=dev)
for arg in sys.argv[1:] or ["64"]:
    parts = arg.split(":")
    d, graph = int(parts[0]), "eager" not in parts[1:]
    r = bench.large_batch_roofline(acf, ops, dev, big, d, graph=graph)
    print(json.dumps({"d": d, "graph": graph, "lib": alt or "package",
                      "triplets_per_s": r["triplets_per_s"], "step_frac": r["step_bandwidth"]["frac"],
                      "avg_launch_us": r.get("avg_launch_us"), "per_kernel_avg_us": r.get("per_kernel_avg_us"),
                      "alone_per_kernel_avg_us": r["alone"]["per_kernel_avg_us"],
                      "step_errors": r["step_errors"]}), flush=True)
