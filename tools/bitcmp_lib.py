"""Bit-compare two builds of libacf_apr.so on one large-batch case (B = 65,536,
Zipf positives, hot slots): prints one JSON line with the sha256 of P, Q, accP,
accQ and the losses after two APR batches.  ACF_ALT_LIB=path loads that build
in place of the package's (as tools/bench_lib.py).  Run it once per build and
compare the digests (tools/gpu_r06_ab.sh BITCMP=1).
usage: python3 tools/bitcmp_lib.py [d ...]"""
import ctypes
import hashlib
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ops = importlib.import_module(bench.PKG + ".ops")
alt = os.environ.get("ACF_ALT_LIB")
if alt:
    nat = importlib.import_module(bench.PKG + "._native")
    lib = ctypes.CDLL(alt)
    for fname, (res, args) in nat.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res, args
    nat._lib = lib
dev = torch.device("cuda", 0)
U1, I1, B, nb = 300_000, 200_000, 65536, 2
for d in [int(x) for x in sys.argv[1:]] or [64, 128]:
    rng = np.random.default_rng(d + 1)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = ((rng.zipf(1.1, nb * B) - 1) % I1).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    tabs = [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.time_kernels(tabs, ops.StepHParams(adver=1))
    torch.cuda.synchronize()
    lc, la = ctx.losses()
    h = hashlib.sha256()
    for t in tabs + [lc, la]:
        h.update(t.cpu().numpy().tobytes())
    print(json.dumps({"d": d, "lib": alt or "package", "plan_kind": ctx.plan_kind(),
                      "sha256": h.hexdigest(), "step_errors": ctx.step_errors()}), flush=True)
