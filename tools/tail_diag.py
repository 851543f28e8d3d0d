#!/usr/bin/env python
"""Where the end of a streamed call goes (r04 A/B aid): runs the driver-shaped
20-batch call with ACF_TAIL_DIAG=1 through the diagnostic library
(tools/libacf_apr_diag.so, tools/build_diag.sh: the tail stamps exist only in
-DACF_DIAG builds since r05) and prints k_stream's tail stamps (us after the
kernel's start), see acf_apr_diag_tail in csrc/acf_apr.hip."""
from __future__ import annotations

import ctypes
import json
import os
import statistics as st
import sys

os.environ["ACF_TAIL_DIAG"] = "1"
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import importlib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    acf = importlib.import_module("adversarial-collaborative-filtering_amd")
    ops = importlib.import_module("adversarial-collaborative-filtering_amd.ops")
    nat = importlib.import_module("adversarial-collaborative-filtering_amd._native")
    # the diagnostic library, without the product library's build-hash check
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libacf_apr_diag.so"))
    for fname, (res, args) in nat.SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.restype, fn.argtypes = res, args
    nat._lib = lib
    lib.acf_apr_diag_tail.restype = ctypes.c_int
    lib.acf_apr_diag_tail.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
    B, d, steps = 512, 64, 20
    ds = acf.ml1m_like(seed=2019)
    u, i, j = bench.make_triplets(acf, ds, B, 25 * steps, dev, seed=0)
    tabs = bench.init_tables(ds.num_users + 1, ds.num_items + 1, d, dev, seed=0)
    pipe = ops.PlanPipeline(ds.num_users + 1, ds.num_items + 1, d, B, steps, dev, overlap=None)
    hp = ops.StepHParams(lr=0.05, eps=0.5, reg=0.0, reg_adv=1.0, adver=1)
    rows = []
    out = (ctypes.c_uint64 * 8)()
    for r in range(20):
        pipe.run(tabs, hp, u, i, j, r * steps, steps)
        torch.cuda.synchronize()
        lib.acf_apr_diag_tail(pipe.ctx[0]._ptr, out, None)
        t0 = out[0]
        rows.append([(out[k] - t0) / 100.0 if out[k] else None for k in range(1, 7)])
    names = ["last_wg_done", "last_arrival", "decided", "actions", "flusher_saw", "flush_done"]
    med = {n: st.median([x[k] for x in rows[2:] if x[k] is not None]) for k, n in enumerate(names)
           if any(x[k] is not None for x in rows[2:])}
    print(json.dumps({
                      "us_after_start_median": med, "reps": rows[-3:]}))


if __name__ == "__main__":
    main()
