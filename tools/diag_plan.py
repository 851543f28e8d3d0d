"""Where does the batch-local plan of a short call spend its time?  (diagnostic)

Plans --nb ml-1m-shaped batches of 512 through tools/libacf_apr_diag.so
(-DACF_DIAG, tools/build_diag.sh) with s_memrealtime stamps (100 MHz) at the
phase boundaries of k_bplan_sort (slots [batch][wave]) and k_bplan_build
(slots [batch][16 + wave]) and prints median phase times per workgroup plus the
kernels' spans.  Stamps cost time themselves: read shares, not totals.
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "adversarial-collaborative-filtering_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lib", default=os.path.join(REPO, "tools", "libacf_apr_diag.so"))
    a = ap.parse_args()
    native = importlib.import_module(PKG + "._native")
    import ctypes
    lib = ctypes.CDLL(a.lib)  # a -DACF_DIAG build: no build-hash check (as tools/bench_lib.py)
    for fname, (res_t, args) in native.SIGNATURES.items():
        if hasattr(lib, fname):
            fn = getattr(lib, fname)
            fn.restype, fn.argtypes = res_t, args
    native._lib = lib
    lib.acf_diag_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda:0")
    B, nb, cap = 512, a.nb, 32
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=0).epoch(0)
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    ctx = ops.APRContext(U1, I1, 64, B, nb, dev)
    stamps = torch.zeros(nb * cap * 8, dtype=torch.int64, device=dev)
    res = []
    for r in range(a.reps + 1):
        s = slice(r * nb * B, (r + 1) * nb * B)
        stamps.zero_()
        native.call("acf_diag_set_stamps", stamps.data_ptr(), cap)
        ctx.plan(ep.user[s], ep.item_pos[s], ep.item_neg[s], B)
        torch.cuda.synchronize()
        native.call("acf_diag_set_stamps", None, 0)
        if r:
            res.append(stamps.view(nb, cap, 8).cpu().numpy().astype(np.int64))
    out = {}
    sort_ph = ["load", "sort", "unique_scan", "writes"]
    build_ph = ["slot_loads", "mask", "slot_of", "info", "records", "task_list", "clear"]
    acc = {k: [] for k in ["sort_" + x for x in sort_ph] + ["build_" + x for x in build_ph] +
           ["sort_span", "build_span", "gap_sort_end_build_start", "sort_first_start_to_build_last_end"]}
    for st in res:
        so = st[:, :8, :5]  # [nb][waves][phase]
        bo = st[:, 16:32, :7]
        b7 = st[:, 16:32, 7]
        live_s = so[:, :, 0] > 0
        live_b = bo[:, :, 0] > 0
        for t in range(nb):
            ws, wb = so[t][live_s[t]], bo[t][live_b[t]]
            for k in range(4):
                acc["sort_" + sort_ph[k]].append(ws[:, k + 1].max() - ws[:, k].max())
            for k in range(6):
                acc["build_" + build_ph[k]].append(wb[:, k + 1].max() - wb[:, k].max())
            w7 = b7[t][live_b[t]]
            if (w7 > 0).all():  # optional stamp 7: after the first task-list scan
                acc.setdefault("build_task_list_first_scan", []).append(w7.max() - wb[:, 4].max())
        s0, s1 = so[:, :, 0][live_s].min(), so[:, :, 4][live_s].max()
        b0, b1 = bo[:, :, 0][live_b].min(), bo[:, :, 6][live_b].max()
        acc["sort_span"].append(s1 - s0)
        acc["build_span"].append(b1 - b0)
        acc["gap_sort_end_build_start"].append(b0 - s1)
        acc["sort_first_start_to_build_last_end"].append(b1 - s0)
    for k, v in acc.items():
        out[k] = round(float(np.median(v)) / 100, 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
