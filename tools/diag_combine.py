"""Where does a configs[4] batch spend its time inside the triplet-centric
launches?  (diagnostic, not product)

Runs NB planned batches of the configs[4] shape (10M x 5M Zipf, alias
negatives, B = 65,536, d from argv) eagerly through tools/libacf_apr_diag.so
(tools/build_diag.sh: -DACF_DIAG, per-wave s_memrealtime stamps at 100 MHz) and
prints, per launch, its span and the end times of each wave role relative to
the launch's first wave start (k_tri_combine: piece waves, combining
workgroups after their first wait and at their end, small-slot waves;
k_tri_clean / k_tri_adv: triplet waves).  Stamps cost time themselves: read the
shares, not the totals.  Usage: python3 tools/diag_combine.py [d]
"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "adversarial-collaborative-filtering_amd"


def pct(x):
    if len(x) == 0:
        return None
    return [round(float(np.percentile(x, q)) * 10 / 1e3, 2) for q in (10, 50, 90, 100)]  # us


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    nb = int(os.environ.get("NB", "4"))
    nat = importlib.import_module(PKG + "._native")
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libacf_apr_diag.so"))
    for fname, (res, args) in nat.SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.restype, fn.argtypes = res, args
    nat._lib = lib
    lib.acf_diag_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda", 0)
    ds = acf.synthetic_large(device=dev)
    U1, I1, B = ds.num_users + 1, ds.num_items + 1, 65536
    ep = acf.DeviceSampler(ds, B, dev, seed=7, weights=np.ones(ds.num_items, np.float32)).epoch(0)
    u, i, j = (x[: 2 * nb * B].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
    del ep
    g = torch.Generator(device=dev).manual_seed(5)
    tabs = [torch.randn(U1, d, device=dev, generator=g) * 0.01, torch.randn(I1, d, device=dev, generator=g) * 0.01,
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    hp = ops.StepHParams(adver=1)
    cap = 12288
    n_launch = 4 * nb + 2
    stamps = torch.zeros(n_launch * cap * 8, dtype=torch.int64, device=dev)
    s0, s1 = slice(0, nb * B), slice(nb * B, 2 * nb * B)
    ctx.plan(u[s0], i[s0], j[s0], B)
    ctx.train_planned(tabs, hp, graph=False)  # warm
    ctx.plan(u[s1], i[s1], j[s1], B)
    torch.cuda.synchronize()
    lib.acf_diag_set_stamps(ctypes.c_void_p(stamps.data_ptr()), cap)
    ctx.train_planned(tabs, hp, graph=False)
    torch.cuda.synchronize()
    lib.acf_diag_set_stamps(None, 0)
    st = stamps.view(n_launch, cap, 8).cpu().numpy().astype(np.int64)
    out = {"d": d, "nb": nb, "launches": []}
    prev_end = None
    for li in range(n_launch):
        w = st[li]
        started = w[:, 0] > 0
        if not started.any():
            continue
        t0 = w[started, 0].min()
        ends = w[:, 1:6].max(axis=1)
        tend = ends[started].max()
        rec = {"launch": li, "waves": int(started.sum()), "span_us": round(float(tend - t0) * 10 / 1e3, 2),
               "gap_from_prev_us": None if prev_end is None else round(float(t0 - prev_end) * 10 / 1e3, 2),
               "start_spread_us": round(float(w[started, 0].max() - t0) * 10 / 1e3, 2)}
        roles = {"piece_end": 1, "combiner_waited": 2, "combiner_end": 3, "slot_end": 4, "triplet_end": 5}
        for name, k in roles.items():
            m = w[:, k] > 0
            if m.any():
                rec[name + "_us_p10_p50_p90_max"] = pct(w[m, k] - t0)
                rec[name + "_waves"] = int(m.sum())
        m = w[:, 2] > 0
        if m.any():
            rec["combiner_start_us_p50_max"] = pct(w[m, 0] - t0)[1::2]
        out["launches"].append(rec)
        prev_end = tend
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
