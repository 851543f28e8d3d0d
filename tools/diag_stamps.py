"""Where does a B = 512 APR step spend its time?  (diagnostic, not product)

Runs planned ml-1m-shaped batches through tools/libacf_apr_diag.so (built with
-DACF_DIAG: per-wave s_memrealtime stamps at 100 MHz) and prints, per kernel
kind, the launch span, the gap to the next launch and the per-wave segment
times.  Stamps cost time themselves: read the shares, not the totals.
"""
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
    native = importlib.import_module(PKG + "._native")
    lib = native.load(os.path.join(REPO, "tools", "libacf_apr_diag.so"))
    import ctypes
    lib.acf_diag_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda:0")
    B, d, nb = 512, 64, int(os.environ.get("NB", "64"))
    graph = os.environ.get("GRAPH", "1") == "1"
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=0).epoch(0)
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    g = torch.Generator().manual_seed(0)
    tabs = [torch.nn.init.trunc_normal_(torch.empty(U1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.nn.init.trunc_normal_(torch.empty(I1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.full((U1, d), .1, device=dev), torch.full((I1, d), .1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    S = 3 * B
    cap = 2 * S
    n_launch = 2 * nb + 1
    stamps = torch.zeros(n_launch * cap * 8, dtype=torch.int64, device=dev)
    hp = ops.StepHParams(adver=int(os.environ.get("ADVER", "1")))
    s = slice(0, nb * B)
    ctx.plan(ep.user[s], ep.item_pos[s], ep.item_neg[s], B)
    ctx.train_planned(tabs, hp, graph=graph)  # warm / capture
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", stamps.data_ptr(), cap)
    ctx.train_planned(tabs, hp, graph=graph)
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", None, 0)
    st = stamps.view(n_launch, cap, 8).cpu().numpy().astype(np.int64)
    out = {"graph": graph, "nb": nb, "launches": []}
    rows = []
    for li in range(n_launch):
        w = st[li]
        started = w[:, 0] > 0
        if not started.any():
            continue
        t0 = w[started, 0].min()
        tend = w[started][:, :6].max()
        last = np.where(w[:, 4] > 0, w[:, 4], np.where(w[:, 5] > 0, w[:, 5], w[:, 1]))
        full = (w[:, 4] > 0)
        seg = {}
        if full.any():
            f = w[full]
            seg = {"hdr": float(np.median(f[:, 1] - f[:, 0])) * 10,
                   "gather_compute": float(np.median(f[:, 2] - f[:, 1])) * 10,
                   "reduce_delta": float(np.median(np.where(f[:, 3] > 0, f[:, 3], f[:, 2]) - f[:, 2])) * 10,
                   "store": float(np.median(f[:, 4] - np.where(f[:, 3] > 0, f[:, 3], f[:, 2]))) * 10,
                   "wave_max_ns": float((f[:, 4] - f[:, 0]).max()) * 10}
        rows.append((li, int(t0), int(tend), int(started.sum()), int(full.sum()),
                     float(w[started, 0].max() - t0) * 10, seg, last))
    for x, (li, t0, tend, ns, nf, spread, seg, _) in enumerate(rows):
        gap = (rows[x + 1][1] - tend) * 10 if x + 1 < len(rows) else None
        out["launches"].append({"launch": li, "span_ns": float(tend - t0) * 10, "gap_to_next_ns": gap,
                                "waves_started": ns, "full_waves": nf, "start_spread_ns": spread,
                                "seg_median_ns": seg})
    spans = [r["span_ns"] for r in out["launches"]]
    gaps = [r["gap_to_next_ns"] for r in out["launches"] if r["gap_to_next_ns"] is not None]
    total = (rows[-1][2] - rows[0][1]) * 10
    summary = {"per_batch_us": total / nb / 1e3,
               "span_even_us": float(np.median(spans[0:-1:2])) / 1e3,
               "span_odd_us": float(np.median(spans[1:-1:2])) / 1e3,
               "gap_median_us": float(np.median(gaps)) / 1e3,
               "start_spread_even_us": float(np.median([r["start_spread_ns"] for r in out["launches"][0:-1:2]])) / 1e3,
               "start_spread_odd_us": float(np.median([r["start_spread_ns"] for r in out["launches"][1:-1:2]])) / 1e3}
    for key in ("hdr", "gather_compute", "reduce_delta", "store", "wave_max_ns"):
        for par, name in ((0, "even"), (1, "odd")):
            v = [r["seg_median_ns"].get(key) for r in out["launches"][par:-1:2] if r["seg_median_ns"]]
            if v:
                summary[f"{key}_{name}_ns"] = float(np.median(v))
    # shader clock during phase-1 waves: d(s_memtime) / d(s_memrealtime) * 100 MHz
    clk = []
    for li in range(0, n_launch - 1, 2):
        w = st[li]
        ok = (w[:, 4] > 0) & (w[:, 7] > w[:, 6])
        if ok.any():
            clk.append(np.median((w[ok, 7] - w[ok, 6]) / np.maximum(w[ok, 4] - w[ok, 0], 1)) * 100.0)
    if clk:
        summary["shader_clock_MHz_median"] = float(np.median(clk))
    # tail: the longest waves of each kind and the occurrence counts of their slots
    u0 = ep.user[:B].cpu().numpy()
    it0 = np.concatenate([ep.item_pos[:B].cpu().numpy(), ep.item_neg[:B].cpu().numpy()])
    cu = np.unique(u0, return_counts=True)[1]
    ci = np.unique(it0, return_counts=True)[1]
    counts = np.concatenate([cu, ci])
    for par, name in ((0, "clean"), (1, "adv")):
        durs, tops = [], []
        for li in range(par, n_launch - 1, 2):
            w = st[li]
            full = w[:, 4] > 0
            dd = np.where(full, w[:, 4] - w[:, 0], 0) * 10
            durs.append(dd[full])
            if li < 2:  # batch 0: slot counts known
                top = np.argsort(dd)[-5:][::-1]
                tops = [(int(k), float(dd[k]), int(counts[k]) if k < len(counts) else -1) for k in top]
        allv = np.concatenate(durs) if durs else np.zeros(1)
        summary[f"wave_ns_{name}"] = {q: float(np.percentile(allv, p)) for q, p in
                                      (("p50", 50), ("p90", 90), ("p99", 99), ("max", 100))}
        summary[f"longest_waves_batch0_{name}"] = tops
    summary["max_slot_count_batch0"] = int(counts.max())
    print(json.dumps(summary, indent=1))
    with open(os.path.join(REPO, "gpurun_out", f"diag_g{int(graph)}_a{hp.adver}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
