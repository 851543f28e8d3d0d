"""Where does an overlapped B = 512 APR step (k_ovl) spend its time?  (diagnostic)

Runs planned ml-1m-shaped batches through tools/libacf_apr_diag.so (-DACF_DIAG
stamps, s_memrealtime at 100 MHz) with step overlap on and prints, per k_ovl
launch (medians over launches), the times from the launch's first wave start to:
the end of the last adv(t) wave, the median clean(t+1) wave's wait end, the last
clean wave's end; plus how many clean waves waited and the clean header time.
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


def main():
    native = importlib.import_module(PKG + "._native")
    lib = native.load(os.path.join(REPO, "tools", "libacf_apr_diag.so"))
    lib.acf_diag_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda:0")
    B, d, nb = 512, 64, int(os.environ.get("NB", "64"))
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=0).epoch(0)
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    g = torch.Generator().manual_seed(0)
    tabs = [torch.nn.init.trunc_normal_(torch.empty(U1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.nn.init.trunc_normal_(torch.empty(I1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.full((U1, d), .1, device=dev), torch.full((I1, d), .1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    S = 3 * B
    SW, TW = S, (B + 3) // 4
    cap = 2 * S + TW + 64
    n_launch = nb + 2
    stamps = torch.zeros(n_launch * cap * 8, dtype=torch.int64, device=dev)
    hp = ops.StepHParams(adver=1)
    s = slice(0, nb * B)
    ctx.plan(ep.user[s], ep.item_pos[s], ep.item_neg[s], B)
    ctx.train_planned(tabs, hp)
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", stamps.data_ptr(), cap)
    ctx.train_planned(tabs, hp)
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", None, 0)
    st = stamps.view(n_launch, cap, 8).cpu().numpy().astype(np.int64)
    aw = SW + TW
    rows = []
    for li in range(1, nb):  # k_ovl launches with both halves
        w = st[li]
        started = w[:, 0] > 0
        t0 = w[started, 0].min()
        adv, cln = w[:aw], w[aw:aw + SW]
        adv_end = adv[adv[:, 4] > 0, 4]
        cl_end = cln[cln[:, 4] > 0, 4]
        waited = cln[cln[:, 5] > 0]
        hdr = (waited[:, 1] - waited[:, 0]) if len(waited) else np.zeros(1)
        wait = (waited[:, 5] - waited[:, 1]) if len(waited) else np.zeros(1)
        rows.append({
            "adv_last_end_us": (adv_end.max() - t0) / 100, "adv_p50_end_us": (np.median(adv_end) - t0) / 100,
            "clean_p50_wait_end_us": (np.median(waited[:, 5]) - t0) / 100 if len(waited) else 0,
            "clean_last_end_us": (cl_end.max() - t0) / 100 if len(cl_end) else 0,
            "clean_waves": int((cln[:, 0] > 0).sum()), "clean_full": int(len(cl_end)),
            "clean_hdr_p50_us": float(np.median(hdr)) / 100, "clean_wait_p50_us": float(np.median(wait)) / 100,
            "clean_wait_max_us": float(wait.max()) / 100,
            "span_us": (w[started][:, :6].max() - t0) / 100,
            "gap_to_next_us": (st[li + 1][st[li + 1][:, 0] > 0, 0].min() - w[started][:, :6].max()) / 100})
        full = adv[:SW][(adv[:SW, 4] > 0) & (adv[:SW, 2] > 0)]
        rows[-1].update({
            "adv_hdr_p50_us": float(np.median(full[:, 1] - full[:, 0])) / 100,
            "adv_loop_p50_us": float(np.median(full[:, 2] - full[:, 1])) / 100,
            "adv_store_p50_us": float(np.median(full[:, 4] - full[:, 2])) / 100,
            "adv_start_p90_us": float(np.percentile(adv[adv[:, 0] > 0, 0] - t0, 90)) / 100,
            "adv_start_max_us": float((adv[adv[:, 0] > 0, 0] - t0).max()) / 100,
            "clean_start_p50_us": float(np.median(cln[cln[:, 0] > 0, 0] - t0)) / 100,
            "fused_end_max_us": float((adv[SW:][adv[SW:, 4] > 0, 4] - t0).max()) / 100 if TW else 0.0})
        if li == 5:
            order = np.argsort(np.where(adv[:, 4] > 0, adv[:, 4], 0))[-8:][::-1]
            print("slowest adv waves of launch 5 (wave, start, hdr_end, loop_end, end) us:")
            for k in order:
                r = adv[k]
                print(int(k), *[round((x - t0) / 100, 2) if x > 0 else None for x in (r[0], r[1], r[2], r[4])])
    keys = rows[0].keys()
    summary = {k: float(np.median([r[k] for r in rows])) for k in keys}
    t_first = st[0][st[0][:, 0] > 0, 0].min()
    t_last = st[nb][st[nb][:, 0] > 0][:, :6].max()
    summary["per_batch_us"] = (t_last - t_first) / 100 / nb
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
