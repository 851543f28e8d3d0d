"""Where does a streamed APR chunk (k_stream) spend its time?  (diagnostic)

Runs ml-1m-shaped batches through tools/libacf_apr_diag.so (-DACF_DIAG stamps,
s_memrealtime at 100 MHz; stamp 'launch' = batch, 'wave' = task) and prints
medians of the per-task segments of slot tasks:
  hdr    start -> slot header loaded
  wait1  header -> own row, Adagrad slot and partner rows all there
  clean  -> delta published
  adv    -> partner deltas there + adversarial terms (one-pass slots split into
           adv_solo: solo deltas formed, adv_wait: published deltas there,
           adv_terms: adversarial terms)
  tail   -> Adagrad + versions stored
plus the time between consecutive batches' completions (per-batch rate) and the
start lag of a batch's tasks behind the previous batch's completion.
Stamps cost time themselves: read shares, not totals.
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
    B, d, nb = 512, 64, int(os.environ.get("NB", "200"))
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=0).epoch(0)
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    g = torch.Generator().manual_seed(0)
    tabs = [torch.nn.init.trunc_normal_(torch.empty(U1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.nn.init.trunc_normal_(torch.empty(I1, d), 0, .01, -.02, .02, generator=g).to(dev),
            torch.full((U1, d), .1, device=dev), torch.full((I1, d), .1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    S = 3 * B
    cap = S + (B + 3) // 4
    stamps = torch.zeros(nb * cap * 8, dtype=torch.int64, device=dev)
    hp = ops.StepHParams(adver=1)
    s = slice(0, nb * B)
    ctx.plan(ep.user[s], ep.item_pos[s], ep.item_neg[s], B)
    ctx.train_planned(tabs, hp, graph=False)
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", stamps.data_ptr(), cap)
    ctx.train_planned(tabs, hp, graph=False)
    torch.cuda.synchronize()
    native.call("acf_diag_set_stamps", None, 0)
    assert ctx.step_errors() == 0
    st = stamps.view(nb, cap, 8).cpu().numpy().astype(np.int64)
    t0 = st[st[:, :, 0] > 0, 0].min()
    seg = {k: [] for k in ("hdr", "wait1", "clean", "adv", "tail", "task", "adv_solo", "adv_wait", "adv_terms")}
    done, first_start, lag = [], [], []
    for t in range(nb):
        w = st[t]
        full = w[:S][(w[:S, 5] > 0) & (w[:S, 1] > 0)]
        seg["hdr"] += list(full[:, 1] - full[:, 0])
        seg["wait1"] += list(full[:, 2] - full[:, 1])
        seg["clean"] += list(full[:, 3] - full[:, 2])
        seg["adv"] += list(full[:, 4] - full[:, 3])
        seg["tail"] += list(full[:, 5] - full[:, 4])
        seg["task"] += list(full[:, 5] - full[:, 0])
        one = full[(full[:, 6] > 0) & (full[:, 7] > 0)]  # one-pass slots: adv split at stamps 6, 7
        seg["adv_solo"] += list(one[:, 6] - one[:, 3])
        seg["adv_wait"] += list(one[:, 7] - one[:, 6])
        seg["adv_terms"] += list(one[:, 4] - one[:, 7])
        ends = w[w[:, 5] > 0, 5]
        starts = w[w[:, 0] > 0, 0]
        done.append(ends.max())
        first_start.append(starts.min())
        if t > 0:
            lag.append(np.median(starts) - done[t - 1])
    done = np.array(done, dtype=np.float64)
    out = {k: round(float(np.median(v)) / 100, 3) for k, v in seg.items()}
    out.update({k + "_p90": round(float(np.percentile(v, 90)) / 100, 3) for k, v in seg.items()})
    out["per_batch_us"] = round(float(np.median(np.diff(done))) / 100, 3)
    out["span_us"] = round(float(done[-1] - t0) / 100, 2)
    out["span_per_batch_us"] = round(float(done[-1] - t0) / 100 / nb, 3)
    out["median_task_start_minus_prev_batch_done_us"] = round(float(np.median(lag)) / 100, 3)
    out["tasks_per_batch"] = round(float(np.mean([(st[t, :, 0] > 0).sum() for t in range(nb)])), 1)
    out.update(critical(st, S, ep, B, nb, done))
    print(json.dumps(out, indent=1))


def slot_counts(ep, B, t):
    """occurrence count of every slot of batch t (slot order: users by row, then items by row)"""
    s = slice(t * B, (t + 1) * B)
    u = ep.user[s].cpu().numpy()
    it = np.concatenate([ep.item_pos[s].cpu().numpy(), ep.item_neg[s].cpu().numpy()])
    _, cu = np.unique(u, return_counts=True)
    _, ci = np.unique(it, return_counts=True)
    return np.concatenate([cu, ci]), len(cu)


def critical(st, S, ep, B, nb, done):
    """What finishes a batch last, and how task time grows with the slot's occurrence count."""
    buckets = [(1, 1), (2, 2), (3, 4), (5, 8), (9, 16), (17, 1 << 30)]
    dur = {b: [] for b in buckets}
    w1 = {b: [] for b in buckets}
    last_cnt, last_item, last_start_lag, hot_end, hot_cnt = [], [], [], [], []
    for t in range(nb):
        cnt, nu = slot_counts(ep, B, t)
        w = st[t][: len(cnt)]
        ok = (w[:, 0] > 0) & (w[:, 5] > 0)
        for lo, hi in buckets:
            m = ok & (cnt >= lo) & (cnt <= hi) & (w[:, 2] > 0)
            dur[(lo, hi)] += list(w[m, 5] - w[m, 0])
            w1[(lo, hi)] += list(w[m, 2] - w[m, 1])
        k = int(np.argmax(np.where(ok, w[:, 5], 0)))
        if w[k, 5] == done[t]:  # a slot task ends the batch (else a fused group)
            last_cnt.append(int(cnt[k]))
            last_item.append(int(k >= nu))
            if t > 0:
                last_start_lag.append(w[k, 0] - done[t - 1])
        h = int(np.argmax(np.where(ok, cnt, 0)))
        hot_end.append(w[h, 5])
        hot_cnt.append(int(cnt[h]))
    med = lambda v: round(float(np.median(v)) / 100, 3) if len(v) else None
    out = {"task_us_by_count": {f"{lo}-{hi if hi < 1 << 30 else 'inf'}": [med(dur[(lo, hi)]), len(dur[(lo, hi)])]
                                for lo, hi in buckets},
           "wait1_us_by_count": {f"{lo}-{hi if hi < 1 << 30 else 'inf'}": med(w1[(lo, hi)]) for lo, hi in buckets},
           "batch_ender_count_median": float(np.median(last_cnt)) if last_cnt else None,
           "batch_ender_count_hist": np.bincount(np.minimum(last_cnt, 40)).tolist() if last_cnt else [],
           "batch_ender_is_item_frac": float(np.mean(last_item)) if last_item else None,
           "batches_ended_by_slot": len(last_cnt),
           "batch_ender_start_minus_prev_done_us": med(last_start_lag),
           "hottest_slot_count_median": float(np.median(hot_cnt)),
           "hottest_slot_end_to_end_us": med(np.diff(np.array(hot_end, dtype=np.float64)))}
    return out


if __name__ == "__main__":
    main()
