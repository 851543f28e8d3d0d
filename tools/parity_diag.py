#!/usr/bin/env python
"""Where the HIP path and the oracle part at the headline shape, and why.

ml-1m-shaped DeviceSampler triplets, B = 512, d = 64, APR.  Batch by batch
(delta_update, optimizer_step: the same per-row summation order as k_stream),
compare the GPU delta rows and tables with the oracle's.  For every touched row
whose delta differs by more than 1e-6, report the conditioning of its clean
gradient sum, kappa = sum_k |term_k| / |sum_k term_k| (elementwise, max over the
row): the summation-order rounding of the gradient is ~ n u sum|term|, and
l2_normalize turns it into a delta change of ~ eps * n u kappa.
"""
from __future__ import annotations

import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
from apr_oracle import COracle, HParams  # noqa: E402

PKG = "adversarial-collaborative-filtering_amd"


def clean_terms(P, Q, u, i, j):
    """Per-occurrence clean gradient terms of every user / item row (oracle order)."""
    p, qi, qj = P[u], Q[i], Q[j]
    x = (p * qi).sum(1) - (p * qj).sum(1)
    g = -1.0 / (np.exp(x) + 1.0)
    terms = {}
    for b in range(len(u)):
        terms.setdefault(("u", u[b]), []).extend([g[b] * qi[b], -g[b] * qj[b]])
        terms.setdefault(("i", i[b]), []).append(g[b] * p[b])
        terms.setdefault(("i", j[b]), []).append(-g[b] * p[b])
    return terms


def main():
    dev = torch.device("cuda", 0)
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    B, d, nb = 512, 64, int(sys.argv[1]) if len(sys.argv) > 1 else 32
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=0).epoch(0)
    u, i, j = (x[: nb * B].cpu().numpy() for x in (ep.user, ep.item_pos, ep.item_neg))
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    g = torch.Generator().manual_seed(0)
    P0 = torch.nn.init.trunc_normal_(torch.empty(U1, d), 0, 0.01, -0.02, 0.02, generator=g).numpy()
    Q0 = torch.nn.init.trunc_normal_(torch.empty(I1, d), 0, 0.01, -0.02, 0.02, generator=g).numpy()
    o = COracle()
    hp_c = HParams(adver=1)
    hp = ops.StepHParams(adver=1)
    rP, rQ = P0.copy(), Q0.copy()
    aP, aQ = np.full(P0.shape, 0.1, np.float32), np.full(Q0.shape, 0.1, np.float32)
    tabs = [torch.tensor(P0, device=dev), torch.tensor(Q0, device=dev),
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, 1, dev)
    out = []
    for t in range(nb):
        s = slice(t * B, (t + 1) * B)
        # the GPU steps from the ORACLE's tables, so each batch's deviation is its own
        for x, w in zip(tabs, (rP, rQ, aP, aQ)):
            x.copy_(torch.from_numpy(w))
        terms = clean_terms(rP.astype(np.float64), rQ.astype(np.float64), u[s], i[s], j[s])
        ctx.plan(torch.tensor(u[s], device=dev), torch.tensor(i[s], device=dev),
                 torch.tensor(j[s], device=dev), B)
        ctx.delta_update(tabs, hp, 0)
        gdP, gdQ = (x.cpu().numpy() for x in ctx.delta_tables())
        ctx.optimizer_step(tabs, hp, 0)
        lc, la, dP, dQ = o.apr_batch(rP, rQ, aP, aQ, u[s], i[s], j[s], hp_c, want_delta=True)
        torch.cuda.synchronize()
        for side, gd, od in (("u", gdP, dP), ("i", gdQ, dQ)):
            diff = np.abs(gd - od).max(1)
            for r in np.nonzero(diff > 1e-6)[0]:
                T = np.array(terms[(side, r)])
                kappa = float((np.abs(T).sum(0) / np.maximum(np.abs(T.sum(0)), 1e-30)).max())
                out.append({"batch": t, "side": side, "row": int(r), "occurrences": len(T),
                            "delta_maxdiff": float(diff[r]), "grad_norm": float(np.linalg.norm(T.sum(0))),
                            "kappa_max": round(kappa, 1)})
        tab_diff = max(float(np.abs(x.cpu().numpy() - w).max()) for x, w in zip(tabs, (rP, rQ, aP, aQ)))
        out.append({"batch": t, "table_maxdiff_one_step": tab_diff})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
