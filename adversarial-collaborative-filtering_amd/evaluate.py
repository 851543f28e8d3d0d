"""All-items / sampled evaluation: ``init_eval_model``, ``evaluate``,
``_eval_by_user`` (``utils.py:178-267``).

Per user the reference builds a candidate list, scores it with one
``sess.run(model.output)`` and takes ``position = #(neg >= pos)``; HR@k, NDCG@k
and AUC for k = 1..K follow from the position alone.  Here the candidate sets are
kept implicit ("all": every item in ``[0, num_items)`` minus the user's
``trainList`` and test item) or explicit ("sample": the 100 draws of
``utils.py:201-209``, reproduced exactly with Python's ``random`` seeded 2019), one
kernel computes every user's position, and the metrics are vectorised on the host.
"""
from __future__ import annotations

import math
import random

import numpy as np

from . import ops


class EvalPlan:
    """What init_eval_model returns: device-ready candidate descriptions."""

    def __init__(self, mode, users, tests, n_neg, K, excl_off=None, excl=None, cand_off=None,
                 cand=None, num_candidates=0):
        self.mode, self.users, self.tests, self.n_neg, self.K = mode, users, tests, n_neg, K
        self.excl_off, self.excl, self.cand_off, self.cand = excl_off, excl, cand_off, cand
        self.num_candidates = num_candidates
        self._dev = {}

    def device_arrays(self, device):
        import torch
        key = str(device)
        if key not in self._dev:
            T = lambda a, dt: torch.as_tensor(a, dtype=dt, device=device)  # noqa: E731
            if self.mode == "all":
                self._dev[key] = (T(self.users, torch.int32), T(self.tests, torch.int32),
                                  T(self.excl_off, torch.int64),
                                  T(self.excl if len(self.excl) else np.zeros(1), torch.int32))
            else:
                self._dev[key] = (T(self.users, torch.int32), T(self.tests, torch.int32),
                                  T(self.cand_off, torch.int64),
                                  T(self.cand if len(self.cand) else np.zeros(1), torch.int32))
        return self._dev[key]


def _sample_candidates(dataset, user, test_item, candidates):
    """utils.py:201-209 verbatim: random.seed(2019) per user, 100 draws from the
    df.iid list, redrawn while in trainList[user] or equal to the test item."""
    random.seed(2019)
    tl = set(dataset.trainList[user])
    out = []
    for _ in range(100):
        r = random.choice(candidates)
        while r in tl or test_item == r:
            r = random.choice(candidates)
        out.append(r)
    return out


def init_eval_model(dataset, args, users=None, twin=False):
    """utils.py:178-195 (twin=True: evaluation_adv.py:406-437 — users 1..U-1,
    item 0 never a candidate, K = 100)."""
    mode = "all" if twin else getattr(args, "eval_mode", "sample")
    if users is None:
        users = np.arange(1 if twin else 0, dataset.num_users, dtype=np.int64)
    users = np.asarray(users, dtype=np.int64)
    tests = np.asarray([dataset.testRatings[u][1] for u in users], dtype=np.int64)
    K = 100 if mode == "all" else 10
    if mode == "all":
        off, items = dataset.sorted_lists()
        n = dataset.num_items
        excl_lists = []
        n_neg = np.empty(len(users), dtype=np.int64)
        for k, u in enumerate(users.tolist()):
            tl = items[off[u]:off[u + 1]] if u < len(off) - 1 else np.zeros(0, np.int32)
            ex = np.union1d(tl, [tests[k]])
            if twin:
                ex = np.union1d(ex, [0])
            ex = ex[(ex >= 0) & (ex < n)]
            excl_lists.append(ex.astype(np.int32))
            n_neg[k] = n - len(ex)
        eo = np.zeros(len(users) + 1, dtype=np.int64)
        np.cumsum([len(e) for e in excl_lists], out=eo[1:])
        ex = np.concatenate(excl_lists) if excl_lists else np.zeros(0, np.int32)
        return EvalPlan("all", users, tests, n_neg, K, excl_off=eo, excl=ex, num_candidates=n)
    candidates = dataset.df.iid.tolist()
    cl = [_sample_candidates(dataset, int(u), int(t), candidates) for u, t in zip(users, tests)]
    co = np.zeros(len(users) + 1, dtype=np.int64)
    np.cumsum([len(c) for c in cl], out=co[1:])
    cand = np.concatenate([np.asarray(c, np.int32) for c in cl]) if cl else np.zeros(0, np.int32)
    n_neg = np.diff(co)
    return EvalPlan("sample", users, tests, n_neg, K, cand_off=co, cand=cand)


def positions(P, Q, plan: EvalPlan, kernel: str = "auto"):
    """Per-user position (#candidates scoring >= the test item), on the GPU
    (kernel: the all-items sweep, ops.eval_positions_all)."""
    dev = P.device
    u, t, o, c = plan.device_arrays(dev)
    if plan.mode == "all":
        return ops.eval_positions_all(P, Q, u, t, plan.num_candidates, o, c, kernel=kernel, unique_lists=True)
    return ops.eval_positions_list(P, Q, u, t, o, c)


def metrics_from_positions(pos, n_neg, K):
    """utils.py:256-261 for k = 1..K -> raw [U, 3, K] array of (hr, ndcg, auc)."""
    pos = np.asarray(pos, dtype=np.int64)
    ks = np.arange(1, K + 1)
    hit = pos[:, None] < ks[None, :]
    ndcg_val = np.array([math.log(2) / math.log(p + 2) for p in pos.tolist()], dtype=np.float64)
    ndcg = np.where(hit, ndcg_val[:, None], 0.0)
    auc = np.repeat((1 - (pos / np.asarray(n_neg, np.float64)))[:, None], K, axis=1)
    return np.stack([hit.astype(np.float64), ndcg, auc], axis=1)


def evaluate(model, sess, dataset, feed_dicts: EvalPlan, output_adv=0, args=None):
    """utils.py:221-241: returns ((hr, ndcg, auc) as per-K lists, raw [U,3,K])."""
    if output_adv:
        raise NotImplementedError("evaluation of model.output_adv is not on the APR path "
                                  "(APR.training always passes output_adv=0)")
    pos = positions(model.embedding_P, model.embedding_Q, feed_dicts).cpu().numpy()
    raw = metrics_from_positions(pos, feed_dicts.n_neg, feed_dicts.K)
    hr, ndcg, auc = raw.mean(axis=0).tolist()
    return (hr, ndcg, auc), raw
