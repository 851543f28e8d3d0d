"""Leave-one-out top-K evaluation of any ranker (evaluation.py:23-140 of the
reference): the protocol run.py uses for the Keras models (NeuMF, BPR, ...).

The ranker's ``rank(users, items)`` is called ONCE for every (user, candidate)
pair of the whole evaluation (the GPU scores them in one launch) instead of once
per user; the ranking rules are the reference's:

- ``evaluate_model`` (evaluation.py:23-80): users 1 .. len(testRatings)-1, item
  ``testRatings[u]`` against ``testNegatives[u]``; the top-K list is
  ``heapq.nlargest(K, {item: score})`` over the candidates in list order (the gt
  item appended), i.e. a stable sort, so a tie goes to the item listed first and
  a duplicated item keeps its first position and last score.  HR = gt in top K,
  NDCG = log 2 / log(rank + 2).
- ``evaluate_apr_mode`` (evaluation.py:94-140): every rating ``[u, gt]``, the first
  100 negatives; position = #(negatives scoring >= gt); HR@k / NDCG@k for
  k = 1..100.

Unlike evaluation.py:59 the caller's negative lists are not mutated (the
reference appends the gt item to them on every call).
"""
from __future__ import annotations

import math

import numpy as np


def getHitRatio(ranklist, gtItem):
    return 1 if gtItem in ranklist else 0


def getNDCG(ranklist, gtItem):
    for i, item in enumerate(ranklist):
        if item == gtItem:
            return math.log(2) / math.log(i + 2)
    return 0


def _scores(model, users, items):
    return np.asarray(model.rank(np.asarray(users), np.asarray(items)), dtype=np.float64).reshape(-1)


def evaluate_model(model, testRatings, testNegatives, K, num_thread=1):
    """evaluation.py:23-51 -> (hits, ndcgs), one entry per user 1..len-1."""
    idxs = range(1, len(testRatings))
    cands = [list(testNegatives[u]) + [testRatings[u]] for u in idxs]
    if not cands:
        return [], []
    users = np.concatenate([np.full(len(c), u, dtype=np.int64) for u, c in zip(idxs, cands)])
    items = np.concatenate([np.asarray(c, dtype=np.int64) for c in cands])
    sc = _scores(model, users, items)
    lens = np.array([len(c) for c in cands], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    # fast path: every list is duplicate-free with the gt item last (the lists
    # getDataset builds): the dict of evaluation.py:60-66 is then the list itself and
    # rank = #(negatives scoring >= gt)
    key = users * (int(items.max(initial=0)) + 1) + items
    if np.unique(key).size == key.size:
        gt_score = sc[starts + lens - 1]
        ge = (sc >= np.repeat(gt_score, lens)).astype(np.int64)
        rank = np.add.reduceat(ge, starts) - 1  # minus the gt item itself
        hits = [1 if r < K else 0 for r in rank.tolist()]
        ndcgs = [math.log(2) / math.log(r + 2) if r < K else 0 for r in rank.tolist()]
        return hits, ndcgs
    hits, ndcgs = [], []
    o = 0
    for u, c in zip(idxs, cands):
        s = sc[o: o + len(c)]
        o += len(c)
        gt = testRatings[u]
        # dict semantics: first position of an item, last score written for it
        first, last = {}, {}
        for pos, it in enumerate(c):
            first.setdefault(it, pos)
            last[it] = s[pos]
        order = sorted(first, key=lambda it: first[it])
        vals = np.array([last[it] for it in order])
        g = order.index(gt)
        rank = int((vals > vals[g]).sum() + (vals[:g] == vals[g]).sum())
        hits.append(1 if rank < K else 0)
        ndcgs.append(math.log(2) / math.log(rank + 2) if rank < K else 0)
    return hits, ndcgs


def evaluate_apr_mode(model, testRatings, testNegatives, K=100):
    """evaluation.py:94-140 -> (hr, ndcg) lists of K values per rating."""
    cands = [list(testNegatives[idx][:100]) + [testRatings[idx][1]] for idx in range(len(testRatings))]
    if not cands:
        return [], []
    users = np.concatenate([np.full(len(c), testRatings[x][0], dtype=np.int64) for x, c in enumerate(cands)])
    items = np.concatenate([np.asarray(c, dtype=np.int64) for c in cands])
    sc = _scores(model, users, items)
    hits, ndcgs = [], []
    o = 0
    for c in cands:
        s = sc[o: o + len(c)]
        o += len(c)
        position = int((s[:-1] >= s[-1]).sum())
        hits.append([position < k for k in range(1, K + 1)])
        ndcgs.append([math.log(2) / math.log(position + 2) if position < k else 0 for k in range(1, K + 1)])
    return hits, ndcgs
