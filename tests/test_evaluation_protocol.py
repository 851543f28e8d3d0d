"""evaluation.py protocol (run.py's leave-one-out top-K) against the reference's
own evaluation.py, run on a tie-heavy fake ranker with duplicated candidates
(fixture made by tests/golden/make_evaluation_fixture.py)."""
import importlib
import os

import numpy as np

from conftest import GOLDEN, PKG


class FakeRanker:
    def rank(self, users, items):
        u = np.asarray(users, dtype=np.int64)
        i = np.asarray(items, dtype=np.int64)
        return (((u * 7 + i * 13) % 11).astype(np.float32)).reshape(-1, 1)


def test_evaluate_model_matches_reference():
    ev = importlib.import_module(PKG + ".evaluation")
    z = np.load(os.path.join(GOLDEN, "evaluation_ref.npz"))
    negs = [list(map(int, r)) for r in z["negs"]]
    before = [list(n) for n in negs]
    hits, ndcgs = ev.evaluate_model(FakeRanker(), [int(x) for x in z["test_items"]], negs, 10)
    np.testing.assert_array_equal(hits, z["hits"])
    np.testing.assert_allclose(ndcgs, z["ndcgs"], rtol=0, atol=1e-15)
    assert negs == before  # the caller's lists are left alone


def test_evaluate_apr_mode_matches_reference():
    ev = importlib.import_module(PKG + ".evaluation")
    z = np.load(os.path.join(GOLDEN, "evaluation_ref.npz"))
    ratings = [[u, int(t)] for u, t in enumerate(z["test_items"])]
    hr, ndcg = ev.evaluate_apr_mode(FakeRanker(), ratings, [list(map(int, r)) for r in z["negs120"]])
    np.testing.assert_array_equal(np.array(hr, dtype=bool), z["hr_apr"])
    np.testing.assert_allclose(ndcg, z["ndcg_apr"], rtol=0, atol=1e-15)


def test_evaluate_model_fast_path_equals_dict_rules():
    """Duplicate-free candidate lists (gt last) take the vectorised path; it must
    give the reference's dict/nlargest ranks (evaluation.py:60-66) exactly, ties
    included."""
    ev = importlib.import_module(PKG + ".evaluation")
    rng = np.random.default_rng(3)
    nu, ni = 40, 30
    S = rng.integers(0, 4, (nu, ni)).astype(np.float64)  # few values: many ties

    class R:
        def rank(self, users, items):
            return S[np.asarray(users), np.asarray(items)].reshape(-1, 1)

    tests = [0] + [int(x) for x in rng.integers(0, ni, nu - 1)]
    negs = [[]] + [[int(x) for x in rng.permutation([k for k in range(ni) if k != tests[u]])[:12]]
                   for u in range(1, nu)]
    hits, ndcgs = ev.evaluate_model(R(), tests, negs, 5)
    for u in range(1, nu):
        c = negs[u] + [tests[u]]
        first = {}
        for p_, it in enumerate(c):
            first.setdefault(it, p_)
        order = sorted(first, key=first.get)
        vals = np.array([S[u, it] for it in order])
        g = order.index(tests[u])
        r = int((vals > vals[g]).sum() + (vals[:g] == vals[g]).sum())
        assert hits[u - 1] == (1 if r < 5 else 0)
        assert ndcgs[u - 1] == (np.log(2) / np.log(r + 2) if r < 5 else 0)
