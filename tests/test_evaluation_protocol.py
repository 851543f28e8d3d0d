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
