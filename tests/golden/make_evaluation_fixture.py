"""Generate tests/golden/evaluation_ref.npz: the reference's evaluation.py
(`evaluate_model`, `evaluate_apr_mode`) run on a deterministic fake ranker whose
integer-valued scores create ties and whose candidate lists contain duplicates.
Run in the build container only (reads /root/reference); the outputs are data.

    python tests/golden/make_evaluation_fixture.py
"""
import os
import sys

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "evaluation_ref.npz")


class FakeRanker:
    """score(u, i) = ((u * 7 + i * 13) % 11), integer-valued -> many ties."""

    def rank(self, users, items):
        u = np.asarray(users, dtype=np.int64)
        i = np.asarray(items, dtype=np.int64)
        return (((u * 7 + i * 13) % 11).astype(np.float32)).reshape(-1, 1)


def main():
    sys.path.insert(0, REF)
    import evaluation as ref  # the reference module, imported as-is
    rng = np.random.default_rng(3)
    n_users, n_items = 60, 50
    test_items = rng.integers(1, n_items, n_users)
    negs = [list(map(int, rng.integers(1, n_items, 30))) for _ in range(n_users)]
    for u in range(0, n_users, 7):  # the gt item also among the negatives
        negs[u][3] = int(test_items[u])
    # DRCF mode: testRatings[u] = item
    hits, ndcgs = ref.evaluate_model(FakeRanker(), [int(x) for x in test_items],
                                     [list(n) for n in negs], 10, 1)
    # APR mode: testRatings[idx] = [u, item]
    ratings = [[u, int(test_items[u])] for u in range(n_users)]
    negs120 = [list(map(int, rng.integers(1, n_items, 120))) for _ in range(n_users)]
    hr_apr, ndcg_apr = ref.evaluate_apr_mode(FakeRanker(), ratings, [list(n) for n in negs120])
    np.savez(OUT, test_items=test_items, negs=np.array(negs), hits=np.array(hits),
             ndcgs=np.array(ndcgs, dtype=np.float64), negs120=np.array(negs120),
             hr_apr=np.array(hr_apr, dtype=bool), ndcg_apr=np.array(ndcg_apr, dtype=np.float64))
    print("wrote", OUT, len(hits), "users")


if __name__ == "__main__":
    main()
