"""Host logic of the Keras BPR drop-in (keras_bpr.py): get_train_instances
(BPR.py:83-99) on CPU tensors; no kernel runs."""
import importlib

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import PKG


def _bpr(uNum, iNum, seed=0):
    return importlib.import_module(PKG + ".keras_bpr").BPR(uNum, iNum, 8, seed=seed, device="cpu")


def test_negatives_are_never_training_pairs():
    """A dense user (every item but two) still gets valid negatives: the redraw
    runs until the negative is not a training pair (BPR.py:90-92)."""
    uNum, iNum = 6, 12
    rows, cols = [0] * 9, list(range(1, 10))  # user 0: items 1..9 of [1, 12) -> negatives 10, 11
    rng = np.random.default_rng(1)
    for u in range(1, uNum):
        for it in rng.choice(np.arange(1, iNum), 3, replace=False):
            rows.append(u)
            cols.append(int(it))
    train = sp.dok_matrix((uNum, iNum), dtype=np.float32)
    for r, c in zip(rows, cols):
        train[r, c] = 1.0
    (u, i, j), y = _bpr(uNum, iNum).get_train_instances(train)
    pairs = set(zip(rows, cols))
    assert len(u) == len(pairs) and (y == 1).all()
    assert all((int(a), int(b)) not in pairs for a, b in zip(u, j))
    assert ((j >= 1) & (j < iNum)).all()
    assert set(j[u == 0].tolist()) <= {10, 11}


def test_saturated_user_is_refused():
    """A user whose pairs cover all of [1, iNum) has no negative: the reference
    loops forever; the drop-in raises."""
    uNum, iNum = 3, 5
    train = sp.dok_matrix((uNum, iNum), dtype=np.float32)
    for it in range(1, iNum):
        train[1, it] = 1.0
    train[2, 3] = 1.0
    with pytest.raises(ValueError):
        _bpr(uNum, iNum).get_train_instances(train)
