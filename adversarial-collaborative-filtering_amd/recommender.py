"""``Recommender`` plugin interface (``Recommender.py:3-27``) and the ``APR`` class
``run.py`` dispatches to (``run.py:157-161,231-244``: ``APR(uNum, iNum, dim,
adver)``, ``get_params``, ``build_graph(path, opath, data, runName[, restore])``,
``get_train_instances``, ``train``, ``rank``, ``save``, ``load_pre_train``).

The reference imports ``from APR import APR`` but ``APR.py`` defines no such class
(``run.py:6``); this is the class that call site expects, implemented on the GPU
APR path.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from types import SimpleNamespace

import numpy as np

from . import ops
from .model import MF
from .sampler import EpochTriplets


class Recommender(ABC):
    """Recommender.py:3-27."""

    @abstractmethod
    def get_params(self):
        pass

    @abstractmethod
    def load_pre_train(self, pre):
        pass

    @abstractmethod
    def save(self, path):
        pass

    @abstractmethod
    def train(self, x_train, y_train, batch_size):
        pass

    @abstractmethod
    def rank(self, users, items):
        pass

    @abstractmethod
    def get_train_instances(self, train):
        pass


class APR(Recommender):
    """BPR-MF (adver=False) or APR (adver=True) behind the Recommender API."""

    def __init__(self, uNum, iNum, dim, adver=False, lr=0.05, eps=0.5, reg=0.0, reg_adv=1.0,
                 adv="grad", seed=None, device=None):
        self.uNum, self.iNum, self.dim, self.adver = int(uNum), int(iNum), int(dim), bool(adver)
        args = SimpleNamespace(embed_size=self.dim, lr=lr, reg=reg, dns=1, adv=adv, eps=eps,
                               adver=int(self.adver), reg_adv=reg_adv, epochs=0, seed=seed)
        # uNum/iNum are max id + 1 in run.py (run.py:114): tables sized like APR.py (+1)
        self.model = MF(self.uNum, self.iNum, args)
        self._device = device
        self._rng = np.random.RandomState(seed)

    def get_params(self):
        return "_e%.2f_l%.2f" % (self.model.eps, self.model.reg_adv) if self.adver else ""

    def build_graph(self, path="", opath="", data="", runName="", restore=False, previous=None):
        """Create the tables.  With restore=True the embeddings of `previous` (the BPR
        phase's ranker) are carried over and the Adagrad slots start fresh, like the
        phase switch of run_adv_ori.py:106-114."""
        self.model.build_graph(device=self._device)
        if restore and previous is not None:
            self.model.load_embeddings(previous.model.embedding_P.cpu(), previous.model.embedding_Q.cpu())
        self.path, self.opath, self.data, self.runName = path, opath, data, runName
        return self

    def _ensure(self):
        if not self.model.built:
            self.build_graph()

    def load_pre_train(self, pre):
        self._ensure()
        with np.load(pre if pre.endswith(".npz") else pre + ".npz", allow_pickle=False) as z:
            self.model.load_embeddings(z["embedding_P"], z["embedding_Q"])

    def save(self, path):
        self._ensure()
        ops.settle_tables()
        np.savez(path if path.endswith(".npz") else path + ".npz",
                 embedding_P=self.model.embedding_P.cpu().numpy(),
                 embedding_Q=self.model.embedding_Q.cpu().numpy())

    def get_train_instances(self, train):
        """Shuffled positives of a dok/CSR train matrix with one uniform negative
        each, rejected while (u, j) is a training pair (APR.py:64-81 rule)."""
        coo = train.tocoo() if hasattr(train, "tocoo") else train
        u = np.asarray(coo.row, dtype=np.int64)
        i = np.asarray(coo.col, dtype=np.int64)
        keys = np.unique(u * self.iNum + i)
        idx = self._rng.permutation(len(u))
        u, i = u[idx], i[idx]
        j = self._rng.randint(self.iNum, size=len(u)).astype(np.int64)
        for _ in range(10000):
            bad = np.isin(u * self.iNum + j, keys, assume_unique=False)
            if not bad.any():
                break
            j[bad] = self._rng.randint(self.iNum, size=int(bad.sum()))
        x = [u.astype(np.int32), i.astype(np.int32), j.astype(np.int32)]
        return x, np.ones(len(u), dtype=np.float32)

    def train(self, x_train, y_train, batch_size):
        """One pass over x_train in batches of batch_size (the trailing partial batch
        is dropped, as in APR.py:52); returns the mean clean loss per triplet."""
        import torch
        from .train import training_batch, training_loss_acc
        self._ensure()
        m = self.model
        n = (len(x_train[0]) // batch_size) * batch_size
        if n == 0:
            return float("nan")
        T = lambda a: torch.as_tensor(np.asarray(a[:n]), dtype=torch.int32, device=m.device)  # noqa
        ep = EpochTriplets(T(x_train[0]), T(x_train[1]), T(x_train[2]), batch_size)
        training_batch(m, None, ep, adver=self.adver)
        loss, _ = training_loss_acc(m, None, ep)
        return loss / batch_size

    def rank(self, users, items):
        self._ensure()
        return self.model.scores(np.asarray(users).reshape(-1), np.asarray(items).reshape(-1))
