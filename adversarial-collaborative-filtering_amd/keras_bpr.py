"""The reference's Keras ``BPR`` (BPR.py:23-99) on the GPU (libacf_neumf.so,
include/acf_neumf.h "Keras BPR"): the model ``run.py --model bpr`` trains
(BASELINE.json configs[0]).

Same surface as the reference class: ``BPR(uNum, iNum, dim)``,
``get_train_instances(train)`` (BPR.py:83-99: every training pair with one
negative drawn uniformly from [1, iNum) and redrawn while it is a training pair
of the user), ``train(x_train, y_train, batch_size)`` (BPR.py:70-81: Keras
``fit(shuffle=True, epochs=1)``: loss mean(1 - log(sigmoid(u.p - u.n))), Keras
2.2 Adam lr 0.001, the last partial batch kept; returns the epoch's mean loss),
``rank(users, items)`` (BPR.py:67-68: the predictor's u.i, shape [n, 1]),
``save`` / ``load_pre_train`` (npz with the Keras layer names ``uEmb`` /
``iEmb``) and ``get_params``.  Initialisation: Keras Embedding's
RandomUniform(-0.05, 0.05).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from .ops import _idx, _stream_ptr
from .recommender import Recommender


class BPR(Recommender):
    def __init__(self, uNum, iNum, dim, lr=0.001, beta1=0.9, beta2=0.999, adam_eps=1e-7, seed=None, device=None):
        self.uNum, self.iNum, self.dim = int(uNum), int(iNum), int(dim)
        self.dns = 1
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.hp = _native.NeuMFHParams(lr, beta1, beta2, adam_eps, 0.0, 0.0, 0, 0)
        f = dict(dtype=torch.float32, device=self.device)
        n = (self.uNum + self.iNum) * self.dim
        rng = np.random.default_rng(seed)
        self.params = torch.as_tensor(rng.uniform(-0.05, 0.05, n).astype(np.float32)).to(self.device)
        self.grad = torch.zeros(n, **f)
        self.m = torch.zeros(n, **f)
        self.v = torch.zeros(n, **f)
        self.t = 0  # Adam iterations done
        self._rng = np.random.RandomState(seed)
        self._ctx, self._ctx_batch = ctypes.c_void_p(), 0

    def __del__(self):
        try:
            if self._ctx:
                _native.load_neumf().acf_kbpr_destroy(self._ctx)
        except Exception:
            pass

    # -- Keras layer views -------------------------------------------------------
    @property
    def uEmb(self) -> torch.Tensor:
        return self.params[: self.uNum * self.dim].view(self.uNum, self.dim)

    @property
    def iEmb(self) -> torch.Tensor:
        return self.params[self.uNum * self.dim:].view(self.iNum, self.dim)

    def _context(self, batch):
        if batch > self._ctx_batch:
            if self._ctx:
                _native.load_neumf().acf_kbpr_destroy(self._ctx)
                self._ctx = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                _native.call_neumf("acf_kbpr_create", ctypes.byref(self._ctx), self.uNum, self.iNum, self.dim,
                                   int(batch))
            self._ctx_batch = int(batch)
        return self._ctx

    # -- Recommender API -----------------------------------------------------------
    def get_params(self):
        return ""

    def get_train_instances(self, train):
        """BPR.py:83-99: pairs in train.keys() order, one rejected negative each."""
        if hasattr(train, "keys") and not hasattr(train, "tocoo"):
            keys = list(train.keys())
            u = np.array([k[0] for k in keys], dtype=np.int64)
            i = np.array([k[1] for k in keys], dtype=np.int64)
        else:
            coo = train.tocoo()
            u, i = np.asarray(coo.row, np.int64), np.asarray(coo.col, np.int64)
        member = np.unique(u * self.iNum + i)
        # the reference redraws until the negative is valid (BPR.py:90-92); a user whose
        # pairs cover every item of [1, iNum) would make it loop forever: refuse instead
        mu = member // self.iNum
        per_user = np.bincount(mu[(member % self.iNum) >= 1], minlength=int(u.max(initial=0)) + 1)
        if len(u) and (per_user[u] >= self.iNum - 1).any():
            raise ValueError("get_train_instances: a user has every item of [1, iNum) as a training pair, "
                             "so no negative exists for it")
        j = self._rng.randint(1, self.iNum, size=len(u)).astype(np.int64)
        bad = np.isin(u * self.iNum + j, member)
        while bad.any():
            j[bad] = self._rng.randint(1, self.iNum, size=int(bad.sum()))
            bad = np.isin(u * self.iNum + j, member)
        return [u.astype(np.int32), i.astype(np.int32), j.astype(np.int32)], np.ones(len(u), dtype=np.int64)

    def train(self, x_train, y_train, batch_size):
        """One Keras fit epoch (shuffle=True); returns the mean loss."""
        n = len(x_train[0])
        if n == 0:
            return float("nan")
        perm = torch.as_tensor(self._rng.permutation(n), device=self.device)
        u, i, j = (torch.as_tensor(np.asarray(x), dtype=torch.int32).to(self.device)[perm].contiguous()
                   for x in x_train)
        losses = torch.empty(n, dtype=torch.float32, device=self.device)
        ctx = self._context(min(batch_size, n))
        with torch.cuda.device(self.device):
            _native.call_neumf("acf_kbpr_train", ctx, self.params.data_ptr(), self.grad.data_ptr(),
                               self.m.data_ptr(), self.v.data_ptr(), u.data_ptr(), i.data_ptr(), j.data_ptr(), n,
                               int(min(batch_size, n)), self.t + 1, ctypes.byref(self.hp), losses.data_ptr(),
                               _stream_ptr(self.device))
        self.t += (n + batch_size - 1) // batch_size
        return float(losses.double().mean())

    def rank(self, users, items):
        u = _idx(users, "users", self.device)
        it = _idx(items, "items", self.device)
        out = torch.empty(u.numel(), dtype=torch.float32, device=self.device)
        ctx = self._context(max(self._ctx_batch, 1))
        with torch.cuda.device(self.device):
            _native.call_neumf("acf_kbpr_predict", ctx, self.params.data_ptr(), u.data_ptr(), it.data_ptr(),
                               u.numel(), out.data_ptr(), _stream_ptr(self.device))
        return out.cpu().numpy().reshape(-1, 1)

    def save(self, path):
        np.savez(path if path.endswith(".npz") else path + ".npz", uEmb=self.uEmb.cpu().numpy(),
                 iEmb=self.iEmb.cpu().numpy())

    def load_pre_train(self, pre):
        with np.load(pre if pre.endswith(".npz") else pre + ".npz", allow_pickle=False) as z:
            self.uEmb.copy_(torch.as_tensor(z["uEmb"]))
            self.iEmb.copy_(torch.as_tensor(z["iEmb"]))
