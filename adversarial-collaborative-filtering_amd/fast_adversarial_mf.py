"""The reference's ``FastAdversarialMF`` (FastAdversarialMF.py:13-144; ``run.py
--model amf2``, run.py:140-141) on the GPU (libacf_neumf.so, include/acf_neumf.h
"FastAdversarialMF").

Model: a MatrixFactorization (MF.py:7-59) -- P[u] . Q[i] trained with MSE on the
0/1 labels of MF.py:42-56 -- and two popularity discriminators Dense(d, relu) ->
Dense(1, sigmoid) (:119-127) on embedding rows of sampled popular / rare users and
items, trained as a three-player keras_adversarial game (:60-71) with
AdversarialOptimizerSimultaneous and one Keras Adam per player.

The reference cannot run as written, so these choices are ours (DESIGN.md §11;
parity unpinned, oracle/amf_oracle.py states the arithmetic):
  * run.py never calls ``init`` for amf2: the popular / rare split is taken from the
    first ``train`` call's instances (users, items), as amf / abpr do (run.py:131-137);
  * ``train`` feeds the encoders' embedding VECTORS to the index inputs
    userAdvInput / itemAdvInput (:98-107): the sampled INDICES are used, which the
    graph (:31-32) gathers through the shared embedding layers;
  * ``fit`` gets 6 targets for 3 players x 3 outputs (:112-115): the mf player takes
    the first triple (label, user_y, item_y), each discriminator player the second
    (label, user_y reversed, item_y reversed);
  * the loss weights are 1 (:69-71) and ``weight`` is kept for get_params only, as in
    the reference (its only use is the commented-out advModel).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from .neumf import mf_train_instances
from .ops import _idx, _stream_ptr
from .recommender import Recommender


def popularity_split(x, pop_percent):
    """get_discriminator_train_data (FastAdversarialMF.py:129-144): ids ranked by
    count, descending; among equal counts the id first seen last comes first (the
    reference's stable ascending sort, reversed); the first pop_percent popular."""
    x = np.asarray(x).reshape(-1)
    ids, first, counts = np.unique(x, return_index=True, return_counts=True)
    order = np.argsort(first, kind="stable")
    ids, counts = ids[order], counts[order]
    ranked = ids[np.argsort(counts, kind="stable")][::-1]
    k = int(len(ranked) * pop_percent)
    return ranked[:k], ranked[k:]


class FastAdversarialMF(Recommender):
    def __init__(self, uNum, iNum, dim, weight=1.0, pop_percent=0.2, lr=0.001, seed=None, device=None):
        if not torch.cuda.is_available() and device is None:
            raise RuntimeError("FastAdversarialMF needs a HIP device: there is no CPU path")
        self.uNum, self.iNum, self.dim = int(uNum), int(iNum), int(dim)
        self.weight, self.pop_percent = float(weight), float(pop_percent)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.hp = _native.NeuMFHParams(lr, 0.9, 0.999, 1e-7, 0.0, 0.0, 0, 0)
        n = self.param_count(self.uNum, self.iNum, self.dim)
        self.params = torch.as_tensor(self.keras_init(self.uNum, self.iNum, self.dim, seed)).to(self.device)
        f = dict(dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(n, **f)
        self.m = torch.zeros(n, **f)
        self.v = torch.zeros(n, **f)
        self.t = 0
        self._rng = np.random.RandomState(seed)
        self.popular_user_x = self.rare_user_x = self.popular_item_x = self.rare_item_x = None
        self._ctx, self._ctx_batch = ctypes.c_void_p(), 0

    # -- layout --------------------------------------------------------------------
    @staticmethod
    def disc_block(d):
        return d * d + 2 * d + 4

    @classmethod
    def param_count(cls, uNum, iNum, d):
        return (uNum + iNum) * d + 2 * cls.disc_block(d)

    @classmethod
    def keras_init(cls, uNum, iNum, d, seed=None):
        """Embedding RandomUniform(-0.05, 0.05); Dense glorot-uniform kernels, zero biases."""
        rng = np.random.default_rng(seed)
        buf = np.zeros(cls.param_count(uNum, iNum, d), np.float32)
        buf[: (uNum + iNum) * d] = rng.uniform(-0.05, 0.05, (uNum + iNum) * d)
        o = (uNum + iNum) * d
        for _ in range(2):
            buf[o: o + d * d] = rng.uniform(-np.sqrt(6.0 / (2 * d)), np.sqrt(6.0 / (2 * d)), d * d)
            lim2 = np.sqrt(6.0 / (d + 1))
            buf[o + d * d + d: o + d * d + 2 * d] = rng.uniform(-lim2, lim2, d)
            o += cls.disc_block(d)
        return buf

    @property
    def uEmb(self) -> torch.Tensor:
        return self.params[: self.uNum * self.dim].view(self.uNum, self.dim)

    @property
    def iEmb(self) -> torch.Tensor:
        return self.params[self.uNum * self.dim: (self.uNum + self.iNum) * self.dim].view(self.iNum, self.dim)

    def discriminator(self, which: str) -> dict:
        """Views of D_u ("user") / D_i ("item"): W1 [d, d], b1 [d], W2 [d], b2 [1]."""
        d = self.dim
        o = (self.uNum + self.iNum) * d + (0 if which == "user" else self.disc_block(d))
        p = self.params
        return {"W1": p[o: o + d * d].view(d, d), "b1": p[o + d * d: o + d * d + d],
                "W2": p[o + d * d + d: o + d * d + 2 * d], "b2": p[o + d * d + 2 * d: o + d * d + 2 * d + 1]}

    def __del__(self):
        try:
            if self._ctx:
                _native.load_neumf().acf_amf_destroy(self._ctx)
        except Exception:
            pass

    def _context(self, batch):
        if batch > self._ctx_batch:
            if self._ctx:
                _native.load_neumf().acf_amf_destroy(self._ctx)
                self._ctx = ctypes.c_void_p()
            with torch.cuda.device(self.device):
                _native.call_neumf("acf_amf_create", ctypes.byref(self._ctx), self.uNum, self.iNum, self.dim,
                                   int(batch))
            self._ctx_batch = int(batch)
        return self._ctx

    # -- Recommender API -----------------------------------------------------------
    def get_params(self):
        return "_w%.3f_pp%.2f" % (self.weight, self.pop_percent)

    def init(self, users, items):
        """FastAdversarialMF.py:84-86."""
        self.popular_user_x, self.rare_user_x = popularity_split(users, self.pop_percent)
        self.popular_item_x, self.rare_item_x = popularity_split(items, self.pop_percent)

    def get_train_instances(self, train):
        return mf_train_instances(train, self.iNum, self._rng)

    def adversarial_instances(self, n):
        """FastAdversarialMF.py:91-107: n // 2 popular and n // 2 rare sampled users
        (and items), labels 1 / 0; the mf player's targets and the discriminators'
        (reversed).  An odd n repeats the last rare draw (the reference's arrays
        would be one short)."""
        h = n // 2

        def draw(pop, rare):
            if len(pop) == 0 or len(rare) == 0:
                raise ValueError("FastAdversarialMF: pop_percent leaves no popular or no rare ids")
            x = np.concatenate([pop[self._rng.randint(0, len(pop), h)], rare[self._rng.randint(0, len(rare), h)]])
            y = np.concatenate([np.ones(h), np.zeros(h)]).astype(np.float32)
            if len(x) < n:
                x, y = np.append(x, x[-1:]), np.append(y, y[-1:])
            return x, y

        ux, uy = draw(self.popular_user_x, self.rare_user_x)
        ix, iy = draw(self.popular_item_x, self.rare_item_x)
        return ux, ix, uy, iy, uy[::-1].copy(), iy[::-1].copy()

    def train(self, x_train, y_train, batch_size):
        """One advModel.fit epoch (FastAdversarialMF.py:89-117, Keras shuffle=True,
        the last partial batch kept); returns the mf player's mean loss (MSE +
        both BCE terms), batch losses weighted by batch size."""
        users = np.asarray(x_train[0]).reshape(-1)
        items = np.asarray(x_train[1]).reshape(-1)
        y = np.asarray(y_train, dtype=np.float32).reshape(-1)
        n = len(y)
        if n == 0:
            return float("nan")
        if self.popular_user_x is None:
            self.init(users, items)
        ux, ix, tu, ti, du, di = self.adversarial_instances(n)
        perm = self._rng.permutation(n)
        dev = self.device
        I32 = lambda a: torch.as_tensor(np.asarray(a)[perm], dtype=torch.int32).to(dev).contiguous()
        F32 = lambda a: torch.as_tensor(np.asarray(a, np.float32)[perm]).to(dev).contiguous()
        U, It, UA, IA = I32(users), I32(items), I32(ux), I32(ix)
        Y, TU, TI, DU, DI = F32(y), F32(tu), F32(ti), F32(du), F32(di)
        B = int(min(batch_size, n))
        losses = torch.empty(n, 3, dtype=torch.float32, device=dev)
        ctx = self._context(B)
        with torch.cuda.device(dev):
            _native.call_neumf("acf_amf_train", ctx, self.params.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(),
                               self.v.data_ptr(), U.data_ptr(), It.data_ptr(), Y.data_ptr(), UA.data_ptr(),
                               IA.data_ptr(), TU.data_ptr(), TI.data_ptr(), DU.data_ptr(), DI.data_ptr(), n, B,
                               self.t + 1, ctypes.byref(self.hp), losses.data_ptr(), _stream_ptr(dev))
        self.t += (n + B - 1) // B
        return float(losses.double().sum(1).mean())

    def grad_batch(self, u, i, y, ua, ia, tu, ti, du, di):
        """The three players' gradient of one batch (device tensors), ADDED to
        self.grad; returns the per-instance losses [B, 3] (tests)."""
        B = int(u.numel())
        out = torch.empty(B, 3, dtype=torch.float32, device=self.device)
        ctx = self._context(B)
        with torch.cuda.device(self.device):
            _native.call_neumf("acf_amf_grad", ctx, self.params.data_ptr(), self.grad.data_ptr(), u.data_ptr(),
                               i.data_ptr(), y.data_ptr(), ua.data_ptr(), ia.data_ptr(), tu.data_ptr(), ti.data_ptr(),
                               du.data_ptr(), di.data_ptr(), B, out.data_ptr(), _stream_ptr(self.device))
        return out

    def rank(self, users, items):
        u = _idx(users, "users", self.device)
        it = _idx(items, "items", self.device)
        out = torch.empty(u.numel(), dtype=torch.float32, device=self.device)
        ctx = self._context(max(self._ctx_batch, 1))
        with torch.cuda.device(self.device):
            _native.call_neumf("acf_amf_predict", ctx, self.params.data_ptr(), u.data_ptr(), it.data_ptr(),
                               u.numel(), out.data_ptr(), _stream_ptr(self.device))
        return out.cpu().numpy().reshape(-1, 1)

    def save(self, path):
        """npz with the Keras layer names: the two embedding tables and the
        discriminators' Dense kernels / biases."""
        du, di = self.discriminator("user"), self.discriminator("item")
        arrs = {"uEmb": self.uEmb.cpu().numpy(), "iEmb": self.iEmb.cpu().numpy()}
        for tag, D in (("disc_u", du), ("disc_i", di)):
            for k, t in D.items():
                arrs[f"{tag}_{k}"] = t.cpu().numpy()
        np.savez(path if path.endswith(".npz") else path + ".npz", **arrs)

    def load_pre_train(self, pre):
        with np.load(pre if pre.endswith(".npz") else pre + ".npz", allow_pickle=False) as z:
            self.uEmb.copy_(torch.as_tensor(z["uEmb"]))
            self.iEmb.copy_(torch.as_tensor(z["iEmb"]))
            for tag, which in (("disc_u", "user"), ("disc_i", "item")):
                D = self.discriminator(which)
                for k in D:
                    if f"{tag}_{k}" in z:
                        D[k].copy_(torch.as_tensor(z[f"{tag}_{k}"]))
