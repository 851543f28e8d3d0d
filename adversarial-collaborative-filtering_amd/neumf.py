"""NeuMF and adversarial NeuMF on the GPU (libacf_neumf.so, include/acf_neumf.h).

``NeuMF(uNum, iNum, mf_dim)`` is the reference's Keras model (NeuMF.py:10-52)
behind the Recommender API run.py drives (run.py:142-146,242-248):
``get_train_instances`` (MF.py:42-56: one positive + one rejected negative per
training pair), ``train(x_train, y_train, batch_size)`` (MF.py:30-33: Keras
``fit(shuffle=True)``, mean binary cross-entropy, Adam, last partial batch kept,
returns the epoch's mean loss), ``rank(users, items)`` (MF.py:38-40: sigmoid
scores, shape [n, 1]) and ``save``.

``AdversarialNeuMF(uNum, iNum, mf_dim, weight, pop_percent)`` keeps the reference
signature (NeuMF.py:58-59).  The reference's discriminator version does not run
(NeuMF.py:131), so the adversary here is APR's: FGSM perturbations of the touched
rows of the four embedding tables (eps * g/|g| of the clean gradient), with the
adversarial loss weighted by ``weight`` (the role of its ``loss_weights``,
NeuMF.py:110).  ``pop_percent`` is accepted and unused.  oracle/neumf_oracle.py
states the arithmetic.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from .ops import _idx, _require, _stream_ptr

NAMES = ("MF_U", "MF_I", "MLP_U", "MLP_I", "W1", "b1", "W2", "b2", "Wo", "bo")


def _shapes(U1, I1, d):
    return {"MF_U": (U1, d), "MF_I": (I1, d), "MLP_U": (U1, d), "MLP_I": (I1, d),
            "W1": (2 * d, 2 * d), "b1": (2 * d,), "W2": (2 * d, d), "b2": (d,),
            "Wo": (2 * d, 1), "bo": (1,)}


class NeuMFState:
    """Flat fp32 parameter / gradient / Adam-moment buffers in the C-ABI layout,
    with per-tensor views (Keras names and shapes)."""

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, device):
        self.U1, self.I1, self.d = int(num_user_rows), int(num_item_rows), int(dim)
        self.device = torch.device(device)
        lib = _native.load_neumf()
        n = lib.acf_neumf_param_count(self.U1, self.I1, self.d)
        if n < 0:
            raise ValueError(lib.acf_neumf_last_error().decode())
        off = (ctypes.c_int64 * 10)()
        _native.call_neumf("acf_neumf_param_offsets", self.U1, self.I1, self.d, off)
        self.offsets = list(off)
        f = dict(dtype=torch.float32, device=self.device)
        self.params = torch.zeros(n, **f)
        self.grad = torch.zeros(n, **f)
        self.m = torch.zeros(n, **f)
        self.v = torch.zeros(n, **f)
        self.t = 0  # Adam iterations done

    def view(self, name: str, buf: torch.Tensor | None = None) -> torch.Tensor:
        buf = self.params if buf is None else buf
        k = NAMES.index(name)
        shape = _shapes(self.U1, self.I1, self.d)[name]
        n = int(np.prod(shape))
        return buf[self.offsets[k]: self.offsets[k] + n].view(*shape)

    def load(self, arrays: dict) -> None:
        for n in NAMES:
            self.view(n).copy_(torch.as_tensor(np.asarray(arrays[n], dtype=np.float32)))

    def numpy(self) -> dict:
        return {n: self.view(n).cpu().numpy() for n in NAMES}

    def keras_init(self, seed=None) -> None:
        """Embedding RandomUniform(-0.05, 0.05); Dense glorot-uniform kernels, zero bias."""
        rng = np.random.default_rng(seed)
        arr = {}
        for n, s in _shapes(self.U1, self.I1, self.d).items():
            if n in ("MF_U", "MF_I", "MLP_U", "MLP_I"):
                arr[n] = rng.uniform(-0.05, 0.05, s)
            elif n.startswith("W"):
                lim = np.sqrt(6.0 / (s[0] + s[1]))
                arr[n] = rng.uniform(-lim, lim, s)
            else:
                arr[n] = np.zeros(s)
        self.load(arr)


class NeuMFContext:
    """Owns an ``acf_neumf_ctx`` (per-batch scratch for up to max_batch instances)."""

    def __init__(self, state: NeuMFState, max_batch: int):
        self.state, self.max_batch = state, int(max_batch)
        self._ptr = ctypes.c_void_p()
        with torch.cuda.device(state.device):
            _native.call_neumf("acf_neumf_create", ctypes.byref(self._ptr), state.U1, state.I1, state.d,
                               self.max_batch)

    def __del__(self):
        try:
            if self._ptr:
                _native.load_neumf().acf_neumf_destroy(self._ptr)
                self._ptr = ctypes.c_void_p()
        except Exception:
            pass

    def set_rows_in_line(self, on: bool) -> None:
        """Batches of <= 1,024 instances: rows summed inside the instance kernels
        (default) or by the separate row-sum kernel (bit-identical; tests / A/B)."""
        _native.call_neumf("acf_neumf_set_rows_in_line", self._ptr, int(bool(on)))

    def set_spin_limit(self, polls: int) -> None:
        """Polls a rows-in-line wait makes before it gives up (0: at once; tests)."""
        _native.call_neumf("acf_neumf_set_spin_limit", self._ptr, int(polls))

    def set_failsafe(self, on: bool) -> None:
        """On (default): a give-up is replayed exactly on the row-sum path;
        off: it raises RuntimeError."""
        _native.call_neumf("acf_neumf_set_failsafe", self._ptr, int(bool(on)))

    def recoveries(self) -> int:
        """Calls replayed after a rows-in-line give-up."""
        out = ctypes.c_int64()
        _native.call_neumf("acf_neumf_recoveries", self._ptr, ctypes.byref(out))
        return int(out.value)

    @staticmethod
    def hparams(lr=0.001, beta1=0.9, beta2=0.999, adam_eps=1e-7, adver=0, eps=0.5, reg_adv=1.0):
        return _native.NeuMFHParams(lr, beta1, beta2, adam_eps, eps, reg_adv, int(bool(adver)), 0)

    def grad(self, user, item, label, hp, loss_out: torch.Tensor | None = None, check=True) -> None:
        """Add the batch's loss gradient to state.grad (see acf_neumf_grad)."""
        s = self.state
        u, i = _idx(user, "user", s.device), _idx(item, "item", s.device)
        y = torch.as_tensor(label, dtype=torch.float32).reshape(-1).to(s.device).contiguous()
        if not (u.numel() == i.numel() == y.numel()):
            raise ValueError("user, item and label lengths differ")
        if not 0 < u.numel() <= self.max_batch:
            raise ValueError(f"batch of {u.numel()} outside (0, {self.max_batch}]")
        lp = 0 if loss_out is None else _require(loss_out, "loss_out", torch.float32, s.device)
        with torch.cuda.device(s.device):
            _native.call_neumf("acf_neumf_grad", self._ptr, s.params.data_ptr(), s.grad.data_ptr(),
                               u.data_ptr(), i.data_ptr(), y.data_ptr(), u.numel(), ctypes.byref(hp),
                               lp, int(bool(check)), _stream_ptr(s.device))
        self._keep = (u, i, y)

    def adam(self, hp) -> None:
        s = self.state
        s.t += 1
        with torch.cuda.device(s.device):
            _native.call_neumf("acf_neumf_adam", self._ptr, s.params.data_ptr(), s.grad.data_ptr(),
                               s.m.data_ptr(), s.v.data_ptr(), s.t, ctypes.byref(hp), _stream_ptr(s.device))

    def train(self, user, item, label, batch_size: int, hp) -> torch.Tensor:
        """One epoch over already-shuffled instances (acf_neumf_train); returns the
        per-batch [clean, adversarial] mean losses as a device tensor."""
        s = self.state
        u, i = _idx(user, "user", s.device), _idx(item, "item", s.device)
        y = torch.as_tensor(label, dtype=torch.float32).reshape(-1).to(s.device).contiguous()
        n = u.numel()
        if not (n == i.numel() == y.numel()):
            raise ValueError("user, item and label lengths differ")
        if not 0 < batch_size <= self.max_batch:
            raise ValueError(f"batch_size {batch_size} outside (0, {self.max_batch}]")
        nb = (n + batch_size - 1) // batch_size
        losses = torch.zeros(nb, 2, dtype=torch.float32, device=s.device)
        with torch.cuda.device(s.device):
            _native.call_neumf("acf_neumf_train", self._ptr, s.params.data_ptr(), s.grad.data_ptr(),
                               s.m.data_ptr(), s.v.data_ptr(), u.data_ptr(), i.data_ptr(), y.data_ptr(), n,
                               batch_size, s.t + 1, ctypes.byref(hp), losses.data_ptr(),
                               _stream_ptr(s.device))
        s.t += nb
        return losses

    def predict(self, user, item) -> torch.Tensor:
        s = self.state
        u, i = _idx(user, "user", s.device), _idx(item, "item", s.device)
        if u.numel() != i.numel():
            raise ValueError("user and item lengths differ")
        out = torch.empty(u.numel(), dtype=torch.float32, device=s.device)
        if u.numel():
            with torch.cuda.device(s.device):
                _native.call_neumf("acf_neumf_predict", self._ptr, s.params.data_ptr(), u.data_ptr(),
                                   i.data_ptr(), u.numel(), out.data_ptr(), _stream_ptr(s.device))
        return out


def mf_train_instances(train, iNum, rng):
    """MF.py:42-56: per training pair (u, i), in the train matrix's key order, a
    positive (label 1) and a negative j ~ U[1, iNum) redrawn while (u, j) is a
    training pair (label 0).  The reference redraws until the negative is valid;
    a user whose pairs cover all of [1, iNum) has none, and is refused here
    (the reference would loop forever)."""
    if hasattr(train, "keys"):
        pairs = np.array(list(train.keys()), dtype=np.int64).reshape(-1, 2)
        u, i = pairs[:, 0], pairs[:, 1]
    else:
        coo = train.tocoo()
        u, i = np.asarray(coo.row, np.int64), np.asarray(coo.col, np.int64)
    keys = np.unique(u * iNum + i)
    per_user = np.bincount((keys // iNum)[(keys % iNum) >= 1], minlength=int(u.max(initial=0)) + 1)
    if len(u) and (per_user[u] >= iNum - 1).any():
        raise ValueError("get_train_instances: a user has every item of [1, iNum) as a training pair")
    j = rng.randint(1, iNum, size=len(u)).astype(np.int64)
    bad = np.isin(u * iNum + j, keys)
    while bad.any():
        j[bad] = rng.randint(1, iNum, size=int(bad.sum()))
        bad = np.isin(u * iNum + j, keys)
    users = np.stack([u, u], 1).reshape(-1)
    items = np.stack([i, j], 1).reshape(-1)
    labels = np.tile(np.array([1, 0], dtype=np.int64), len(u))
    return [users, items], labels


class NeuMF:
    """NeuMF.py:10-55 on the GPU, with the run.py Recommender surface."""

    adver = 0

    def __init__(self, uNum, iNum, mf_dim=10, lr=0.001, seed=None, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("NeuMF needs a HIP device: there is no CPU path")
        self.uNum, self.iNum, self.dim = int(uNum) + 1, int(iNum) + 1, int(mf_dim)  # NeuMF.py:12-13
        self.device = torch.device(device if device is not None else "cuda")
        self.state = NeuMFState(self.uNum, self.iNum, self.dim, self.device)
        self.state.keras_init(seed)
        self.lr = float(lr)
        self.eps, self.reg_adv = 0.5, 1.0
        self._rng = np.random.RandomState(seed)
        self._ctx = None

    # -- helpers -----------------------------------------------------------------
    def _context(self, batch_size: int) -> NeuMFContext:
        if self._ctx is None or self._ctx.max_batch < batch_size:
            self._ctx = NeuMFContext(self.state, max(batch_size, 1024))
        return self._ctx

    def hparams(self):
        return NeuMFContext.hparams(lr=self.lr, adver=self.adver, eps=self.eps, reg_adv=self.reg_adv)

    # -- Recommender API -----------------------------------------------------------
    def get_params(self):
        return ""

    def get_train_instances(self, train):
        """MF.py:42-56 (see mf_train_instances)."""
        return mf_train_instances(train, self.iNum, self._rng)

    def train(self, x_train, y_train, batch_size):
        """Keras fit for one epoch (MF.py:30-33): shuffled, batches of batch_size
        including the last partial one, one Adam step each; returns the mean loss
        (batch losses weighted by batch size, as Keras' History reports)."""
        users = np.asarray(x_train[0]).reshape(-1)
        items = np.asarray(x_train[1]).reshape(-1)
        y = np.asarray(y_train, dtype=np.float32).reshape(-1)
        n = len(y)
        if n == 0:
            return float("nan")
        perm = self._rng.permutation(n)
        dev = self.device
        U = torch.as_tensor(users[perm], dtype=torch.int32).to(dev)
        I = torch.as_tensor(items[perm], dtype=torch.int32).to(dev)
        Y = torch.as_tensor(y[perm]).to(dev)
        ctx = self._context(batch_size)
        nb = (n + batch_size - 1) // batch_size
        losses = ctx.train(U, I, Y, batch_size, self.hparams())
        weights = torch.full((nb,), float(batch_size))
        weights[-1] = n - (nb - 1) * batch_size
        lc = losses[:, 0].cpu()
        la = losses[:, 1].cpu()
        total = lc + (self.reg_adv * la if self.adver else 0.0)
        return float((total * weights).sum() / weights.sum())

    def rank(self, users, items):
        """MF.py:38-40 (model.predict): scores of shape [n, 1]."""
        ctx = self._context(1)
        out = ctx.predict(np.asarray(users).reshape(-1), np.asarray(items).reshape(-1))
        return out.cpu().numpy().reshape(-1, 1)

    def save(self, path):
        np.savez(path if path.endswith(".npz") else path + ".npz", **self.state.numpy())

    def load_pre_train(self, pre):
        with np.load(pre if pre.endswith(".npz") else pre + ".npz", allow_pickle=False) as z:
            self.state.load({n: z[n] for n in NAMES})


class AdversarialNeuMF(NeuMF):
    """NeuMF + FGSM adversary on the four embedding tables (see module docstring)."""

    adver = 1

    def __init__(self, uNum, iNum, mf_dim, weight=1.0, pop_percent=0.2, eps=0.5, lr=0.001, seed=None,
                 device=None):
        super().__init__(uNum, iNum, mf_dim, lr=lr, seed=seed, device=device)
        self.weight, self.pop_percent = float(weight), float(pop_percent)
        self.eps, self.reg_adv = float(eps), float(weight)

    def get_params(self):
        return "_w%.3f_e%.2f" % (self.weight, self.eps)
