"""CPU oracle for the APR hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the checker / the timed CPU baseline.  The
product package never imports it.

Two independent restatements of the reference's TF1 graph (``APR.py:121-195``
driven by ``utils.py:106-119``):

* :class:`COracle` — ctypes binding of ``oracle/apr_oracle.c`` (row-set based,
  optionally doing the reference's dense full-table delta work).
* :func:`tf_graph_step` — numpy, materialises the graph the way TF evaluates it:
  gathers, ``matmul(p*q, h)``, ``clip_by_value``, ``softplus``, IndexedSlices
  densified with an unsorted segment sum, full-table ``l2_normalize`` and
  ``assign``, then the optimizer's dedup + ``SparseApplyAdagrad``.

Parity status: op-level parity with the reference is UNPINNED (TensorFlow is not
installed, so the reference graph cannot be executed here); see the header of
``apr_oracle.c`` and DESIGN.md §Oracle for what pins it instead.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle_apr.so")

SOFTPLUS_T = np.float32(13.942385)


class _OHP(ctypes.Structure):
    _fields_ = [
        ("lr", ctypes.c_float), ("eps", ctypes.c_float), ("reg", ctypes.c_float),
        ("reg_adv", ctypes.c_float), ("clip_lo", ctypes.c_float), ("clip_hi", ctypes.c_float),
        ("adver", ctypes.c_int32), ("zero_delta", ctypes.c_int32), ("dense", ctypes.c_int32),
        ("adv_mode", ctypes.c_int32), ("call", ctypes.c_uint32), ("t", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]


@dataclass
class HParams:
    lr: float = 0.05
    eps: float = 0.5
    reg: float = 0.0
    reg_adv: float = 1.0
    clip_lo: float = -80.0
    clip_hi: float = 1e8
    adver: int = 1
    zero_delta: int = 0
    adv: str = "grad"   # "grad" | "random" (APR.py:170-191)
    seed: int = 0       # random mode: the HIP step's hparams seed ...
    call: int = 1       # ... the context's call counter (1 for a fresh context's first call) ...
    t: int = 0          # ... and the batch index inside the planned range (apr_batch)


def _f32p(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i32p(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _i64p(a):
    assert a.dtype == np.int64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


class COracle:
    """ctypes wrapper of liboracle_apr.so (built by build_native.build_oracle)."""

    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            import importlib.util
            spec = importlib.util.spec_from_file_location("_acf_oracle_build", os.path.join(HERE, "build.py"))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build(verbose=False)
        self.lib = ctypes.CDLL(path)
        L = self.lib
        P = ctypes.c_void_p
        L.oracle_apr_batch.restype = ctypes.c_int
        L.oracle_apr_batch.argtypes = [P, P, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                       P, P, P, ctypes.c_int, ctypes.POINTER(_OHP), P, P, P, P]
        L.oracle_apr_train.restype = ctypes.c_int
        L.oracle_apr_train.argtypes = [P, P, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                       P, P, P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_OHP)]
        L.oracle_apr_train_mt.restype = ctypes.c_int
        L.oracle_apr_train_mt.argtypes = [P, P, P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                          P, P, P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_OHP), ctypes.c_int]
        L.oracle_bpr_forward.restype = ctypes.c_int
        L.oracle_bpr_forward.argtypes = [P, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, P, P, P,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                         P, P, P, P]
        L.oracle_eval_positions_all.restype = ctypes.c_int
        L.oracle_eval_positions_all.argtypes = [P, P, ctypes.c_int, P, P, ctypes.c_int, ctypes.c_int,
                                                P, P, P]
        L.oracle_eval_positions_list.restype = ctypes.c_int
        L.oracle_eval_positions_list.argtypes = [P, P, ctypes.c_int, P, P, ctypes.c_int, P, P, P]

    @staticmethod
    def _hp(hp: HParams, dense: bool) -> _OHP:
        if hp.adv not in ("grad", "random"):
            raise ValueError(f"adv must be 'grad' or 'random', got {hp.adv!r}")
        return _OHP(hp.lr, hp.eps, hp.reg, hp.reg_adv, hp.clip_lo, hp.clip_hi, int(hp.adver),
                    int(hp.zero_delta), int(dense), 0 if hp.adv == "grad" else 1, int(hp.call) & 0xFFFFFFFF,
                    int(hp.t), int(hp.seed) & 0xFFFFFFFFFFFFFFFF)

    def apr_batch(self, P, Q, accP, accQ, u, i, j, hp: HParams, dense=False, want_delta=False):
        """One training_batch iteration, in place.  Returns (loss_clean, loss_adv, dP, dQ)."""
        B = len(u)
        lc = np.zeros(B, np.float32)
        la = np.zeros(B, np.float32)
        dP = np.zeros_like(P) if want_delta else None
        dQ = np.zeros_like(Q) if want_delta else None
        h = self._hp(hp, dense)
        r = self.lib.oracle_apr_batch(
            P.ctypes.data, Q.ctypes.data, accP.ctypes.data, accQ.ctypes.data, P.shape[0], Q.shape[0],
            P.shape[1], _c(u), _c(i), _c(j), B, ctypes.byref(h), lc.ctypes.data, la.ctypes.data,
            dP.ctypes.data if want_delta else None, dQ.ctypes.data if want_delta else None)
        if r:
            raise ValueError(f"oracle_apr_batch failed ({r}): index out of range" if r == -2
                             else f"oracle_apr_batch failed ({r})")
        return lc, la, dP, dQ

    def apr_train(self, P, Q, accP, accQ, u, i, j, batch_size, hp: HParams, dense=False):
        nb = len(u) // batch_size
        h = self._hp(hp, dense)
        r = self.lib.oracle_apr_train(P.ctypes.data, Q.ctypes.data, accP.ctypes.data,
                                      accQ.ctypes.data, P.shape[0], Q.shape[0], P.shape[1], _c(u),
                                      _c(i), _c(j), batch_size, nb, ctypes.byref(h))
        if r:
            raise ValueError(f"oracle_apr_train failed ({r})")

    def apr_train_mt(self, P, Q, accP, accQ, u, i, j, batch_size, hp: HParams, dense=False, threads=None):
        """apr_train on `threads` OpenMP threads (default: every core of this
        process's affinity mask): the same bits (apr_oracle.c, oracle_apr_train_mt)."""
        nb = len(u) // batch_size
        h = self._hp(hp, dense)
        nt = int(threads or len(os.sched_getaffinity(0)))
        r = self.lib.oracle_apr_train_mt(P.ctypes.data, Q.ctypes.data, accP.ctypes.data,
                                         accQ.ctypes.data, P.shape[0], Q.shape[0], P.shape[1], _c(u),
                                         _c(i), _c(j), batch_size, nb, ctypes.byref(h), nt)
        if r:
            raise ValueError(f"oracle_apr_train_mt failed ({r})")
        return nt

    def bpr_forward(self, P, Q, u, i, j, batch_size, clip_lo=-80.0, clip_hi=1e8):
        nb = len(u) // batch_size
        bl = np.zeros(nb, np.float32)
        bc = np.zeros(nb, np.int32)
        op = np.zeros(nb * batch_size, np.float32)
        on = np.zeros(nb * batch_size, np.float32)
        r = self.lib.oracle_bpr_forward(P.ctypes.data, Q.ctypes.data, P.shape[0], Q.shape[0],
                                        P.shape[1], _c(u), _c(i), _c(j), batch_size, nb, clip_lo,
                                        clip_hi, bl.ctypes.data, bc.ctypes.data, op.ctypes.data,
                                        on.ctypes.data)
        if r:
            raise ValueError(f"oracle_bpr_forward failed ({r})")
        return bl, bc, op, on

    def eval_positions_all(self, P, Q, users, tests, num_cand, excl_off, excl):
        pos = np.zeros(len(users), np.int32)
        self.lib.oracle_eval_positions_all(P.ctypes.data, Q.ctypes.data, P.shape[1], _c(users),
                                           _c(tests), len(users), int(num_cand),
                                           _c64(excl_off), _c(excl), pos.ctypes.data)
        return pos

    def eval_positions_list(self, P, Q, users, tests, cand_off, cand):
        pos = np.zeros(len(users), np.int32)
        self.lib.oracle_eval_positions_list(P.ctypes.data, Q.ctypes.data, P.shape[1], _c(users),
                                            _c(tests), len(users), _c64(cand_off), _c(cand),
                                            pos.ctypes.data)
        return pos


def _c(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    _c._keep.append(a)
    if len(_c._keep) > 64:
        del _c._keep[:32]
    return a.ctypes.data


_c._keep = []


def _c64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    _c._keep.append(a)
    return a.ctypes.data


# ---------------------------------------------------------------------------
# numpy restatement that evaluates the TF graph literally (dense)
# ---------------------------------------------------------------------------
def _softplus(f):
    f = f.astype(np.float32)
    with np.errstate(over="ignore"):
        e = np.exp(f)
        return np.where(f > SOFTPLUS_T, f,
                        np.where(f < -SOFTPLUS_T, e, np.log(e + np.float32(1)))).astype(np.float32)


def _sigmoid_grad(r):
    # SoftplusGrad(1, -r) negated: -1 / (exp(r) + 1)
    with np.errstate(over="ignore"):
        return (-np.float32(1) / (np.exp(r) + np.float32(1))).astype(np.float32)


def _inference(P, Q, u, items, dP=None, dQ=None):
    p = P[u]
    q = Q[items]
    if dP is not None:
        p = (p + dP[u]).astype(np.float32)
        q = (q + dQ[items]).astype(np.float32)
    return (p * q).astype(np.float32).sum(axis=1, dtype=np.float32), p, q


def _l2_normalize(x):
    ss = np.square(x).sum(axis=1, keepdims=True, dtype=np.float32)
    return (x * (np.float32(1) / np.sqrt(np.maximum(ss, np.float32(1e-12))))).astype(np.float32)


def tf_graph_step(P, Q, accP, accQ, u, i, j, hp: HParams):
    """One training_batch iteration evaluated like the TF graph (dense delta).

    Returns (loss_clean, loss_adv, delta_P, delta_Q); P, Q, accP, accQ updated in
    place.  utils.py:117-119 / APR.py:143-195.
    """
    f32 = np.float32
    B, d = len(u), P.shape[1]
    xp, p, qi = _inference(P, Q, u, i)
    xn, _, qj = _inference(P, Q, u, j)
    x = (xp - xn).astype(f32)
    r = np.clip(x, f32(hp.clip_lo), f32(hp.clip_hi))
    mask = ((x >= hp.clip_lo) & (x <= hp.clip_hi)).astype(f32)
    loss_clean = _softplus(-r)
    g = (_sigmoid_grad(r) * mask).astype(f32)
    dP = np.zeros_like(P)
    dQ = np.zeros_like(Q)
    loss_adv = None
    if hp.adver:
        # tf.gradients(loss, [P, Q]) -> IndexedSlices -> dense (unsorted_segment_sum)
        gP = np.zeros_like(P)
        gQ = np.zeros_like(Q)
        np.add.at(gP, u, g[:, None] * qi)
        np.add.at(gQ, i, g[:, None] * p)
        np.add.at(gP, u, -g[:, None] * qj)
        np.add.at(gQ, j, -g[:, None] * p)
        if not hp.zero_delta:
            dP = (_l2_normalize(gP) * f32(hp.eps)).astype(f32)
            dQ = (_l2_normalize(gQ) * f32(hp.eps)).astype(f32)
        xpa, pa, qia = _inference(P, Q, u, i, dP, dQ)
        xna, _, qja = _inference(P, Q, u, j, dP, dQ)
        xa = (xpa - xna).astype(f32)
        ra = np.clip(xa, f32(hp.clip_lo), f32(hp.clip_hi))
        maska = ((xa >= hp.clip_lo) & (xa <= hp.clip_hi)).astype(f32)
        loss_adv = _softplus(-ra)
        ga = (_sigmoid_grad(ra) * maska).astype(f32)
    # optimizer: IndexedSlices of opt_loss, deduplicated by summation
    GP = np.zeros_like(P)
    GQ = np.zeros_like(Q)
    np.add.at(GP, u, g[:, None] * qi)
    np.add.at(GQ, i, g[:, None] * p)
    np.add.at(GP, u, -g[:, None] * qj)
    np.add.at(GQ, j, -g[:, None] * p)
    if hp.reg:
        coef = f32(2.0 * hp.reg / (B * d)) * f32(2 if hp.adver else 1)
        np.add.at(GP, u, coef * p)
        np.add.at(GQ, i, coef * qi)
        np.add.at(GQ, j, coef * qj)
    if hp.adver:
        lam = f32(hp.reg_adv)
        np.add.at(GP, u, lam * ga[:, None] * qia)
        np.add.at(GQ, i, lam * ga[:, None] * pa)
        np.add.at(GP, u, -lam * ga[:, None] * qja)
        np.add.at(GQ, j, -lam * ga[:, None] * pa)
    for W, A, G, rows in ((P, accP, GP, np.unique(u)), (Q, accQ, GQ, np.unique(np.concatenate([i, j])))):
        gr = G[rows]
        A[rows] = (A[rows] + gr * gr).astype(f32)
        W[rows] = (W[rows] - (f32(hp.lr) * gr) * (f32(1) / np.sqrt(A[rows]))).astype(f32)
    return loss_clean, loss_adv, dP, dQ


def eval_metrics(positions, n_neg, K):
    """HR/NDCG/AUC for k = 1..K from positions (utils.py:256-261)."""
    positions = np.asarray(positions, dtype=np.int64)
    ks = np.arange(1, K + 1)
    hit = positions[:, None] < ks[None, :]
    hr = hit.astype(np.float64)
    ndcg = np.where(hit, np.log(2) / np.log(positions[:, None] + 2.0), 0.0)
    auc = np.repeat((1.0 - positions / np.asarray(n_neg, dtype=np.float64))[:, None], K, axis=1)
    return hr, ndcg, auc
