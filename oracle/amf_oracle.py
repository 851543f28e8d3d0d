"""CPU restatement (numpy, fp32) of the reference's FastAdversarialMF ("amf2") training step.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and nothing on the product path).

Reference: FastAdversarialMF.py:13-144 (run.py --model amf2, run.py:140-141), a Keras
model built on MatrixFactorization (MF.py:7-59) and the third-party keras_adversarial
(AdversarialModel + AdversarialOptimizerSimultaneous; not vendored, not installed).
The reference does not run as written, so parity with it is
UNPINNED; this file states the arithmetic the HIP path implements:

  tables     P [uNum, d], Q [iNum, d] (Embedding, RandomUniform(-0.05, 0.05)), :28-29
  prediction pred = P[u] . Q[i] (dot), :48; loss MSE vs the 0/1 label, :74
  discriminators D_u, D_i: Dense(d, relu) -> Dense(1, sigmoid) on an embedding row
             (generate_discriminator, :119-127; glorot-uniform kernels, zero bias),
             fed P[ua] / Q[ia] for sampled popular / rare user and item indices
             (:31-32 uAdvEmb / iAdvEmb go through the shared embedding layers)
  players    (AdversarialModel, :60-67; AdversarialOptimizerSimultaneous: every
             player's gradient taken at the same pre-step parameters, each player's
             own Keras Adam applied at once):
               "mf"     params P, Q:  MSE + BCE(D_u(P[ua]), tu) + BCE(D_i(Q[ia]), ti)
               "disc_u" params D_u:   BCE(D_u(P[ua]), du)
               "disc_i" params D_i:   BCE(D_i(Q[ia]), di)
             loss weights 1 (:69-71).  Targets as train() writes them (:112-113):
             the mf player (y, user_y, item_y), the discriminator players the
             reversed popularity labels (y, user_y[::-1], item_y[::-1]).
  Adam       Keras 2.2 Adam (lr 0.001) per player; all three step every batch,
             so one dense Adam over the whole buffer with one iteration count is
             the same arithmetic (embedding IndexedSlices densified: every row's
             moments decay).

BCE is Keras 2.2's binary_crossentropy (prediction clipped to [1e-7, 1 - 1e-7];
gradient (s - t) / B inside the clip, 0 outside), as in oracle/neumf_oracle.py.
Row gradients are summed per row in occurrence order (P: the u gathers, then the
ua gathers; Q: i, then ia); weight gradients over instances in order.
"""
from __future__ import annotations

import numpy as np

from neumf_oracle import CLIP, lr_t_f32, sigmoid

F = np.float32
DISC = ("W1", "b1", "W2", "b2")


def disc_shapes(d: int):
    return {"W1": (d, d), "b1": (d,), "W2": (d,), "b2": (1,)}


def disc_block(d: int) -> int:
    """Floats of one discriminator in the flat buffer: W1 | b1 | W2 | b2 | 3 pad."""
    return d * d + 2 * d + 4


def param_count(uNum: int, iNum: int, d: int) -> int:
    return (uNum + iNum) * d + 2 * disc_block(d)


def unflatten(buf, uNum, iNum, d):
    """Views of the flat buffer: P, Q, Du{W1,b1,W2,b2}, Di{...}."""
    P = buf[: uNum * d].reshape(uNum, d)
    Q = buf[uNum * d: (uNum + iNum) * d].reshape(iNum, d)
    discs = []
    o = (uNum + iNum) * d
    for _ in range(2):
        D = {"W1": buf[o: o + d * d].reshape(d, d), "b1": buf[o + d * d: o + d * d + d],
             "W2": buf[o + d * d + d: o + d * d + 2 * d], "b2": buf[o + d * d + 2 * d: o + d * d + 2 * d + 1]}
        discs.append(D)
        o += disc_block(d)
    return P, Q, discs[0], discs[1]


def init_params(uNum: int, iNum: int, d: int, seed: int = 0):
    """Keras initialisers: Embedding U(-0.05, 0.05); Dense glorot-uniform, zero bias."""
    rng = np.random.default_rng(seed)
    buf = np.zeros(param_count(uNum, iNum, d), F)
    P, Q, Du, Di = unflatten(buf, uNum, iNum, d)
    P[:] = rng.uniform(-0.05, 0.05, P.shape)
    Q[:] = rng.uniform(-0.05, 0.05, Q.shape)
    for D in (Du, Di):
        lim = np.sqrt(6.0 / (d + d))
        D["W1"][:] = rng.uniform(-lim, lim, (d, d))
        lim2 = np.sqrt(6.0 / (d + 1))
        D["W2"][:] = rng.uniform(-lim2, lim2, d)
    return buf


def bce_terms(s, t):
    sc = np.clip(s, CLIP, F(1) - CLIP)
    return (-(t * np.log(sc) + (1 - t) * np.log(1 - sc))).astype(F)


def popularity_split(x, pop_percent):
    """get_discriminator_train_data (FastAdversarialMF.py:129-144): ids by count,
    descending (Python's stable ascending sort, reversed: among equal counts the
    one first seen LAST comes first), the first pop_percent of them popular."""
    x = np.asarray(x).reshape(-1)
    ids, first, counts = np.unique(x, return_index=True, return_counts=True)
    order = np.argsort(first, kind="stable")  # dict insertion order
    ids, counts = ids[order], counts[order]
    asc = np.argsort(counts, kind="stable")   # sorted(..., key=count)
    ranked = ids[asc][::-1]
    k = int(len(ranked) * pop_percent)
    return ranked[:k], ranked[k:]


def disc_forward(D, e):
    h = (e @ D["W1"] + D["b1"]).astype(F)
    a = np.maximum(h, F(0))
    z = ((a * D["W2"]).sum(1, dtype=F) + D["b2"][0]).astype(F)
    return h, a, sigmoid(z)


def grad_step(buf, uNum, iNum, d, u, i, y, ua, ia, tu, ti, du, di):
    """Dense gradient of the three players' losses for one batch (each player's
    segment of the flat buffer gets its own loss's gradient); returns
    (grad, mf_loss, (mse, bce_u, bce_i))."""
    P, Q, Du, Di = unflatten(buf, uNum, iNum, d)
    G = np.zeros_like(buf)
    GP, GQ, GDu, GDi = unflatten(G, uNum, iNum, d)
    B = len(u)
    y, tu, ti, du, di = (np.asarray(x, F) for x in (y, tu, ti, du, di))
    invB = F(1.0 / B)
    pu, qi = P[u], Q[i]
    pred = (pu * qi).sum(1, dtype=F)
    diff = (pred - y).astype(F)
    mse = (diff * diff).astype(F)
    dpred = ((diff * F(2)) * invB).astype(F)
    rowsP = [(u, (dpred[:, None] * qi).astype(F))]
    rowsQ = [(i, (dpred[:, None] * pu).astype(F))]
    bces = []
    for D, GD, E, idx, tm, td, rows in ((Du, GDu, P, ua, tu, du, rowsP), (Di, GDi, Q, ia, ti, di, rowsQ)):
        e = E[idx]
        h, a, s = disc_forward(D, e)
        bces.append(bce_terms(s, tm))
        inside = (s >= CLIP) & (s <= F(1) - CLIP)
        dzm = np.where(inside, ((s - tm) * invB).astype(F), F(0)).astype(F)
        dzd = np.where(inside, ((s - td) * invB).astype(F), F(0)).astype(F)
        relu = h > 0
        dhm = np.where(relu, (dzm[:, None] * D["W2"][None, :]).astype(F), F(0)).astype(F)
        de = (dhm @ D["W1"].T).astype(F)
        rows.append((idx, de))
        dhd = np.where(relu, (dzd[:, None] * D["W2"][None, :]).astype(F), F(0)).astype(F)
        GD["W1"][:] = (e.T @ dhd).astype(F)
        GD["b1"][:] = dhd.sum(0, dtype=F)
        GD["W2"][:] = (a * dzd[:, None]).sum(0, dtype=F)
        GD["b2"][:] = dzd.sum(dtype=F)
    for GT, rows in ((GP, rowsP), (GQ, rowsQ)):
        for idx, c in rows:  # occurrence order
            for b in range(B):
                GT[idx[b]] = GT[idx[b]] + c[b]
    parts = (float(mse.astype(np.float64).mean()), float(bces[0].astype(np.float64).mean()),
             float(bces[1].astype(np.float64).mean()))
    return G, sum(parts), parts


def adam(buf, G, m, v, t, lr=0.001, beta1=0.9, beta2=0.999, eps=1e-7):
    """Keras 2.2 Adam, dense, iteration t (1-based)."""
    b1, b2 = F(beta1), F(beta2)
    lr_t = lr_t_f32(lr, beta1, beta2, t)
    m[:] = (b1 * m + (F(1) - b1) * G).astype(F)
    v[:] = (b2 * v + (F(1) - b2) * (G * G)).astype(F)
    buf[:] = (buf - (lr_t * m) / (np.sqrt(v) + F(eps))).astype(F)


def train_epoch(buf, m, v, t_first, uNum, iNum, d, inst, batch):
    """One Keras fit epoch over already-shuffled instances `inst` = (u, i, y, ua, ia,
    tu, ti, du, di) arrays; batches of `batch`, the last one partial.  Returns the
    per-batch mf-player losses."""
    n = len(inst[0])
    out = []
    for k, o in enumerate(range(0, n, batch)):
        s = slice(o, o + batch)
        G, loss, _ = grad_step(buf, uNum, iNum, d, *(x[s] for x in inst))
        adam(buf, G, m, v, t_first + k)
        out.append(loss)
    return out
