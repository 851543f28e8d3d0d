"""CPU restatement of the reference's Keras BPR training epoch — TEST INFRASTRUCTURE ONLY.

BPR.py:23-81 (run.py --model bpr): x = u.p - u.n (Dot layers, BPR.py:42-43);
loss = 1 - log(sigmoid(x)) (bpr_triplet_loss, BPR.py:11-16); the Keras loss is
its batch mean (identity_loss, BPR.py:19-20); the embedding gradients are
IndexedSlices densified by summing per row (users in batch order, items: the
positive gathers then the negative ones); Keras 2.2 Adam (keras/optimizers.py
Adam.get_updates: lr_t = lr sqrt(1 - b2^t) / (1 - b1^t), m, v, p -= lr_t m /
(sqrt(v) + eps)) over the whole buffer (dense: every row's moments decay).
Keras/TF are not installed here, so parity with the reference is UNPINNED at
op level; tests check this restatement against torch autograd of the same loss
(tests/test_neumf_oracle.py) and the HIP path against this restatement.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def kbpr_grad(params, U1, d, u, i, j):
    """Dense gradient of mean(1 - log(sigmoid(u.p - u.n))) over one batch and the
    per-triplet losses."""
    P = params[: U1 * d].reshape(U1, d)
    Q = params[U1 * d:].reshape(-1, d)
    B = len(u)
    pu, pp, pn = P[u], Q[i], Q[j]
    x = ((pu * pp).sum(1, dtype=f32) - (pu * pn).sum(1, dtype=f32)).astype(f32)
    with np.errstate(over="ignore"):
        s = (f32(1) / (f32(1) + np.exp(-x))).astype(f32)
    loss = (f32(1) - np.log(s)).astype(f32)
    up = f32(-1.0 / B)
    g = ((up * (f32(1) / s)) * s * (f32(1) - s)).astype(f32)
    G = np.zeros_like(params)
    GP = G[: U1 * d].reshape(U1, d)
    GQ = G[U1 * d:].reshape(-1, d)
    gu = (g[:, None] * pp + (-g)[:, None] * pn).astype(f32)
    for b in range(B):
        GP[u[b]] = GP[u[b]] + gu[b]
    for b in range(B):
        GQ[i[b]] = GQ[i[b]] + (g[b] * pu[b]).astype(f32)
    for b in range(B):
        GQ[j[b]] = GQ[j[b]] + (-g[b] * pu[b]).astype(f32)
    return G, loss


def keras_adam(params, G, m, v, t, lr=0.001, b1=0.9, b2=0.999, eps=1e-7):
    tt = f32(t)
    lr_t = f32(lr) * (np.sqrt(f32(1) - np.power(f32(b2), tt)) / (f32(1) - np.power(f32(b1), tt)))
    c1, c2 = f32(1) - f32(b1), f32(1) - f32(b2)  # float32, as Keras' constants
    m[:] = (f32(b1) * m + c1 * G).astype(f32)
    v[:] = (f32(b2) * v + c2 * (G * G)).astype(f32)
    params[:] = (params - (f32(lr_t) * m) / (np.sqrt(v) + f32(eps))).astype(f32)


def kbpr_epoch(params, m, v, t_first, U1, d, u, i, j, batch):
    """One Keras fit epoch over already-shuffled triplets; returns per-triplet losses."""
    losses = []
    for k, o in enumerate(range(0, len(u), batch)):
        s = slice(o, o + batch)
        G, loss = kbpr_grad(params, U1, d, u[s], i[s], j[s])
        keras_adam(params, G, m, v, t_first + k)
        losses.append(loss)
    return np.concatenate(losses) if losses else np.zeros(0, f32)
