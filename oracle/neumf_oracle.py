"""CPU restatement (numpy, fp32) of NeuMF and its adversarial training step.

TEST INFRASTRUCTURE ONLY: imported by tests/ (and nothing on the product path).

Model: the reference's `NeuMF` (NeuMF.py:10-52), a Keras graph:
  - four embedding tables MF_U [U+1, d], MF_I [I+1, d], MLP_U [U+1, d], MLP_I [I+1, d]
    (NeuMF.py:12-13,23-29; Keras `Embedding` init RandomUniform(-0.05, 0.05));
  - GMF tower: mf = MF_U[u] * MF_I[i] (NeuMF.py:32-34);
  - MLP tower: h0 = [MLP_U[u], MLP_I[i]] (2d), a1 = relu(h0 W1 + b1) (2d),
    a2 = relu(a1 W2 + b2) (d) (layers [d, 2d, d], NeuMF.py:15,37-42; Dense kernels
    [in, out], glorot-uniform init, zero bias);
  - head: p = sigmoid([mf, a2] Wo + bo) (NeuMF.py:44-47);
  - loss: Keras binary_crossentropy (mean over the batch; the prediction clipped
    to [1e-7, 1 - 1e-7], whose gradient passes only inside the clip range);
  - optimizer: Keras 2.2 Adam (lr 0.001, beta1 0.9, beta2 0.999, epsilon 1e-7),
    DENSE over every parameter every step: embedding rows without a gradient
    still decay their moments and move (Keras densifies IndexedSlices);
  - data: MF.py:42-56 `get_train_instances` (one positive + one rejected negative
    per training pair), Keras `fit(batch_size, shuffle=True)` keeps the last
    partial batch.

Adversarial variant: the reference's `AdversarialNeuMF` (NeuMF.py:58-185) trains
popularity discriminators and does not run (`self.popular_user_y` undefined,
NeuMF.py:131), so parity with it is unpinned.  This build defines it the APR way
(BASELINE configs[3]): the clean loss's batch gradient of each
touched row of the four tables gives delta = eps * g / sqrt(max(|g|^2, 1e-12))
(APR.py:180-191 applied per table), the adversarial loss is the same BCE on the
perturbed rows, and the optimised loss is clean + reg_adv * adversarial (the MLP
and head weights receive both gradients).

Row gradients are summed over a row's occurrences in instance order; weight
gradients over instances in order.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

F = np.float32
CLIP = F(1e-7)


@dataclass
class NeuMFHParams:
    lr: float = 0.001
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-7
    adver: int = 0
    eps: float = 0.5
    reg_adv: float = 1.0


NAMES = ("MF_U", "MF_I", "MLP_U", "MLP_I", "W1", "b1", "W2", "b2", "Wo", "bo")


def shapes(U1: int, I1: int, d: int):
    return {"MF_U": (U1, d), "MF_I": (I1, d), "MLP_U": (U1, d), "MLP_I": (I1, d),
            "W1": (2 * d, 2 * d), "b1": (2 * d,), "W2": (2 * d, d), "b2": (d,),
            "Wo": (2 * d, 1), "bo": (1,)}


def init_params(U1: int, I1: int, d: int, seed: int = 0):
    """Keras initialisers: Embedding U(-0.05, 0.05); Dense glorot-uniform, zero bias."""
    rng = np.random.default_rng(seed)
    out = {}
    for n, s in shapes(U1, I1, d).items():
        if n in ("MF_U", "MF_I", "MLP_U", "MLP_I"):
            out[n] = rng.uniform(-0.05, 0.05, s).astype(F)
        elif n.startswith("W"):
            lim = np.sqrt(6.0 / (s[0] + s[1]))
            out[n] = rng.uniform(-lim, lim, s).astype(F)
        else:
            out[n] = np.zeros(s, F)
    return out


def sigmoid(x):
    return (F(1) / (F(1) + np.exp(-x))).astype(F)


def forward(P, u, i, delta=None):
    """Per-instance activations; delta: optional dict table -> [B, d] perturbations."""
    mu, mi = P["MF_U"][u], P["MF_I"][i]
    lu, li = P["MLP_U"][u], P["MLP_I"][i]
    if delta is not None:
        mu, mi = mu + delta["MF_U"], mi + delta["MF_I"]
        lu, li = lu + delta["MLP_U"], li + delta["MLP_I"]
    h0 = np.concatenate([lu, li], 1).astype(F)
    z1 = (h0 @ P["W1"] + P["b1"]).astype(F)
    a1 = np.maximum(z1, F(0))
    z2 = (a1 @ P["W2"] + P["b2"]).astype(F)
    a2 = np.maximum(z2, F(0))
    f = np.concatenate([(mu * mi).astype(F), a2], 1).astype(F)
    logit = (f @ P["Wo"])[:, 0] + P["bo"][0]
    p = sigmoid(logit.astype(F))
    return dict(mu=mu, mi=mi, h0=h0, z1=z1, a1=a1, z2=z2, f=f, p=p)


def bce(p, y):
    pc = np.clip(p, CLIP, F(1) - CLIP)
    return float(np.mean(-(y * np.log(pc) + (1 - y) * np.log(1 - pc))))


def backward(P, act, u, i, y, scale=1.0):
    """Gradients of scale * mean-BCE: weight grads and per-instance row grads."""
    B = len(u)
    p = act["p"]
    inside = (p >= CLIP) & (p <= F(1) - CLIP)
    dlogit = np.where(inside, (p - y.astype(F)) * F(scale / B), F(0)).astype(F)
    g = {}
    g["Wo"] = (act["f"].T @ dlogit[:, None]).astype(F)
    g["bo"] = np.array([dlogit.sum()], F)
    df = (dlogit[:, None] * P["Wo"][:, 0][None, :]).astype(F)
    d = P["b2"].shape[0]
    dmf = df[:, :d]
    da2 = df[:, d:]
    dz2 = np.where(act["z2"] > 0, da2, F(0)).astype(F)
    g["W2"] = (act["a1"].T @ dz2).astype(F)
    g["b2"] = dz2.sum(0).astype(F)
    da1 = (dz2 @ P["W2"].T).astype(F)
    dz1 = np.where(act["z1"] > 0, da1, F(0)).astype(F)
    g["W1"] = (act["h0"].T @ dz1).astype(F)
    g["b1"] = dz1.sum(0).astype(F)
    dh0 = (dz1 @ P["W1"].T).astype(F)
    rows = {"MF_U": (dmf * act["mi"]).astype(F), "MF_I": (dmf * act["mu"]).astype(F),
            "MLP_U": dh0[:, :d], "MLP_I": dh0[:, d:]}
    return g, rows


def segment_sum(idx, contrib, n_rows):
    """Per-row sums in instance order (dense [n_rows, d])."""
    out = np.zeros((n_rows, contrib.shape[1]), F)
    for b in range(len(idx)):
        out[idx[b]] += contrib[b]
    return out


def grad_step(P, u, i, y, hp: NeuMFHParams):
    """Dense gradient of clean (+ reg_adv * adversarial) loss; returns (grads, loss_clean, loss_adv)."""
    U1, I1 = P["MF_U"].shape[0], P["MF_I"].shape[0]
    act = forward(P, u, i)
    g, rows = backward(P, act, u, i, y)
    lc = bce(act["p"], y)
    grads = {n: np.zeros_like(P[n]) for n in NAMES}
    for n in ("W1", "b1", "W2", "b2", "Wo", "bo"):
        grads[n] += g[n]
    sides = {"MF_U": (u, U1), "MF_I": (i, I1), "MLP_U": (u, U1), "MLP_I": (i, I1)}
    dense_rows = {n: segment_sum(sides[n][0], rows[n], sides[n][1]) for n in sides}
    for n in sides:
        grads[n] += dense_rows[n]
    la = 0.0
    if hp.adver:
        delta = {}
        for n, (idx, _) in sides.items():
            G = dense_rows[n][idx]
            ss = (G * G).sum(1, dtype=F)
            inv = (F(1) / np.sqrt(np.maximum(ss, F(1e-12)))).astype(F)
            delta[n] = (G * inv[:, None] * F(hp.eps)).astype(F)
        act_a = forward(P, u, i, delta)
        ga, rows_a = backward(P, act_a, u, i, y, scale=hp.reg_adv)
        la = bce(act_a["p"], y)
        for n in ("W1", "b1", "W2", "b2", "Wo", "bo"):
            grads[n] += ga[n]
        for n in sides:
            grads[n] += segment_sum(sides[n][0], rows_a[n], sides[n][1])
    return grads, lc, la


def adam(P, grads, m, v, t: int, hp: NeuMFHParams):
    """Keras 2.2 Adam, dense, iteration t (1-based)."""
    b1, b2 = F(hp.beta1), F(hp.beta2)
    lr_t = lr_t_f32(hp.lr, hp.beta1, hp.beta2, t)
    for n in NAMES:  # Keras: (b1 * m) + (1 - b1) * g; (b2 * v) + (1 - b2) * square(g)
        g = grads[n].astype(F)
        m[n] = (b1 * m[n] + (F(1) - b1) * g).astype(F)
        v[n] = (b2 * v[n] + (F(1) - b2) * (g * g)).astype(F)
        P[n] = (P[n] - (lr_t * m[n]) / (np.sqrt(v[n]) + F(hp.adam_eps))).astype(F)


def lr_t_f32(lr, beta1, beta2, t):
    """lr * sqrt(1 - b2^t) / (1 - b1^t) in float32 (Keras evaluates it on K.variables)."""
    b1, b2, tt = np.float32(beta1), np.float32(beta2), np.float32(t)
    num = np.sqrt(np.float32(1) - np.power(b2, tt, dtype=np.float32), dtype=np.float32)
    return np.float32(np.float32(lr) * np.float32(num / (np.float32(1) - np.power(b1, tt, dtype=np.float32))))


def predict(P, u, i):
    return forward(P, np.asarray(u), np.asarray(i))["p"]
