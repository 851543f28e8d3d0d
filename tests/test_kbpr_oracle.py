"""The Keras-BPR restatement (oracle/kbpr_oracle.py, BPR.py:11-81) against torch
autograd of the same loss: mean over the batch of 1 - log(sigmoid(u.p - u.n))."""
import numpy as np
import torch

from kbpr_oracle import kbpr_epoch, kbpr_grad


def _problem(seed=0, U1=17, I1=13, d=8, B=24):
    rng = np.random.default_rng(seed)
    params = rng.uniform(-0.5, 0.5, (U1 + I1) * d).astype(np.float32)
    u = rng.integers(0, U1, B)
    i = rng.integers(1, I1, B)
    j = rng.integers(1, I1, B)
    j[::5] = i[::5]
    return params, U1, I1, d, u, i, j


def test_grad_matches_autograd():
    params, U1, I1, d, u, i, j = _problem()
    G, loss = kbpr_grad(params, U1, d, u, i, j)
    p = torch.tensor(params, dtype=torch.float64, requires_grad=True)
    P, Q = p[: U1 * d].view(U1, d), p[U1 * d:].view(I1, d)
    x = (P[u] * Q[i]).sum(1) - (P[u] * Q[j]).sum(1)
    lt = 1 - torch.log(torch.sigmoid(x))
    lt.mean().backward()
    np.testing.assert_allclose(G, p.grad.numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(loss, lt.detach().numpy(), rtol=1e-6)


def test_epoch_equals_autograd_with_keras_adam():
    """Three batches (the last partial) of the epoch: the restatement vs autograd
    gradients fed to Keras 2.2's Adam update (keras/optimizers.py) in float64."""
    params, U1, I1, d, u, i, j = _problem(3, B=40)
    m, v = np.zeros_like(params), np.zeros_like(params)
    w = params.copy()
    losses = kbpr_epoch(w, m, v, 1, U1, d, u, i, j, 16)
    assert losses.shape == (40,)
    p = torch.tensor(params.astype(np.float64))
    M, V = torch.zeros_like(p), torch.zeros_like(p)
    for t, o in enumerate(range(0, 40, 16), start=1):
        s = slice(o, o + 16)
        q = p.clone().requires_grad_(True)
        P, Q = q[: U1 * d].view(U1, d), q[U1 * d:].view(I1, d)
        x = (P[u[s]] * Q[i[s]]).sum(1) - (P[u[s]] * Q[j[s]]).sum(1)
        (1 - torch.log(torch.sigmoid(x))).mean().backward()
        g = q.grad
        lr_t = 1e-3 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        M = 0.9 * M + 0.1 * g
        V = 0.999 * V + 0.001 * g * g
        p = p - lr_t * M / (torch.sqrt(V) + 1e-7)
    np.testing.assert_allclose(w, p.numpy(), rtol=1e-4, atol=1e-6)
