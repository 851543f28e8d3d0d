"""The NeuMF oracle (oracle/neumf_oracle.py) against torch-CPU autograd (float64)
of the same graph: gradients of the clean and the adversarial objective, the
delta, and the Keras Adam update.  Parity with the reference's own adversarial
NeuMF is unpinned (it does not run: NeuMF.py:131); the clean NeuMF graph follows
NeuMF.py:10-52."""
import numpy as np
import pytest
import torch

import neumf_oracle as N

U1, I1, D, B = 23, 19, 8, 40


def _problem(seed):
    P = N.init_params(U1, I1, D, seed)
    rng = np.random.default_rng(seed + 1)
    u = rng.integers(0, U1, B)
    i = rng.integers(0, I1, B)
    u[:5] = 3  # duplicated rows
    i[3:9] = 7
    y = (rng.random(B) < 0.5).astype(np.float32)
    return P, u, i, y


def _torch_grads(P, u, i, y, hp):
    T = {n: torch.tensor(P[n], dtype=torch.float64, requires_grad=True) for n in N.NAMES}
    ut, it = torch.tensor(u), torch.tensor(i)
    yt = torch.tensor(y, dtype=torch.float64)

    def loss_fn(delta=None):
        mu, mi, lu, li = T["MF_U"][ut], T["MF_I"][it], T["MLP_U"][ut], T["MLP_I"][it]
        if delta is not None:
            mu, mi, lu, li = mu + delta["MF_U"], mi + delta["MF_I"], lu + delta["MLP_U"], li + delta["MLP_I"]
        a1 = torch.relu(torch.cat([lu, li], 1) @ T["W1"] + T["b1"])
        a2 = torch.relu(a1 @ T["W2"] + T["b2"])
        p = torch.sigmoid(torch.cat([mu * mi, a2], 1) @ T["Wo"] + T["bo"])[:, 0]
        pc = torch.clamp(p, 1e-7, 1 - 1e-7)
        return -(yt * torch.log(pc) + (1 - yt) * torch.log(1 - pc)).mean()

    lc = loss_fn()
    total = lc
    if hp.adver:
        tabs = ("MF_U", "MF_I", "MLP_U", "MLP_I")
        G = torch.autograd.grad(lc, [T[n] for n in tabs], retain_graph=True)
        delta = {}
        for n, g in zip(tabs, G):
            idx = ut if n.endswith("_U") else it
            r = g[idx]
            delta[n] = (hp.eps * r / torch.sqrt(torch.clamp((r * r).sum(1, keepdim=True), min=1e-12))).detach()
        total = lc + hp.reg_adv * loss_fn(delta)
    grads = torch.autograd.grad(total, [T[n] for n in N.NAMES])
    return {n: g.numpy() for n, g in zip(N.NAMES, grads)}, float(lc)


@pytest.mark.parametrize("adver", [0, 1])
def test_oracle_grads_match_autograd(adver):
    P, u, i, y = _problem(3 + adver)
    hp = N.NeuMFHParams(adver=adver, eps=0.5, reg_adv=1.0)
    g, lc, la = N.grad_step(P, u, i, y, hp)
    want, lc_t = _torch_grads(P, u, i, y, hp)
    assert abs(lc - lc_t) < 1e-5
    for n in N.NAMES:
        np.testing.assert_allclose(g[n], want[n], rtol=2e-4, atol=2e-7, err_msg=n)
    if adver:
        assert la > 0


def test_untouched_rows_have_zero_gradient():
    P, u, i, y = _problem(5)
    g, *_ = N.grad_step(P, u, i, y, N.NeuMFHParams(adver=1))
    untouched = np.setdiff1d(np.arange(U1), u)
    assert np.all(g["MF_U"][untouched] == 0) and np.all(g["MLP_U"][untouched] == 0)


def test_adam_matches_keras_formula():
    """Keras 2.2 Adam: lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t); dense update, so a
    parameter with zero gradient still moves when its moment is non-zero."""
    hp = N.NeuMFHParams()
    P = {n: np.ones(s, np.float32) for n, s in N.shapes(3, 3, 4).items()}
    m = {n: np.zeros_like(P[n]) for n in N.NAMES}
    v = {n: np.zeros_like(P[n]) for n in N.NAMES}
    g = {n: np.full_like(P[n], 0.5) for n in N.NAMES}
    N.adam(P, g, m, v, 1, hp)
    lr_t = 0.001 * np.sqrt(1 - 0.999) / (1 - 0.9)
    want = 1 - lr_t * (0.1 * 0.5) / (np.sqrt(0.001 * 0.25) + 1e-7)
    np.testing.assert_allclose(P["W1"], want, rtol=1e-6)
    g0 = {n: np.zeros_like(P[n]) for n in N.NAMES}
    before = P["W1"].copy()
    N.adam(P, g0, m, v, 2, hp)
    assert np.all(P["W1"] < before)  # momentum keeps moving it
