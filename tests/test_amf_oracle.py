"""oracle/amf_oracle.py (FastAdversarialMF, FastAdversarialMF.py:13-144) against
torch-CPU autograd of the same three player losses; the popularity split against
the reference's get_discriminator_train_data rule (dict order, stable sort,
reversed)."""
import numpy as np
import torch

import amf_oracle as A


def _batch(seed, uNum=30, iNum=25, d=8, B=24):
    rng = np.random.default_rng(seed)
    buf = A.init_params(uNum, iNum, d, seed)
    u = rng.integers(0, uNum, B)
    i = rng.integers(0, iNum, B)
    u[::5] = u[0]  # repeated rows: occurrence sums
    ua = rng.integers(0, uNum, B)
    ua[1] = u[2]   # a row both gathered for the MSE and for the discriminator
    ia = rng.integers(0, iNum, B)
    y = rng.integers(0, 2, B).astype(np.float32)
    tu = np.r_[np.ones(B // 2), np.zeros(B - B // 2)].astype(np.float32)
    ti = tu.copy()
    return buf, uNum, iNum, d, u, i, y, ua, ia, tu, ti, tu[::-1].copy(), ti[::-1].copy()


def _autograd(buf, uNum, iNum, d, u, i, y, ua, ia, tu, ti, du, di):
    t = torch.tensor(buf.astype(np.float64), requires_grad=True)
    P = t[: uNum * d].view(uNum, d)
    Q = t[uNum * d: (uNum + iNum) * d].view(iNum, d)
    o = (uNum + iNum) * d
    blk = A.disc_block(d)
    discs = []
    for k in range(2):
        s = o + k * blk
        discs.append((t[s: s + d * d].view(d, d), t[s + d * d: s + d * d + d], t[s + d * d + d: s + d * d + 2 * d],
                      t[s + d * d + 2 * d]))
    tt = lambda x: torch.tensor(np.asarray(x, np.float64))
    B = len(u)
    mse = ((P[u] * Q[i]).sum(1) - tt(y)) ** 2

    def disc(D, e):
        W1, b1, W2, b2 = D
        return torch.sigmoid(torch.relu(e @ W1 + b1) @ W2 + b2)

    def bce(s, target):
        sc = s.clamp(1e-7, 1 - 1e-7)
        return -(target * sc.log() + (1 - target) * (1 - sc).log())

    # mf player: embeddings see every term, discriminators frozen
    Dfix = [tuple(x.detach() for x in D) for D in discs]
    loss_mf = mse.mean() + bce(disc(Dfix[0], P[ua]), tt(tu)).mean() + bce(disc(Dfix[1], Q[ia]), tt(ti)).mean()
    g_mf = torch.autograd.grad(loss_mf, t)[0]
    g_du = torch.autograd.grad(bce(disc(discs[0], P[ua].detach()), tt(du)).mean(), t)[0]
    g_di = torch.autograd.grad(bce(disc(discs[1], Q[ia].detach()), tt(di)).mean(), t)[0]
    G = g_mf.clone()
    G[o: o + blk] = g_du[o: o + blk]
    G[o + blk: o + 2 * blk] = g_di[o + blk: o + 2 * blk]
    return G.numpy(), float(loss_mf)


def test_grad_step_matches_autograd():
    for seed in range(3):
        args = _batch(seed)
        G, loss, parts = A.grad_step(*args)
        W, wl = _autograd(*args)
        np.testing.assert_allclose(G, W, rtol=1e-4, atol=1e-8)
        assert abs(loss - wl) < 1e-5 and len(parts) == 3


def test_train_epoch_moves_every_player():
    buf, uNum, iNum, d, *inst = _batch(7)
    b0 = buf.copy()
    m, v = np.zeros_like(buf), np.zeros_like(buf)
    losses = A.train_epoch(buf, m, v, 1, uNum, iNum, d, [np.asarray(x) for x in inst], 10)
    assert len(losses) == 3 and all(np.isfinite(losses))
    P, Q, Du, Di = A.unflatten(buf, uNum, iNum, d)
    P0, Q0, Du0, Di0 = A.unflatten(b0, uNum, iNum, d)
    assert not np.array_equal(P, P0) and not np.array_equal(Q, Q0)
    for D, D0 in ((Du, Du0), (Di, Di0)):
        assert not np.array_equal(D["W1"], D0["W1"]) and not np.array_equal(D["W2"], D0["W2"])


def test_popularity_split_follows_reference_rule():
    x = [5, 3, 3, 9, 5, 7, 7, 2, 3]  # counts: 3->3, 5->2, 7->2, 9->1, 2->1; first seen 5,3,9,7,2
    pop, rare = A.popularity_split(x, 0.4)
    popularity = {}
    for k in x:
        popularity[k] = popularity.get(k, 0) + 1
    ranked = list({k: v for k, v in sorted(popularity.items(), key=lambda kv: kv[1])[::-1]}.keys())
    assert list(pop) + list(rare) == ranked
    assert list(pop) == ranked[: int(len(ranked) * 0.4)]
