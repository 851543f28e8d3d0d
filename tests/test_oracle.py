"""The CPU oracle, pinned: golden vectors, two independent restatements of the
TF graph, and the reference's own evaluation outputs (tests/golden/)."""
import os

import numpy as np
import pytest
import torch

from apr_oracle import HParams, eval_metrics, tf_graph_step
from conftest import GOLDEN


def _rand_problem(seed, U1, I1, d, B, nb, scale=0.2, dup=True):
    rng = np.random.default_rng(seed)
    P = (rng.standard_normal((U1, d)) * scale).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * scale).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    if dup:
        j[::9] = i[::9]
    return P, Q, u, i, j


def test_golden_vectors(oracle):
    """tests/golden/oracle_tiny.npz (make_oracle_fixtures.py) reproduces."""
    z = np.load(os.path.join(GOLDEN, "oracle_tiny.npz"))
    cases = sorted({k.rsplit("_", 1)[0] for k in z.files if k.endswith("_P0")})
    assert len(cases) == 8
    for c in cases:
        d, adver, reg = c.split("_")
        hp = HParams(adver=int(adver[1:]), reg=float(reg[1:]))
        P, Q = z[c + "_P0"].copy(), z[c + "_Q0"].copy()
        aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
        u, i, j = z[c + "_u"], z[c + "_i"], z[c + "_j"]
        B = 32
        losses = []
        for t in range(len(u) // B):
            s = slice(t * B, (t + 1) * B)
            lc, _, dP, dQ = oracle.apr_batch(P, Q, aP, aQ, u[s], i[s], j[s], hp, want_delta=True)
            losses.append(lc)
            if hp.adver:
                np.testing.assert_allclose(dP, z[f"{c}_dP{t}"], rtol=1e-6, atol=1e-8)
                np.testing.assert_allclose(dQ, z[f"{c}_dQ{t}"], rtol=1e-6, atol=1e-8)
        for name, got in (("P", P), ("Q", Q), ("accP", aP), ("accQ", aQ)):
            np.testing.assert_allclose(got, z[f"{c}_{name}"], rtol=1e-6, atol=1e-8, err_msg=f"{c} {name}")
        np.testing.assert_allclose(np.concatenate(losses), z[c + "_loss_clean"], rtol=1e-6)


@pytest.mark.parametrize("adver", [0, 1])
@pytest.mark.parametrize("reg", [0.0, 0.05])
@pytest.mark.parametrize("d", [4, 16, 64])
def test_c_oracle_matches_dense_tf_graph(oracle, adver, reg, d):
    """Row-set C restatement == dense numpy evaluation of the TF graph."""
    P, Q, u, i, j = _rand_problem(d + 7 * adver, 37, 29, d, 40, 3)
    hp = HParams(adver=adver, reg=reg)
    a = [P.copy(), Q.copy(), np.full_like(P, 0.1), np.full_like(Q, 0.1)]
    b = [x.copy() for x in a]
    for t in range(3):
        s = slice(t * 40, (t + 1) * 40)
        lc, la, dP, dQ = oracle.apr_batch(*a, u[s], i[s], j[s], hp, want_delta=True)
        tlc, tla, tdP, tdQ = tf_graph_step(*b, u[s], i[s], j[s], hp)
        np.testing.assert_allclose(lc, tlc, rtol=1e-6)
        if adver:
            np.testing.assert_allclose(la, tla, rtol=1e-5)
            np.testing.assert_allclose(dP, tdP, rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(dQ, tdQ, rtol=1e-5, atol=1e-7)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-7)


def torch_autograd_step(P, Q, aP, aQ, u, i, j, hp):
    """The TF graph written with torch ops; every gradient from autograd."""
    f32 = torch.float32
    Pt = torch.tensor(P, dtype=f32, requires_grad=True)
    Qt = torch.tensor(Q, dtype=f32, requires_grad=True)
    ut, it, jt = (torch.tensor(x, dtype=torch.long) for x in (u, i, j))
    B, d = len(u), P.shape[1]

    def bpr(Pm, Qm, dP=None, dQ=None):
        p, qi, qj = Pm[ut], Qm[it], Qm[jt]
        if dP is not None:
            p, qi, qj = p + dP[ut], qi + dQ[it], qj + dQ[jt]
        x = (p * qi).sum(1) - (p * qj).sum(1)
        r = torch.clamp(x, hp.clip_lo, hp.clip_hi)
        return torch.nn.functional.softplus(-r).sum()

    loss = bpr(Pt, Qt)
    dP = dQ = None
    if hp.adver:
        gP, gQ = torch.autograd.grad(loss, [Pt, Qt], retain_graph=True)
        nP = torch.rsqrt(torch.clamp((gP * gP).sum(1, keepdim=True), min=1e-12))
        nQ = torch.rsqrt(torch.clamp((gQ * gQ).sum(1, keepdim=True), min=1e-12))
        dP, dQ = (gP * nP * hp.eps).detach(), (gQ * nQ * hp.eps).detach()
    reg_term = hp.reg * ((Pt[ut] ** 2 + Qt[it] ** 2 + Qt[jt] ** 2).mean())
    opt = loss + reg_term
    if hp.adver:
        opt = opt + hp.reg_adv * bpr(Pt, Qt, dP, dQ) + reg_term
    GP, GQ = torch.autograd.grad(opt, [Pt, Qt])
    out = []
    for W, A, G, rows in ((P, aP, GP.numpy(), np.unique(u)), (Q, aQ, GQ.numpy(), np.unique(np.r_[i, j]))):
        A[rows] = A[rows] + G[rows] ** 2
        W[rows] = W[rows] - hp.lr * G[rows] / np.sqrt(A[rows])
        out.append(W)
    return dP, dQ


@pytest.mark.parametrize("adver", [0, 1])
@pytest.mark.parametrize("reg", [0.0, 0.02])
def test_c_oracle_matches_torch_autograd(oracle, adver, reg):
    """Hand-derived gradients (Appendix A) == autograd of the same graph."""
    P, Q, u, i, j = _rand_problem(50 + adver, 31, 23, 32, 48, 2)
    hp = HParams(adver=adver, reg=reg)
    a = [P.copy(), Q.copy(), np.full_like(P, 0.1), np.full_like(Q, 0.1)]
    b = [x.copy() for x in a]
    for t in range(2):
        s = slice(t * 48, (t + 1) * 48)
        _, _, dP, dQ = oracle.apr_batch(*a, u[s], i[s], j[s], hp, want_delta=True)
        tdP, tdQ = torch_autograd_step(*b, u[s], i[s], j[s], hp)
        if adver:
            np.testing.assert_allclose(dP, tdP.numpy(), rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(dQ, tdQ.numpy(), rtol=1e-4, atol=1e-6)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)


def test_dense_mode_equals_sparse_mode(oracle):
    P, Q, u, i, j = _rand_problem(3, 80, 60, 16, 64, 3)
    hp = HParams(adver=1)
    a = [P.copy(), Q.copy(), np.full_like(P, 0.1), np.full_like(Q, 0.1)]
    b = [x.copy() for x in a]
    oracle.apr_train(*a, u, i, j, 64, hp, dense=False)
    oracle.apr_train(*b, u, i, j, 64, hp, dense=True)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_i_equals_j_cancels_exactly(oracle):
    """A user whose only triplet has i == j gets gradient 0 and delta 0 (TF sums
    rounded products, so +g*q - g*q is exactly 0)."""
    P = np.full((3, 8), 0.3, np.float32)
    Q = np.linspace(-1, 1, 40, dtype=np.float32).reshape(5, 8)
    u = np.array([1], np.int32)
    i = np.array([2], np.int32)
    P0 = P.copy()
    _, _, dP, dQ = oracle.apr_batch(P, Q, np.full_like(P, .1), np.full_like(Q, .1), u, i, i,
                                    HParams(adver=1), want_delta=True)
    assert np.all(dP == 0) and np.all(dQ == 0)
    np.testing.assert_array_equal(P, P0)


def test_out_of_range_rejected(oracle):
    P = np.zeros((4, 8), np.float32)
    Q = np.zeros((4, 8), np.float32)
    with pytest.raises(ValueError):
        oracle.apr_batch(P, Q, P + .1, Q + .1, np.array([4], np.int32), np.array([0], np.int32),
                         np.array([1], np.int32), HParams())


def test_forward_and_metrics(oracle):
    P, Q, u, i, j = _rand_problem(9, 20, 15, 8, 10, 4, dup=False)
    bl, bc, op, on = oracle.bpr_forward(P, Q, u, i, j, 10)
    x = (P[u] * Q[i]).sum(1) - (P[u] * Q[j]).sum(1)
    np.testing.assert_allclose(op - on, x, rtol=1e-5, atol=1e-6)
    assert np.array_equal(bc, (x.reshape(4, 10) > 0).sum(1))
    hr, ndcg, auc = eval_metrics([0, 3, 150], [100, 100, 200], 10)
    assert hr[0].sum() == 10 and hr[1].sum() == 7 and hr[2].sum() == 0
    assert ndcg[0, 0] == 1.0 and np.isclose(ndcg[1, 9], np.log(2) / np.log(5))
    assert np.isclose(auc[2, 0], 1 - 150 / 200)


# --- pinned by the reference's own evaluation code (tests/golden/eval_video.npz) ----
def _ref_eval():
    z = np.load(os.path.join(GOLDEN, "eval_video.npz"))
    lists = np.load(os.path.join(GOLDEN, "dataset_video_lists.npz"))
    data = np.load(os.path.join(GOLDEN, "video_data.npz"))
    return z, lists, data


def _ref_positions(z, mode):
    """position = #(neg >= pos): exact from AUC = 1 - position / ncand."""
    return np.rint((1.0 - z[f"{mode}_auc"]) * z[f"{mode}_ncand"]).astype(np.int64)


def test_oracle_eval_matches_reference_all_mode(oracle):
    z, lists, data = _ref_eval()
    P, Q = z["P"].astype(np.float32), z["Q"].astype(np.float32)
    users = z["users"].astype(np.int32)
    num_items = 23714
    tests = data["test_i"][users].astype(np.int32)
    off, items = lists["off"], lists["items"]
    ex = [np.unique(np.r_[items[off[u]:off[u + 1]], tests[k]]) for k, u in enumerate(users)]
    ex = [e[e < num_items].astype(np.int32) for e in ex]
    eo = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(e) for e in ex], out=eo[1:])
    pos = oracle.eval_positions_all(P, Q, users, tests, num_items, eo, np.concatenate(ex))
    np.testing.assert_array_equal(pos, _ref_positions(z, "all"))
    np.testing.assert_array_equal(num_items - np.diff(eo), z["all_ncand"])


def test_oracle_eval_matches_reference_sample_mode(oracle):
    z, _, _ = _ref_eval()
    P, Q = z["P"].astype(np.float32), z["Q"].astype(np.float32)
    users = z["users"].astype(np.int32)
    cand = z["sample_cand"]
    co = np.arange(0, cand.size + 1, cand.shape[1], dtype=np.int64)
    pos = oracle.eval_positions_list(P, Q, users, z["sample_test"], co, cand.reshape(-1))
    np.testing.assert_array_equal(pos, _ref_positions(z, "sample"))
    hr, ndcg, auc = eval_metrics(pos, z["sample_ncand"], 10)
    np.testing.assert_allclose(np.stack([hr, ndcg, auc], 1), z["sample_raw"], rtol=1e-12)


def test_random_delta_mode(oracle):
    """adv = "random" (APR.py:170-177): every touched row's delta has norm eps and
    untouched rows stay 0; the draw depends on (seed, call, batch) and not on the
    gradient; the components look like a normalised N(0,1) sample (mean ~0,
    variance ~eps^2/d)."""
    rng = np.random.default_rng(0)
    U1, I1, d, B = 300, 200, 64, 256
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u, i, j = (rng.integers(0, N, B).astype(np.int32) for N in (U1, I1, I1))

    def draw(**kw):
        hp = HParams(adver=1, adv="random", seed=5, **kw)
        tabs = [P.copy(), Q.copy(), np.full(P.shape, 0.1, np.float32), np.full(Q.shape, 0.1, np.float32)]
        _, _, dP, dQ = oracle.apr_batch(*tabs, u, i, j, hp, want_delta=True)
        return dP, dQ

    dP, dQ = draw(call=1, t=0)
    touched = np.zeros(U1, bool)
    touched[u] = True
    np.testing.assert_allclose(np.linalg.norm(dP[touched], axis=1), 0.5, rtol=1e-5)
    assert not dP[~touched].any()
    np.testing.assert_allclose(np.linalg.norm(dQ[np.unique(np.concatenate([i, j]))], axis=1), 0.5, rtol=1e-5)
    for kw in (dict(call=2, t=0), dict(call=1, t=1)):
        assert not np.array_equal(draw(**kw)[0][touched], dP[touched])
    np.testing.assert_array_equal(draw(call=1, t=0)[0], dP)  # deterministic
    x = dP[touched].ravel()
    assert abs(x.mean()) < 0.01 and abs(x.var() - 0.25 / d) < 0.1 * 0.25 / d


@pytest.mark.parametrize("adver,dense", [(0, True), (1, True), (1, False)])
def test_torch_cpu_baseline_matches_c_oracle(oracle, adver, dense):
    """oracle/apr_torch_cpu.py (the multi-threaded CPU baseline) computes the same
    steps as the C oracle, to fp32 rounding."""
    import torch
    from apr_torch_cpu import apr_step
    rng = np.random.default_rng(7)
    U1, I1, d, B, nb = 120, 90, 32, 64, 4
    P = (rng.standard_normal((U1, d)) * 0.3).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.3).astype(np.float32)
    u, i, j = (rng.integers(0, N, nb * B).astype(np.int32) for N in (U1, I1, I1))
    rP, rQ = P.copy(), Q.copy()
    aP, aQ = np.full(P.shape, 0.1, np.float32), np.full(Q.shape, 0.1, np.float32)
    oracle.apr_train(rP, rQ, aP, aQ, u, i, j, B, HParams(adver=adver))
    tabs = [torch.tensor(P), torch.tensor(Q), torch.full(P.shape, 0.1), torch.full(Q.shape, 0.1)]
    for t in range(nb):
        s = slice(t * B, (t + 1) * B)
        apr_step(*tabs, torch.tensor(u[s]).long(), torch.tensor(i[s]).long(), torch.tensor(j[s]).long(),
                 adver=bool(adver), dense=dense)
    for g, w in zip(tabs, (rP, rQ, aP, aQ)):
        np.testing.assert_allclose(g.numpy(), w, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("adver,reg,dense,adv,threads", [(1, 0.0, True, "grad", 8), (1, 0.01, False, "grad", 3),
                                                         (0, 0.01, True, "grad", 5), (1, 0.0, False, "random", 4)])
def test_threaded_oracle_bit_identical(oracle, adver, reg, dense, adv, threads):
    """oracle_apr_train_mt (bench.py's CPU baseline on every host core, VERDICT
    r05 #7) gives the bits of the one-thread oracle_apr_train: per-triplet terms
    split by triplet, per-row sums split by row slot in occurrence order, a hot
    row and i == j triplets included."""
    rng = np.random.default_rng(11 + adver)
    U1, I1, d, B, nb = 61, 53, 16, 64, 6
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    i[::5] = 7
    j[::9] = i[::9]
    hp = HParams(adver=adver, reg=reg, adv=adv, seed=3)
    outs = []
    for mt in (False, True):
        t = [P.copy(), Q.copy(), np.full_like(P, 0.1), np.full_like(Q, 0.1)]
        if mt:
            assert oracle.apr_train_mt(*t, u, i, j, B, hp, dense=dense, threads=threads) == threads
        else:
            oracle.apr_train(*t, u, i, j, B, hp, dense=dense)
        outs.append(t)
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
