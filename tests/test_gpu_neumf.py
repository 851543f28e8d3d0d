"""NeuMF / adversarial NeuMF HIP path (libacf_neumf.so) vs the CPU oracle
(oracle/neumf_oracle.py, itself checked against torch autograd in
test_neumf_oracle.py).  Tolerance: fp32, rtol 1e-4 / atol 1e-6 on gradients —
the MLP sums run in a different order than numpy's BLAS.  Parity with the
reference's own adversarial NeuMF is unpinned (it does not run, NeuMF.py:131)."""
import ctypes

import numpy as np
import pytest
import torch

import neumf_oracle as N

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nm(acf):
    import importlib
    from conftest import PKG
    return importlib.import_module(PKG + ".neumf")


def _problem(seed, U1=41, I1=37, d=16, B=96):
    P = N.init_params(U1, I1, d, seed)
    rng = np.random.default_rng(seed + 7)
    u = rng.integers(0, U1, B).astype(np.int32)
    i = rng.integers(0, I1, B).astype(np.int32)
    u[:6] = 5
    i[10:20] = 3
    y = (rng.random(B) < 0.5).astype(np.float32)
    return P, u, i, y


def _state(nm, P, dev):
    U1, d = P["MF_U"].shape
    st = nm.NeuMFState(U1, P["MF_I"].shape[0], d, dev)
    st.load(P)
    return st


@pytest.mark.parametrize("d", [8, 16, 64, 128])
@pytest.mark.parametrize("adver", [0, 1])
def test_grad_matches_oracle(nm, dev, d, adver):
    P, u, i, y = _problem(d + adver, d=d)
    hp_o = N.NeuMFHParams(adver=adver, eps=0.5, reg_adv=0.7)
    want, lc, la = N.grad_step(P, u, i, y, hp_o)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, 256)
    loss = torch.zeros(2, device=dev)
    ctx.grad(u, i, y, ctx.hparams(adver=adver, eps=0.5, reg_adv=0.7), loss)
    torch.cuda.synchronize()
    # rtol 1e-4 on gradients: the weight gradients are split-K sums over the batch
    # (fixed chunk order on the GPU, numpy's pairwise sum in the oracle) of terms
    # that partly cancel, and the MFMA products accumulate in k order
    for n in N.NAMES:
        np.testing.assert_allclose(st.view(n, st.grad).cpu().numpy(), want[n], rtol=1e-4, atol=1e-6,
                                   err_msg=n)
    np.testing.assert_allclose(loss.cpu().numpy(), [lc, la], rtol=1e-5)


def test_predict_matches_oracle(nm, dev):
    P, u, i, _ = _problem(3, d=64, B=1000)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, 64)
    got = ctx.predict(u, i).cpu().numpy()
    np.testing.assert_allclose(got, N.predict(P, u, i), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("adver", [0, 1])
def test_training_steps_match_oracle(nm, dev, adver):
    """Several grad + dense-Adam steps (Keras train_on_batch) track the oracle."""
    P, _, _, _ = _problem(11, d=32)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, 128)
    hp = ctx.hparams(adver=adver, reg_adv=1.0)
    hp_o = N.NeuMFHParams(adver=adver, reg_adv=1.0)
    m = {n: np.zeros_like(P[n]) for n in N.NAMES}
    v = {n: np.zeros_like(P[n]) for n in N.NAMES}
    rng = np.random.default_rng(5)
    for t in range(1, 6):
        u = rng.integers(0, 41, 128).astype(np.int32)
        i = rng.integers(0, 37, 128).astype(np.int32)
        y = (rng.random(128) < 0.5).astype(np.float32)
        g, *_ = N.grad_step(P, u, i, y, hp_o)
        N.adam(P, g, m, v, t, hp_o)
        ctx.grad(u, i, y, hp)
        ctx.adam(hp)
    torch.cuda.synchronize()
    assert float(st.grad.abs().max()) == 0.0  # Adam re-zeroes the gradient
    for n in N.NAMES:  # parameters after Adam steps of those gradients (tolerance as above)
        np.testing.assert_allclose(st.view(n).cpu().numpy(), P[n], rtol=1e-4, atol=2e-6, err_msg=n)


def test_dense_adam_moves_untouched_rows(nm, dev):
    """Keras densifies the embedding gradient: rows outside the batch still move
    once their first moment is non-zero."""
    P, u, i, y = _problem(2, d=16)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, 128)
    hp = ctx.hparams()
    ctx.grad(u[:10], i[:10], y[:10], hp)
    ctx.adam(hp)
    before = st.view("MF_U").clone()
    ctx.grad(u[10:12], i[10:12], y[10:12], hp)
    ctx.adam(hp)
    moved = (st.view("MF_U") != before).any(1).cpu().numpy()
    assert moved[np.setdiff1d(np.unique(u[:10]), u[10:12])].all()


def test_out_of_range_raises(nm, dev):
    from conftest import PKG
    import importlib
    native = importlib.import_module(PKG + "._native")
    P, u, i, y = _problem(4)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, 128)
    u = u.copy()
    u[3] = 41
    with pytest.raises(native.NativeIndexError):
        ctx.grad(u, i, y, ctx.hparams())


def test_recommender_surface(nm, dev):
    """get_train_instances / train / rank as run.py drives them (run.py:242-248)."""
    import scipy.sparse as sp
    rng = np.random.default_rng(0)
    U, I = 60, 80
    train = sp.dok_matrix((U + 1, I + 1), dtype=np.float32)
    for uu in range(1, U + 1):
        for ii in rng.choice(np.arange(1, I + 1), 6, replace=False):
            train[uu, ii] = 1
    for cls, kw in ((nm.NeuMF, {}), (nm.AdversarialNeuMF, {"weight": 1.0, "pop_percent": 0.2})):
        r = cls(U, I, 16, seed=1, device=dev, **kw)
        x, y = r.get_train_instances(train)
        assert len(x[0]) == 2 * train.nnz and y.sum() == train.nnz
        neg = x[1][1::2]
        assert not any((int(a), int(b)) in train for a, b in zip(x[0][1::2], neg))
        losses = [r.train(x, y, 64) for _ in range(30)]
        assert losses[-1] < losses[0]
        s = r.rank(np.full(5, 3), np.arange(1, 6))
        assert s.shape == (5, 1) and np.all((s > 0) & (s < 1))


@pytest.mark.parametrize("B,U1,I1,n,d,calls", [
    (96, 41, 37, 1000, 64, 1),     # every batch re-gathers rows the previous one touched
    (300, 41, 37, 1000, 64, 1),    # 19 weight-gradient slots, summed in three groups
    (16, 500, 300, 640, 16, 2),    # most rows idle for many steps; two calls (t continues)
    (64, 200, 150, 1200, 128, 1),  # a full wave per row
])
def test_train_epoch_equals_stepwise(nm, dev, B, U1, I1, n, d, calls):
    """acf_neumf_train (native batch loop, lazy Adam: batch k's and k+1's rows and
    the MLP at step k, every other row's zero-gradient iterations later in a
    rotating catch-up slice and at the end of the call) == grad + dense adam per
    batch, bit for bit, including the trailing partial batch."""
    P, _, _, _ = _problem(21, U1=U1, I1=I1, d=d)
    rng = np.random.default_rng(9)
    u = rng.integers(0, U1, n).astype(np.int32)
    i = rng.integers(0, I1, n).astype(np.int32)
    y = (rng.random(n) < 0.5).astype(np.float32)
    cut = [0, n] if calls == 1 else [0, (n // B // 2) * B, n]
    for adver in (0, 1):
        a, b = _state(nm, P, dev), _state(nm, P, dev)
        ca, cb = nm.NeuMFContext(a, B), nm.NeuMFContext(b, B)
        hp = ca.hparams(adver=adver)
        la = torch.cat([ca.train(u[c0:c1], i[c0:c1], y[c0:c1], B, hp) for c0, c1 in zip(cut, cut[1:])])
        lb = torch.zeros_like(la)
        k = 0
        for c0, c1 in zip(cut, cut[1:]):
            for o in range(c0, c1, B):
                e = min(o + B, c1)
                cb.grad(u[o:e], i[o:e], y[o:e], hp, lb[k])
                cb.adam(hp)
                k += 1
        torch.cuda.synchronize()
        assert a.t == b.t == k
        assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
        assert torch.equal(la, lb)
        assert not a.grad.any() and not b.grad.any()


def test_neumf_ranker_in_evaluation_protocol(nm, acf, dev):
    """run.py's evaluate_model / evaluate_apr_mode driving the GPU ranker: same
    result as scoring with the oracle's forward (scores agree to ~1e-7; the
    integer-free random parameters make exact ties unlikely)."""
    P = N.init_params(41, 37, 16, 8)
    st = _state(nm, P, dev)

    class R:
        def __init__(self):
            self.ctx = nm.NeuMFContext(st, 64)

        def rank(self, users, items):
            return self.ctx.predict(users, items).cpu().numpy().reshape(-1, 1)

    class O:
        def rank(self, users, items):
            return N.predict(P, np.asarray(users), np.asarray(items)).reshape(-1, 1)

    rng = np.random.default_rng(1)
    test_items = [int(x) for x in rng.integers(1, 37, 40)]
    negs = [list(map(int, rng.integers(1, 37, 20))) for _ in range(40)]
    got = acf.evaluate_model(R(), test_items, negs, 10)
    want = acf.evaluate_model(O(), test_items, negs, 10)
    assert got[0] == want[0]
    ratings = [[u, t] for u, t in enumerate(test_items)]
    assert acf.evaluate_apr_mode(R(), ratings, negs)[0] == acf.evaluate_apr_mode(O(), ratings, negs)[0]


@pytest.mark.parametrize("adver", [0, 1])
def test_yelp_shaped_grad_matches_oracle(nm, dev, adver):
    """The bench's configs[3] shape (yelp-sort-shaped: 25,677 x 25,815 rows, d = 64,
    batch 512) with Zipf-popular items (rows with many occurrences per batch):
    one gradient of the adversarial step vs the oracle, rtol 1e-4 as above."""
    U1, I1, d, B = 25_678, 25_816, 64, 512
    P = N.init_params(U1, I1, d, 17)
    rng = np.random.default_rng(4 + adver)
    u = rng.integers(0, U1, B).astype(np.int32)
    i = ((rng.zipf(1.2, B) - 1) % I1).astype(np.int32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    hp_o = N.NeuMFHParams(adver=adver, eps=0.5, reg_adv=1.0)
    want, lc, la = N.grad_step(P, u, i, y, hp_o)
    st = _state(nm, P, dev)
    ctx = nm.NeuMFContext(st, B)
    loss = torch.zeros(2, device=dev)
    ctx.grad(u, i, y, ctx.hparams(adver=adver, eps=0.5, reg_adv=1.0), loss)
    torch.cuda.synchronize()
    # rtol 1e-4 on gradients: the weight gradients are split-K sums over the batch
    # (fixed chunk order on the GPU, numpy's pairwise sum in the oracle) of terms
    # that partly cancel, and the MFMA products accumulate in k order
    for n in N.NAMES:
        np.testing.assert_allclose(st.view(n, st.grad).cpu().numpy(), want[n], rtol=1e-4, atol=1e-6,
                                   err_msg=n)
    np.testing.assert_allclose(loss.cpu().numpy(), [lc, la], rtol=1e-5)


@pytest.mark.parametrize("B,U1,I1,n,d", [
    (512, 2000, 3000, 1500, 64),   # the bench's batch; Zipf items; a partial last batch (476)
    (1024, 300, 200, 2048, 16),    # the largest rows-in-line batch, rows with many occurrences
    (100, 41, 37, 300, 128),       # d = 128 (weights read from global), partial blocks
])
def test_neumf_rows_in_line_matches_rows_kernel(nm, dev, B, U1, I1, n, d):
    """Batches of <= 1,024 instances sum their rows inside the instance launch
    (each row's first occurrence owns it: its row wave waits for the row's
    arrival count, then adds the write-through contributions in instance order;
    the block's weight-gradient tiles from LDS): one gradient and one train epoch
    equal the k_nmf_rows path's bit for bit (parameters, Adam moments, losses)."""
    P = N.init_params(U1, I1, d, 31)
    rng = np.random.default_rng(13)
    u = rng.integers(0, U1, n).astype(np.int32)
    i = ((rng.zipf(1.3, n) - 1) % I1).astype(np.int32)
    y = (rng.random(n) < 0.5).astype(np.float32)
    for adver in (0, 1):
        a, b = _state(nm, P, dev), _state(nm, P, dev)
        ca, cb = nm.NeuMFContext(a, B), nm.NeuMFContext(b, B)
        cb.set_rows_in_line(False)
        hp = ca.hparams(adver=adver, eps=0.5, reg_adv=0.7)
        la, lb = torch.zeros(2, device=dev), torch.zeros(2, device=dev)
        ca.grad(u[:B], i[:B], y[:B], hp, la)
        cb.grad(u[:B], i[:B], y[:B], hp, lb)
        torch.cuda.synchronize()
        assert a.grad.any()
        assert torch.equal(a.grad, b.grad) and torch.equal(la, lb)
        a.grad.zero_()
        b.grad.zero_()
        ta, tb = ca.train(u, i, y, B, hp), cb.train(u, i, y, B, hp)
        torch.cuda.synchronize()
        assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
        assert torch.equal(ta, tb)


@pytest.mark.parametrize("B,U1,I1,n,d", [(512, 2000, 3000, 1500, 64), (100, 41, 37, 300, 128)])
def test_neumf_give_up_replays_exactly(nm, dev, B, U1, I1, n, d):
    """ Spin limit 0 makes every rows-in-line wait give up at
    once.  With the failsafe on, acf_neumf_train and a checked acf_neumf_grad
    restore what they wrote from their snapshot and replay on the row-sum path:
    the bits of set_rows_in_line(False), one recovery per call, and the context
    is sound afterwards (the stale arrival counters were zeroed: a normal call
    then matches too).  Failsafe off: the give-up raises; an unchecked grad's
    give-up is raised by the next checking call."""
    P = N.init_params(U1, I1, d, 47)
    rng = np.random.default_rng(19)
    u = rng.integers(0, U1, n).astype(np.int32)
    i = ((rng.zipf(1.3, n) - 1) % I1).astype(np.int32)
    y = (rng.random(n) < 0.5).astype(np.float32)
    for adver in (1, 0):
        a, b = _state(nm, P, dev), _state(nm, P, dev)
        ca, cb = nm.NeuMFContext(a, B), nm.NeuMFContext(b, B)
        cb.set_rows_in_line(False)
        hp = ca.hparams(adver=adver, eps=0.5, reg_adv=0.7)
        ca.set_spin_limit(0)
        la, lb = torch.zeros(2, device=dev), torch.zeros(2, device=dev)
        ca.grad(u[:B], i[:B], y[:B], hp, la)
        cb.grad(u[:B], i[:B], y[:B], hp, lb)
        torch.cuda.synchronize()
        assert ca.recoveries() == 1
        assert torch.equal(a.grad, b.grad) and torch.equal(la, lb)
        a.grad.zero_()
        b.grad.zero_()
        ta, tb = ca.train(u, i, y, B, hp), cb.train(u, i, y, B, hp)
        torch.cuda.synchronize()
        assert ca.recoveries() == 2
        assert torch.equal(a.params, b.params) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v)
        assert torch.equal(ta, tb)
        # back to the default limit: the next call runs in line and still matches
        ca.set_spin_limit(1 << 22)
        ta, tb = ca.train(u, i, y, B, hp), cb.train(u, i, y, B, hp)
        torch.cuda.synchronize()
        assert ca.recoveries() == 2
        assert torch.equal(a.params, b.params) and torch.equal(ta, tb)
        # failsafe off: reported, and the context recovers for the next call
        ca.set_failsafe(False)
        ca.set_spin_limit(0)
        with pytest.raises(RuntimeError, match="timed out"):
            ca.train(u, i, y, B, hp)
        # an unchecked grad that gives up is raised by the next checking call
        ca.grad(u[:B], i[:B], y[:B], hp, None, check=False)
        ca.set_spin_limit(1 << 22)
        with pytest.raises(RuntimeError, match="earlier unchecked"):
            ca.predict(u[:8], i[:8])
        ca.predict(u[:8], i[:8])  # reported once
