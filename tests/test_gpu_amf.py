"""FastAdversarialMF (FastAdversarialMF.py:13-144, run.py --model amf2) on the GPU
(libacf_neumf.so acf_amf_*) against oracle/amf_oracle.py, and run.py end to end.
Parity with the reference itself is unpinned (it does not run: DESIGN.md §11)."""
import ctypes
import glob
import importlib
import os

import numpy as np
import pytest
import torch

import amf_oracle as A
from conftest import PKG

pytestmark = pytest.mark.gpu


def _inst(seed, uNum, iNum, n):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, uNum, n).astype(np.int32)
    i = rng.integers(0, iNum, n).astype(np.int32)
    u[::7] = u[0]                          # a hot user: many occurrences per batch
    ua = rng.integers(0, uNum, n).astype(np.int32)
    ua[::5] = u[::5][: len(ua[::5])]       # rows gathered by both the MSE and the discriminator
    ia = rng.integers(0, iNum, n).astype(np.int32)
    y = rng.integers(0, 2, n).astype(np.float32)
    tu = rng.integers(0, 2, n).astype(np.float32)
    ti = rng.integers(0, 2, n).astype(np.float32)
    return [u, i, y, ua, ia, tu, ti, (1 - tu).astype(np.float32), (1 - ti).astype(np.float32)]


def _model(uNum, iNum, d, dev, seed=1):
    FM = importlib.import_module(PKG + ".fast_adversarial_mf").FastAdversarialMF
    r = FM(uNum, iNum, d, seed=seed, device=dev)
    buf = A.init_params(uNum, iNum, d, seed)
    r.params.copy_(torch.as_tensor(buf))
    return r, buf


@pytest.mark.parametrize("d,B", [(8, 64), (64, 512), (32, 37)])
def test_batch_gradient_matches_oracle(dev, d, B):
    uNum, iNum = 50, 40
    r, buf = _model(uNum, iNum, d, dev)
    inst = _inst(d, uNum, iNum, B)
    u, i, y, ua, ia, tu, ti, du, di = inst
    T = lambda x: torch.as_tensor(x).to(dev)
    loss = r.grad_batch(T(u), T(i), T(y), T(ua), T(ia), T(tu), T(ti), T(du), T(di))
    G, want_loss, parts = A.grad_step(buf, uNum, iNum, d, u, i, y, ua, ia, tu, ti, du, di)
    np.testing.assert_allclose(r.grad.cpu().numpy(), G, rtol=1e-4, atol=1e-7)
    got = loss.double().mean(0).cpu().numpy()
    np.testing.assert_allclose(got, parts, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("d", [16, 64])
def test_train_batches_match_oracle(dev, d):
    """acf_amf_train over 6 batches (the last one partial) vs the oracle's epoch:
    weights and both Adam moments."""
    uNum, iNum, B, n = 60, 45, 100, 560
    r, buf = _model(uNum, iNum, d, dev, seed=2)
    inst = _inst(100 + d, uNum, iNum, n)
    T = [torch.as_tensor(x).to(dev).contiguous() for x in inst]
    losses = torch.empty(n, 3, device=dev)
    ctx = r._context(B)
    nat = importlib.import_module(PKG + "._native")
    nat.call_neumf("acf_amf_train", ctx, r.params.data_ptr(), r.grad.data_ptr(), r.m.data_ptr(), r.v.data_ptr(),
                   *[t.data_ptr() for t in T], n, B, 1, ctypes.byref(r.hp), losses.data_ptr(),
                   torch.cuda.current_stream().cuda_stream)
    m, v = np.zeros_like(buf), np.zeros_like(buf)
    want = A.train_epoch(buf, m, v, 1, uNum, iNum, d, inst, B)
    np.testing.assert_allclose(r.params.cpu().numpy(), buf, rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(r.m.cpu().numpy(), m, rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(r.v.cpu().numpy(), v, rtol=1e-4, atol=1e-12)
    got = [float(losses[o: o + B].double().sum(1).mean()) for o in range(0, n, B)]
    np.testing.assert_allclose(got, want, rtol=1e-5)
    assert not r.grad.any()  # Adam re-zeroes the gradient


def test_out_of_range_raises(dev):
    uNum, iNum, d = 20, 10, 8
    r, _ = _model(uNum, iNum, d, dev)
    inst = _inst(0, uNum, iNum, 16)
    inst[4][3] = iNum  # an item_adv index past the table
    T = [torch.as_tensor(x).to(dev) for x in inst]
    nat = importlib.import_module(PKG + "._native")
    with pytest.raises(nat.NativeIndexError):
        r.grad_batch(*T)


def test_recommender_surface(dev):
    """get_train_instances (MF.py:42-56) / init / train / rank / save / load as
    run.py drives them."""
    import scipy.sparse as sp
    FM = importlib.import_module(PKG + ".fast_adversarial_mf").FastAdversarialMF
    rng = np.random.default_rng(3)
    uNum, iNum = 80, 60
    train = sp.dok_matrix((uNum, iNum), dtype=np.float32)
    for u in range(1, uNum):
        for it in rng.choice(np.arange(1, iNum), 6, replace=False):
            train[u, int(it)] = 1.0
    r = FM(uNum, iNum, 16, weight=0.5, pop_percent=0.2, seed=0, device=dev)
    (us, its), y = r.get_train_instances(train)
    assert len(us) == 2 * train.nnz and set(np.unique(y)) == {0, 1}
    assert all((int(a), int(b)) not in train for a, b in zip(us[y == 0], its[y == 0]))
    l0 = r.train([us, its], y, 64)
    l1 = r.train([us, its], y, 64)
    assert np.isfinite(l0) and np.isfinite(l1) and r.t == 2 * ((len(y) + 63) // 64)
    sc = r.rank(us[:20], its[:20]).reshape(-1)
    P, Q = r.uEmb.cpu().numpy(), r.iEmb.cpu().numpy()
    np.testing.assert_allclose(sc, (P[us[:20]] * Q[its[:20]]).sum(1), rtol=1e-5, atol=1e-6)


def test_run_py_amf2_end_to_end(tmp_path, dev):
    rc = importlib.import_module(PKG + ".run_cli")
    path = str(tmp_path) + "/"
    res = rc.main(["--path", path, "--opath", "t/", "--model", "amf2", "--data", "synthetic:300:200:6000",
                   "--d", "16", "--epochs", "3", "--bs", "256", "--eval", "all"], device=dev)
    out = glob.glob(os.path.join(path, "out", "t", "*.out"))
    assert len(out) == 1
    lines = open(out[0]).read().splitlines()
    its = [ln for ln in lines if ln.startswith("Iteration ")]
    assert len(its) == 3 and lines[-1].startswith("End. Best Iteration")
    assert all(np.isfinite(float(ln.split("loss = ")[1].split(" ")[0])) for ln in its)
    assert "amf2_d16_w" in res["runName"]
    assert glob.glob(os.path.join(path, "h5", "*.last.h5.npz"))
