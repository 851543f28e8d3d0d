"""Keras BPR (BPR.py:23-99, run.py --model bpr, BASELINE configs[0]) on the GPU
(libacf_neumf.so acf_kbpr_*) vs the CPU restatement (oracle/kbpr_oracle.py),
and run.py end to end."""
import glob
import importlib
import os

import numpy as np
import pytest
import torch

from conftest import PKG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,batch", [(32, 512), (64, 100), (8, 37)])
def test_epoch_matches_oracle(dev, d, batch):
    from kbpr_oracle import kbpr_epoch
    KB = importlib.import_module(PKG + ".keras_bpr")
    U1, I1, n = 400, 300, 2300
    rng = np.random.default_rng(d)
    u = rng.integers(1, U1, n).astype(np.int32)
    i = (rng.zipf(1.3, n) % (I1 - 1) + 1).astype(np.int32)  # hot items: many occurrences per batch
    j = rng.integers(1, I1, n).astype(np.int32)
    j[::11] = i[::11]
    r = KB.BPR(U1, I1, d, seed=3, device=dev)
    w0 = r.params.cpu().numpy().copy()
    r._rng = np.random.RandomState(5)  # no shuffle difference: the oracle gets the same order
    perm = np.random.RandomState(5).permutation(n)
    loss = r.train([u, i, j], np.ones(n), batch)
    m, v = np.zeros_like(w0), np.zeros_like(w0)
    want_l = kbpr_epoch(w0, m, v, 1, U1, d, u[perm], i[perm], j[perm], batch)
    got = r.params.cpu().numpy()
    np.testing.assert_allclose(got, w0, rtol=1e-5, atol=2e-6)
    # Adam's first moments are 0.1 x a gradient of 1/B-scaled terms: tiny values whose
    # relative error reflects the gradient's last-bit differences (summation order)
    np.testing.assert_allclose(r.m.cpu().numpy(), m, rtol=1e-4, atol=1e-9)
    assert abs(loss - float(want_l.astype(np.float64).mean())) < 1e-5
    assert r.t == (n + batch - 1) // batch
    sc = r.rank(u[:50], i[:50]).reshape(-1)
    P, Q = got[: U1 * d].reshape(U1, d), got[U1 * d:].reshape(I1, d)
    np.testing.assert_allclose(sc, (P[u[:50]] * Q[i[:50]]).sum(1), rtol=1e-5, atol=1e-6)


def test_run_py_bpr_end_to_end(tmp_path, dev):
    """run.py --model bpr --d 32 on a small synthetic ml-1m-like set: the .out log
    lines of run.py, checkpoints, and HR@100 above the random init."""
    rc = importlib.import_module(PKG + ".run_cli")
    path = str(tmp_path) + "/"
    res = rc.main(["--path", path, "--opath", "t/", "--model", "bpr", "--data", "synthetic:400:300:12000",
                   "--d", "32", "--epochs", "6", "--bs", "256", "--eval", "all"], device=dev)
    out = glob.glob(os.path.join(path, "out", "t", "*.out"))
    assert len(out) == 1
    lines = open(out[0]).read().splitlines()
    assert lines[0].startswith("Load data done") and lines[2].startswith("Init: HR = ")
    assert sum(ln.startswith("Iteration ") for ln in lines) == 6 and lines[-1].startswith("End. Best Iteration")
    init_hr = float(lines[2].split("HR = ")[1].split(",")[0])
    assert res["best_hr"] > init_hr + 0.05
    assert glob.glob(os.path.join(path, "h5", "*.last.h5.npz"))
