"""BASELINE configs[0] at its stated workload: ``run.py --model bpr --data ml-1m
--d 32`` (run.py:25-280, BPR.py:23-99) on ml-1m-shaped synthetic data (6,040 x
3,706, ~994k training pairs), batch 512 (run.py's --bs default).

* the Keras BPR on the GPU (keras_bpr.BPR -> acf_kbpr_* in libacf_neumf.so) vs the
  CPU restatement (oracle/kbpr_oracle.py) batch by batch for 32 batches, the
  oracle in lockstep (free-running: neither side is re-synchronised);
* run.py's driver end to end at that size (run_cli.main), "all" evaluation.
"""
import glob
import importlib
import os

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import PKG

pytestmark = pytest.mark.gpu
D, BS, NBATCH = 32, 512, 32


def _ml1m_train():
    acf = importlib.import_module(PKG)
    ds = acf.ml1m_like(seed=2019)
    u = np.asarray(ds.pair_user, np.int64) + 1  # run.py's datasets are 1-based (0 = masking id)
    i = np.asarray(ds.pair_item, np.int64) + 1
    uNum, iNum = ds.num_users + 1, ds.num_items + 1
    train = sp.coo_matrix((np.ones(len(u), np.float32), (u, i)), shape=(uNum, iNum))
    return train, uNum, iNum


def test_kbpr_ml1m_batches_match_oracle(dev):
    from kbpr_oracle import kbpr_epoch
    KB = importlib.import_module(PKG + ".keras_bpr")
    train, uNum, iNum = _ml1m_train()
    assert (uNum, iNum) == (6041, 3707) and train.nnz > 990_000
    r = KB.BPR(uNum, iNum, D, seed=3, device=dev)
    (u, i, j), _ = r.get_train_instances(train)
    assert len(u) == train.nnz
    sel = np.random.default_rng(0).permutation(len(u))[: NBATCH * BS]
    u, i, j = u[sel], i[sel], j[sel]
    w = r.params.cpu().numpy().copy()
    m, v = np.zeros_like(w), np.zeros_like(w)
    for k in range(NBATCH):
        s = slice(k * BS, (k + 1) * BS)
        r._rng = np.random.RandomState(100 + k)  # train()'s shuffle, replayed for the oracle
        perm = np.random.RandomState(100 + k).permutation(BS)
        loss = r.train([u[s], i[s], j[s]], np.ones(BS), BS)
        want_l = kbpr_epoch(w, m, v, k + 1, uNum, D, u[s][perm], i[s][perm], j[s][perm], BS)
        np.testing.assert_allclose(r.params.cpu().numpy(), w, rtol=1e-5, atol=2e-6, err_msg=f"weights, batch {k}")
        assert abs(loss - float(want_l.astype(np.float64).mean())) < 1e-5, f"loss, batch {k}"
    assert r.t == NBATCH
    # Adam moments after 32 batches (tests/test_gpu_keras_bpr.py: the first moments are
    # 0.1 x 1/B-scaled gradients, their last bits follow the summation order)
    np.testing.assert_allclose(r.m.cpu().numpy(), m, rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(r.v.cpu().numpy(), v, rtol=1e-4, atol=1e-12)


def test_run_py_bpr_ml1m_end_to_end(tmp_path, dev):
    """run.py --model bpr --data ml-1m --d 32 (configs[0]) at the ml-1m shape: two
    full epochs (1,942 batches each, the last partial batch kept), all-items
    evaluation (K = 100) before and after each epoch, the .out log, checkpoints."""
    rc = importlib.import_module(PKG + ".run_cli")
    path = str(tmp_path) + "/"
    res = rc.main(["--path", path, "--opath", "t/", "--model", "bpr", "--data", "ml-1m-synthetic",
                   "--d", "32", "--epochs", "2", "--bs", "512", "--eval", "all"], device=dev)
    out = glob.glob(os.path.join(path, "out", "t", "*.out"))
    assert len(out) == 1
    lines = open(out[0]).read().splitlines()
    assert lines[0].startswith("Load data done") and "#user=6041, #item=3707" in lines[0]
    assert lines[2].startswith("Init: HR = ")
    its = [ln for ln in lines if ln.startswith("Iteration ")]
    assert len(its) == 2 and lines[-1].startswith("End. Best Iteration")
    init_hr = float(lines[2].split("HR = ")[1].split(",")[0])
    losses = [float(ln.split("loss = ")[1].split(" ")[0]) for ln in its]
    assert all(np.isfinite(losses)) and losses[1] < losses[0]
    assert res["best_hr"] > init_hr + 0.02
    assert glob.glob(os.path.join(path, "h5", "*.last.h5.npz"))
