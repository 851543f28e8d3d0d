"""Drop-in surface: CLI flags and defaults (run_adv_ori.py:17-64,
run_adv.py:15-54), the Recommender ABC (Recommender.py:3-27), MF attributes
(APR.py:86-97) and log/checkpoint formats (utils.py:18-32,95-97)."""
import importlib
import os
from argparse import Namespace

import numpy as np
import pytest

from conftest import PKG

# flag -> default, transcribed from the reference scripts
RUN_ADV_ORI = {"path": "", "opath": "aaa/", "dataset": "fsq11-sort", "model": "pop", "verbose": 1,
               "batch_size": 512, "epochs": 10, "adv_epoch": 0, "embed_size": 64, "dns": 1, "reg": 0,
               "lr": 0.05, "reg_adv": 1, "restore": None, "ckpt": 10, "task": "", "adv": "grad",
               "eps": 0.5, "eps_dense": 0.5, "eps_conv": 0.5, "eps_pos": 0.5, "eval_mode": "sample"}
RUN_ADV = {"path": "", "opath": "aaa/", "model": "apr", "dataset": "ml-1m", "verbose": 1,
           "batch_size": 512, "epochs": 2, "adv_epoch": 1, "embed_size": 64, "dns": 1, "reg": 0,
           "lr": 0.05, "reg_adv": 1, "restore": None, "ckpt": 1, "task": "", "adv": "grad", "eps": 0.5}


@pytest.fixture(scope="module")
def cli():
    return importlib.import_module(PKG + ".cli")


@pytest.mark.parametrize("flavor,table", [("ori", RUN_ADV_ORI), ("adv", RUN_ADV)])
def test_flag_defaults(cli, flavor, table):
    a = vars(cli.parse_args([], flavor))
    for k, v in table.items():
        assert a[k] == v, k


def test_flags_parse_like_the_published_runs(cli):
    a = cli.parse_args("--model apr --dataset ml-1m-sort --epochs 2000 --adv_epoch 1000 --verbose 20 "
                       "--eval_mode all --embed_size 64".split(), "ori")
    assert (a.model, a.epochs, a.adv_epoch, a.eval_mode, a.embed_size) == ("apr", 2000, 1000, "all", 64)


def test_recommender_abc(acf):
    abstract = set(acf.Recommender.__abstractmethods__)
    assert abstract == {"get_params", "load_pre_train", "save", "train", "rank", "get_train_instances"}
    assert issubclass(acf.APR, acf.Recommender)
    r = acf.APR(10, 12, 8, adver=True)
    assert r.get_params() == "_e0.50_l1.00"


def test_mf_attributes(acf):
    args = Namespace(embed_size=16, lr=0.05, reg=0.0, dns=1, adv="grad", eps=0.5, adver=1, reg_adv=1.0,
                     epochs=3)
    m = acf.MF(100, 50, args)
    for k, v in dict(num_users=100, num_items=50, embedding_size=16, learning_rate=0.05, reg=0.0, dns=1,
                     adv="grad", eps=0.5, adver=1, reg_adv=1.0, epochs=3).items():
        assert getattr(m, k) == v


def test_write2file_and_prediction2file(acf, tmp_path):
    p = str(tmp_path) + "/out/"
    acf.write2file(p, "run.out", "Epoch 0 [1.0s + 2.0s]: HR = 0.1000")
    acf.write2file(p, "run.out", "line2")
    assert open(p + "run.out").read() == "Epoch 0 [1.0s + 2.0s]: HR = 0.1000\nline2\n"
    acf.prediction2file(p, "run.hr", np.array([1.0, 0.0]))
    assert open(p + "run.hr").read() == "1.000000\n0.000000\n"


def test_checkpoint_roundtrip_format(tmp_path):
    train = importlib.import_module(PKG + ".train")
    args = Namespace(adver=0, dataset="ds", embed_size=8, restore=None)
    save, restore = train.ckpt_dirs(args, "TS")
    assert save == "Pretrain/ds/MF_BPR/embed_8/TS/" and restore == 0
    args.adver = 1
    save, restore = train.ckpt_dirs(args, "TS")
    assert save == "Pretrain/ds/APR/embed_8/TS/" and restore == "Pretrain/ds/MF_BPR/embed_8/TS/"

    class M:  # minimal model with the two checkpointed tensors
        import torch
        embedding_P = torch.arange(12.).reshape(3, 4)
        embedding_Q = torch.ones(2, 4)

    path = train.save_checkpoint(M, str(tmp_path), 7)
    assert train.latest_checkpoint(str(tmp_path)) == path
    z = np.load(path + ".npz")
    assert set(z.files) == {"embedding_P", "embedding_Q"}


# --- run.py (run.py:25-280): the Keras-style Recommender driver -------------------
def _run_cli():
    import importlib
    return importlib.import_module(PKG + ".run_cli")


def test_run_py_flags_match_reference_defaults():
    a = _run_cli().parse_args([])
    assert (a.path, a.opath, a.model, a.data, a.d, a.verbose_eval, a.eval, a.maxlen, a.epochs, a.adv_epochs,
            a.w, a.pp, a.bs, a.pre, a.mode, a.ckpt, a.save_model) == (
        "", "test/", "bpr", "test", 64, 1, "all", 10, 10, 5, 0.001, 0.2, 512, "", 0, 1, 1)


def test_run_py_dataset_semantics():
    """1-based ids (0 = masking id), leave-one-out test item, all-mode negatives =
    every item but 0, the user's train items and the test item; sample mode 100
    draws outside the user's items."""
    rc = _run_cli()
    ds = rc.get_dataset("synthetic:60:45:1300", "", "all")
    assert ds.testRatings[0] is None and len(ds.testRatings) == ds.num_users == 61
    seq = ds.trainSeq
    for u in (1, 7, 60):
        negs = set(ds.testNegatives[u])
        assert 0 not in negs and ds.testRatings[u] not in negs and not negs & set(seq[u])
        assert negs | set(seq[u]) | {ds.testRatings[u], 0} == set(range(ds.num_items))
        assert (u, seq[u][0]) in ds.trainMatrix
    sm = rc.get_dataset("synthetic:60:45:1300", "", "sample")
    for u in (1, 30):
        assert len(sm.testNegatives[u]) == 100 and not set(sm.testNegatives[u]) & set(seq[u])


def test_run_py_rejects_out_of_scope_models():
    import pytest
    rc = _run_cli()
    with pytest.raises(SystemExit, match="scope"):
        rc.make_ranker("sasrec", 10, 10, 8, rc.parse_args([]))
