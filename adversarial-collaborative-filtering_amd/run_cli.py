"""Drop-in for the reference's ``run.py`` (run.py:25-280): the Keras-style
``Recommender`` driver, for the models on the MI355X build's path.

    python run.py --model bpr --data ml-1m-synthetic --d 32 --epochs 10 --eval all

Same flags (run.py:25-75) and the same loop: ``getDataset``, the ranker,
``Init`` evaluation, per epoch ``get_train_instances`` -> ``train`` ->
``evaluate_model`` every ``verbose_eval`` epochs, best-NDCG tracking with
``.hr`` / ``.ndcg`` files and ``.best`` / ``.last`` checkpoints, the ``.out``
log lines of run.py:117-119,215-280.  Models: ``bpr`` (the Keras BPR of
BPR.py:23-99, BASELINE configs[0]), ``apr`` / ``bpr-tf`` (the APR graph,
switching to the adversarial model at ``--adv_epochs``, run.py:157-161,233-236),
``neumf`` / ``aneumf`` (NeuMF.py:10-55), ``amf2`` (FastAdversarialMF.py:13-144).
The others (SASRec, Caser, GRU4Rec, DRCF, DREAM, APL, IRGAN, the
discriminator-adversarial MF/BPR of MF.py / BPR.py and the naive baselines) are
out of scope and rejected.

Datasets (``getDataset``, utils.py:44-78): the reference's ``Dataset`` class
(Dataset.py:59-107) cannot run (``df = df.sort_values(..., inplace=True)`` binds
None), so its intended semantics are implemented here on the loaders this build
has (``data.get_dataset``: rating-file prefixes and the synthetic shapes):
ids shifted to start at 1 (0 is the masking id), the leave-one-out test item,
``testNegatives`` = every item the user never trained on except 0 and the test
item (``--eval all``) or 100 popularity-weighted draws, Python ``random``
seeded 2019 (``--eval sample``); top-K 100 / 10 (run.py:105).
"""
from __future__ import annotations

import argparse
import math
import os
import random
from datetime import datetime
from time import time

import numpy as np

OUT_OF_SCOPE = {"mf", "amf", "abpr", "apl", "irgan", "sasrec", "drcf", "gru4rec", "dream", "dream-tf",
                "caser", "pop", "mrv", "mfv", "av"}


def parse_args(argv=None):
    """run.py:25-75."""
    p = argparse.ArgumentParser(description="Run Adversarial Collaborative Filtering")
    p.add_argument("--path", type=str, help="Path to data", default="")
    p.add_argument("--opath", type=str, help="Path to output", default="test/")
    p.add_argument("--model", type=str, help="Model Name: lstm", default="bpr")
    p.add_argument("--data", type=str, help="Dataset name", default="test")
    p.add_argument("--d", type=int, default=64, help="Dimension")
    p.add_argument("--verbose_eval", type=int, default=1, help="Evaluate per X epochs.")
    p.add_argument("--eval", type=str, default="all", help="DRCF evaluation mode or APR evaluation mode")
    p.add_argument("--maxlen", type=int, default=10, help="Maxlen")
    p.add_argument("--epochs", type=int, default=10, help="Epoch number")
    p.add_argument("--adv_epochs", type=int, default=5, help="Adversarial Epoch number")
    p.add_argument("--w", type=float, default=0.001, help="Weight:")
    p.add_argument("--pp", type=float, default=0.2, help="Popularity Percentage:")
    p.add_argument("--bs", type=int, default=512, help="Batch Size:")
    p.add_argument("--pre", type=str, default="", help="Pre-trained dir:")
    p.add_argument("--mode", type=int, default=0, help="mode")
    p.add_argument("--ckpt", type=int, default=1, help="Save the model per X epochs.")
    p.add_argument("--save_model", type=int, default=1, help="Save model")
    p.add_argument("--seed", type=int, default=0, help="(MI355X build) seed of init and sampling")
    return p.parse_args(argv)


class RunDataset:
    """What run.py reads from getDataset(...) (run.py:111-114): trainMatrix (dok,
    1-based ids), trainSeq, df, testRatings (indexable by user, entry 0 unused),
    testNegatives."""

    def __init__(self, base, eval_mode="all"):
        import pandas as pd
        import scipy.sparse as sp
        u = np.asarray(base.pair_user, np.int64) + 1
        i = np.asarray(base.pair_item, np.int64) + 1
        self.num_users, self.num_items = int(base.num_users) + 1, int(base.num_items) + 1
        self.df = pd.DataFrame({"uid": u, "iid": i})
        mat = sp.coo_matrix((np.ones(len(u), np.float32), (u, i)), shape=(self.num_users, self.num_items)).todok()
        self.trainMatrix = mat
        seq = {}
        for a, b in zip(u.tolist(), i.tolist()):
            seq.setdefault(a, []).append(b)
        self.trainSeq = seq
        tests = {int(k) + 1: int(t) + 1 for k, t in base.testRatings}
        self.testRatings = [None] + [tests.get(x, 0) for x in range(1, self.num_users)]
        self.testNegatives = [[]] * self.num_users
        if eval_mode == "all":
            every = np.arange(1, self.num_items)
            for x in range(1, self.num_users):
                keep = np.ones(self.num_items, bool)
                keep[0] = False
                keep[np.asarray(seq.get(x, []), np.int64)] = False
                keep[self.testRatings[x]] = False
                self.testNegatives[x] = every[keep[1:]].tolist()
        else:
            random.seed(2019)
            cand = i.tolist()
            for x in range(1, self.num_users):
                negs = []
                own = set(seq.get(x, []))
                for _ in range(100):
                    r = random.choice(cand)
                    while r in own or r == self.testRatings[x]:
                        r = random.choice(cand)
                    negs.append(r)
                self.testNegatives[x] = negs


def get_dataset(data, path, eval_mode, seed=2019):
    """utils.getDataset (utils.py:44-78) on this build's loaders."""
    from .data import get_dataset as base_dataset
    return RunDataset(base_dataset(data, path, seed=seed), eval_mode)


def make_ranker(name, uNum, iNum, dim, args, device=None):
    if name in OUT_OF_SCOPE:
        raise SystemExit(f"--model {name}: outside the MI355X build's scope (DESIGN.md §10); "
                         "supported: bpr, apr, bpr-tf, neumf, aneumf, amf2")
    if name == "bpr":
        from .keras_bpr import BPR
        return BPR(uNum, iNum, dim, seed=args.seed, device=device)
    if name in ("apr", "bpr-tf"):
        from .recommender import APR
        return APR(uNum, iNum, dim, False, seed=args.seed, device=device)
    if name == "neumf":
        from .neumf import NeuMF
        return NeuMF(uNum, iNum, dim, seed=args.seed, device=device)
    if name == "aneumf":
        from .neumf import AdversarialNeuMF
        return AdversarialNeuMF(uNum, iNum, dim, args.w, args.pp, seed=args.seed, device=device)
    if name == "amf2":  # run.py:140-141
        from .fast_adversarial_mf import FastAdversarialMF
        return FastAdversarialMF(uNum, iNum, dim, args.w, args.pp, seed=args.seed, device=device)
    raise SystemExit(f"--model {name}: unknown model")


def main(argv=None, device=None):
    from .evaluation import evaluate_model
    from .train import prediction2file, write2file
    args = parse_args(argv)
    path, opath, data, modelName, dim = args.path, args.opath, args.data, args.model, args.d
    batch_size, epochs, adv_epochs = args.bs, args.epochs, args.adv_epochs
    pre, evalMode, verbose_eval = args.pre, args.eval, args.verbose_eval
    save_model = args.save_model == 1
    topK = 100 if evalMode == "all" else 10
    t1 = time()
    dataset = get_dataset(data, path, evalMode)
    train, testRatings, testNegatives = dataset.trainMatrix, dataset.testRatings, dataset.testNegatives
    uNum, iNum = dataset.num_users, dataset.num_items
    stat = "Load data done [%.1f s]. #user=%d, #item=%d, #train=%d, #test=%d" % (
        time() - t1, uNum, iNum, len(dataset.df), len(testRatings) - 1)
    ranker = make_ranker(modelName, uNum, iNum, dim, args, device)
    runName = "%s_%s_d%d%s_%s" % (data, modelName, dim, ranker.get_params(),
                                  datetime.now().strftime("%m-%d-%Y_%H-%M-%S"))
    if modelName in ("apr", "bpr-tf"):
        ranker.build_graph(path, opath, data, runName)
    saveName = "%s_%s_d%d%s" % (data, modelName, dim, ranker.get_params())
    if pre != "":
        ranker.load_pre_train(path + "h5/" + pre)
        runName = "%s_%s_%s.%s_d%d_%s" % (data, modelName, pre.split("_")[1], pre.split(".")[1], dim,
                                          datetime.now().strftime("%m-%d-%Y_%H-%M-%S"))
    out = path + "out/" + opath
    if save_model:
        os.makedirs(path + "h5/", exist_ok=True)
    write2file(out, runName + ".out", stat)
    write2file(out, runName + ".out", runName)
    if pre != "":
        write2file(out, runName + ".out", pre)
    hits, ndcgs = evaluate_model(ranker, testRatings, testNegatives, topK, 1)
    hr, ndcg = np.array(hits).mean(), np.array(ndcgs).mean()
    write2file(out, runName + ".out", "Init: HR = %f, NDCG = %f" % (hr, ndcg))
    best_hr, best_ndcg, best_iter = hr, ndcg, -1
    start = time()
    for epoch in range(epochs):
        if modelName == "apr" and epoch == adv_epochs:  # run.py:233-236
            from .recommender import APR
            prev = ranker
            ranker = APR(uNum, iNum, dim, True, seed=args.seed, device=device)
            ranker.build_graph(path, opath, data, runName, True, previous=prev)
        t1 = time()
        x_train, y_train = ranker.get_train_instances(train)
        loss = ranker.train(x_train, y_train, batch_size)
        t2 = time()
        if epoch % verbose_eval == 0:
            hits, ndcgs = evaluate_model(ranker, testRatings, testNegatives, topK, 1)
            hr, ndcg = np.array(hits).mean(), np.array(ndcgs).mean()
        write2file(out, runName + ".out", "Iteration %d [%.1f s]: HR = %f, NDCG = %f, loss = %.4f [%.1f s]" % (
            epoch, t2 - t1, hr, ndcg, loss, time() - t2))
        if ndcg > best_ndcg:
            best_hr, best_ndcg, best_iter = hr, ndcg, epoch
            if save_model:
                ranker.save(path + "h5/" + saveName + ".best.h5")
            prediction2file(out, runName + ".hr", hits)
            prediction2file(out, runName + ".ndcg", ndcgs)
        if math.isnan(loss):
            break
        if save_model:
            ranker.save(path + "h5/" + saveName + ".last.h5")
    write2file(out, runName + ".out", "End. Best Iteration %d:  HR = %.4f, NDCG = %.4f, Total time = %.2f" % (
        best_iter, best_hr, best_ndcg, (time() - start) / 3600))
    return {"best_iter": best_iter, "best_hr": float(best_hr), "best_ndcg": float(best_ndcg), "runName": runName}
