"""Generate golden fixtures from the REFERENCE's own Python code.

Runs only in the development container, where the reference is mounted at
/root/reference (read-only).  TensorFlow is not installed there, so
``sys.modules['tensorflow']`` is a stub module: Dataset.py, APR.py's sampler
(``sampling`` / ``_get_train_batch``) and utils.py's evaluation
(``_evaluate_input`` / ``_eval_by_user``) never touch TF at run time and execute
as written.  Outputs (data, not source) are committed next to this script:

  video_data.npz          Video.train/test.rating (u, i) columns — the inputs
                          (reference data/; the GPU box has no /root/reference)
  dataset_video.json      OriginalDataset facts: sizes, trainMatrix.keys()
                          order hash, trainList lengths/quirk, testRatings
  dataset_video_lists.npz trainList (CSR) exactly as the reference builds it
  sampler_video.npz       triplets from _get_train_batch (np.random.seed 2019,
                          called in-process instead of through Pool)
  eval_video.npz          _evaluate_input candidates ("sample" mode, exact —
                          Python random seeded 2019) and _eval_by_user outputs
                          (positions, HR/NDCG/AUC) for fixed integer-valued
                          embeddings, "all" and "sample" modes
  published_logs.json     parsed epoch lines / best-epoch tables of the
                          reference's published runs (out/janEval/*.out)

Usage:  python tests/golden/make_reference_fixtures.py
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import re
import sys
import types
from argparse import Namespace

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_reference():
    sys.modules.setdefault("tensorflow", types.ModuleType("tensorflow"))
    sys.path.insert(0, REF)
    import APR  # noqa: E402  (sampler functions; MF needs TF only inside build_graph)
    import Dataset  # noqa: E402
    import utils  # noqa: E402
    return APR, Dataset, utils


def dataset_fixture(Dataset):
    ds = Dataset.OriginalDataset(os.path.join(REF, "data", "Video"))
    keys = np.asarray(list(ds.trainMatrix.keys()), dtype=np.int32)
    lens = np.asarray([len(x) for x in ds.trainList], dtype=np.int32)
    flat = np.asarray([i for x in ds.trainList for i in x], dtype=np.int32)
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    tests = np.asarray(ds.testRatings, dtype=np.int32)
    facts = {
        "num_users": int(ds.num_users), "num_items": int(ds.num_items),
        "n_train_keys": int(len(keys)), "keys_sha256": sha(keys), "keys_head": keys[:50].tolist(),
        "trainList_len": int(len(ds.trainList)), "trainList_lens_sha256": sha(lens),
        "trainList_items_sha256": sha(flat), "testRatings_sha256": sha(tests),
        "df_shape": list(ds.df.shape), "trainSeq_users": int(len(ds.trainSeq)),
    }
    # users absent from the train file, and the list of the uid after each gap
    present = np.zeros(ds.num_users, bool)
    present[keys[:, 0]] = True
    facts["missing_uids"] = np.flatnonzero(~present).tolist()
    np.savez_compressed(os.path.join(HERE, "dataset_video_lists.npz"), off=off, items=flat)
    with open(os.path.join(HERE, "dataset_video.json"), "w") as f:
        json.dump(facts, f, indent=1)
    return ds


def data_fixture():
    tr = np.loadtxt(os.path.join(REF, "data", "Video.train.rating"), dtype=np.int64)
    te = np.loadtxt(os.path.join(REF, "data", "Video.test.rating"), dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "video_data.npz"),
                        train_u=tr[:, 0].astype(np.int32), train_i=tr[:, 1].astype(np.int32),
                        train_r=tr[:, 2].astype(np.int32), test_u=te[:, 0].astype(np.int32),
                        test_i=te[:, 1].astype(np.int32))


def sampler_fixture(APR, ds, n_batches=20, batch_size=512):
    """APR.shuffle's per-batch work (APR.py:39-81) in-process, seeded."""
    np.random.seed(2019)
    samples = APR.sampling(ds)
    APR._user_input, APR._item_input_pos = samples
    APR._batch_size = batch_size
    APR._index = list(range(len(samples[0])))
    APR._model = Namespace(dns=1)
    APR._dataset = ds
    np.random.shuffle(APR._index)
    res = [APR._get_train_batch(b) for b in range(n_batches)]
    u = np.concatenate([r[0][:, 0] for r in res]).astype(np.int32)
    i = np.concatenate([r[1][:, 0] for r in res]).astype(np.int32)
    j = np.concatenate([r[3][:, 0] for r in res]).astype(np.int32)
    su = np.asarray(samples[0][:1000], np.int32)
    si = np.asarray(samples[1][:1000], np.int32)
    np.savez_compressed(os.path.join(HERE, "sampler_video.npz"), user=u, item_pos=i, item_neg=j,
                        batch_size=batch_size, sampling_user_head=su, sampling_item_head=si,
                        n_samples=len(samples[0]))


class _FakeSession:
    """sess.run(model.output, feed) -> P[u] . Q[i] (float32, numpy)."""

    def __init__(self, P, Q):
        self.P, self.Q = P, Q

    def run(self, fetch, feed_dict):
        u = np.asarray(feed_dict["user_input"]).reshape(-1)
        i = np.asarray(feed_dict["item_input_pos"]).reshape(-1)
        return (self.P[u] * self.Q[i]).sum(axis=1, dtype=np.float32).reshape(-1, 1)


def eval_fixture(utils, ds, n_users=300, d=8):
    rng = np.random.default_rng(2019)
    # integer-valued embeddings: every score is exact in fp32, ties are real
    P = rng.integers(-2, 3, (ds.num_users + 1, d)).astype(np.int8)
    Q = rng.integers(-2, 3, (ds.num_items + 1, d)).astype(np.int8)
    users = np.arange(n_users)
    model = Namespace(user_input="user_input", item_input_pos="item_input_pos", output="output",
                      output_adv="output_adv")
    sess = _FakeSession(P.astype(np.float32), Q.astype(np.float32))
    out = {"P": P, "Q": Q, "users": users}
    for mode in ("sample", "all"):
        args = Namespace(eval_mode=mode)
        utils._dataset = ds
        utils._args = args
        utils._candidates = ds.df.iid.tolist()
        feeds = [utils._evaluate_input(int(u)) for u in users]
        utils._model, utils._sess, utils._feed_dicts, utils._output = model, sess, feeds, 0
        utils._K = 100 if mode == "all" else 10
        res = np.asarray([utils._eval_by_user(int(u)) for u in users], dtype=np.float64)
        # the reference's position, recovered from HR@k (first k with a hit - 1)
        hr = res[:, 0, :]
        pos = np.where(hr.any(axis=1), np.argmax(hr > 0, axis=1), -1)
        out[f"{mode}_raw"] = res
        out[f"{mode}_pos_lt_K"] = pos
        out[f"{mode}_auc"] = res[:, 2, 0]
        out[f"{mode}_ncand"] = np.asarray([len(f[1]) - 1 for f in feeds], np.int32)
        if mode == "sample":
            out["sample_cand"] = np.asarray([f[1][:-1, 0] for f in feeds], np.int32)
            out["sample_test"] = np.asarray([f[1][-1, 0] for f in feeds], np.int32)
    np.savez_compressed(os.path.join(HERE, "eval_video.npz"), **out)


_EPOCH = re.compile(r"Epoch (\d+) \[([\d.]+)s \+ ([\d.]+)s\]: HR = ([\d.]+), NDCG = ([\d.]+) "
                    r"ACC = ([\d.]+) ACC_adv = ([\d.]+) \[([\d.]+)s\], \|P\|=([\d.]+), \|Q\|=([\d.]+)")
_BEST = re.compile(r"K = (\d+): HR = ([\d.]+), NDCG = ([\d.]+) AUC = ([\d.]+)")


def logs_fixture():
    runs = {}
    for f in sorted(glob.glob(os.path.join(REF, "out", "janEval", "*_bpr_*.out")) +
                    glob.glob(os.path.join(REF, "out", "janEval", "*_apr_*.out"))):
        name = os.path.basename(f)
        epochs, best, best_epoch = [], [], None
        for line in open(f):
            m = _EPOCH.search(line)
            if m:
                g = m.groups()
                epochs.append({"epoch": int(g[0]), "batch_s": float(g[1]), "train_s": float(g[2]),
                               "hr": float(g[3]), "ndcg": float(g[4]), "acc": float(g[5]),
                               "acc_adv": float(g[6]), "eval_s": float(g[7]), "normP": float(g[8]),
                               "normQ": float(g[9])})
            m = _BEST.search(line)
            if m:
                best.append([int(m.group(1)), float(m.group(2)), float(m.group(3)), float(m.group(4))])
            m = re.search(r"Epoch (\d+) is the best epoch", line)
            if m:
                best_epoch = int(m.group(1))
        runs[name] = {"epochs": epochs, "best_epoch": best_epoch, "best": best,
                      "apr_switch": "Initialize APR" in open(f).read()}
    with open(os.path.join(HERE, "published_logs.json"), "w") as f:
        json.dump(runs, f)


def main():
    APR, Dataset, utils = load_reference()
    data_fixture()
    ds = dataset_fixture(Dataset)
    sampler_fixture(APR, ds)
    eval_fixture(utils, ds)
    logs_fixture()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
