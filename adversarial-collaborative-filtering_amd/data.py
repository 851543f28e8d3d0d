"""Triplet-source datasets.

:class:`OriginalDataset` is a drop-in for ``Dataset.OriginalDataset``
(``Dataset.py:226-327``), the loader behind every published APR log: same
attributes (``trainMatrix``, ``trainList``, ``testRatings``, ``num_users``,
``num_items``, ``df``, ``trainSeq``) with the same values, including the
``trainList`` misalignment of ``Dataset.py:306-327`` (a uid missing from the
train file shifts the next user's first item into the missing uid's list).  The
arrays the GPU path needs (positive pairs, per-user sorted lists) are built once
with numpy; the scipy ``dok_matrix`` is only materialised on first access.

:func:`synthetic_dataset` generates the ml-1m / pinterest-shaped data that the
benchmarks use: user degree >= 20, heavy-tailed; Zipf item
popularity; leave-one-out test item per user; seeded.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

ML1M_SHAPE = dict(num_users=6040, num_items=3706, n_train=994169)
PINTEREST_SHAPE = dict(num_users=55187, num_items=9916, n_train=1445622)
# yelp-sort: 25,677 users (the test file), 25,815 items and 730,791 ratings in the
# public release, one held out per user (train file absent here)
YELP_SHAPE = dict(num_users=25677, num_items=25815, n_train=705114, min_degree=10)


class _DatasetBase:
    """Shared array views.  Subclasses set pair_user/pair_item (positive pairs in
    ``trainMatrix.keys()`` order), list_off/list_items (trainList, CSR) and
    test_items."""

    num_users: int
    num_items: int
    pair_user: np.ndarray
    pair_item: np.ndarray
    test_items: np.ndarray

    # --- per-user sorted unique lists (for samplers / eval exclusion) -------
    def sorted_lists(self):
        """CSR (offsets int64, items int32) of sorted unique trainList[u]."""
        if getattr(self, "_sorted_csr", None) is None:
            off, items = self.list_off, self.list_items
            owner = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
            key = np.unique(owner * (np.int64(items.max(initial=0)) + 1) + items)
            stride = np.int64(items.max(initial=0)) + 1
            own = key // stride
            cnt = np.bincount(own, minlength=len(off) - 1)
            soff = np.zeros(len(off), dtype=np.int64)
            np.cumsum(cnt, out=soff[1:])
            self._sorted_csr = (soff, (key % stride).astype(np.int32))
        return self._sorted_csr

    def trainlist_len(self) -> int:
        return len(self.list_off) - 1


class OriginalDataset(_DatasetBase):
    """Drop-in for Dataset.OriginalDataset(path) (Dataset.py:235-252)."""

    def __init__(self, path: str):
        import pandas as pd

        train = self._read(path + ".train.rating")
        u, i, rating = train[:, 0].astype(np.int64), train[:, 1].astype(np.int64), train[:, 2]
        # num_users/num_items = max id + 1 over every line (Dataset.py:284-294)
        self.num_users = int(u.max()) + 1 if len(u) else 1
        self.num_items = int(i.max()) + 1 if len(i) else 1
        # trainMatrix keys: rating > 0, first-insertion order (dok dict order)
        keep = rating > 0
        key = u[keep] * self.num_items + i[keep]
        _, first = np.unique(key, return_index=True)
        first.sort()
        self.pair_user = u[keep][first].astype(np.int32)
        self.pair_item = i[keep][first].astype(np.int32)
        self.list_off, self.list_items = self._train_lists(u, i)
        test = self._read(path + ".test.rating")
        self.testRatings = [[int(a), int(b)] for a, b in zip(test[:, 0], test[:, 1])]
        self.test_items = test[:, 1].astype(np.int32)
        names = ["uid", "iid", "rating", "timestamp"]
        self.df = pd.read_csv(path + ".train.rating", sep="\t", names=names)
        self._trainMatrix = None
        self._trainList = None
        self._trainSeq = None
        self._sorted_csr = None

    @staticmethod
    def _read(fname: str) -> np.ndarray:
        import pandas as pd
        a = pd.read_csv(fname, sep="\t", header=None, usecols=[0, 1, 2], dtype=np.float64).to_numpy()
        return a.reshape(-1, 3)

    @staticmethod
    def _train_lists(u: np.ndarray, i: np.ndarray):
        """Dataset.py:306-327 verbatim semantics: the list index advances by ONE
        per line on which the uid exceeds it."""
        n = len(u)
        bounds = []  # line index at which a new list starts
        u_ = 0
        uu = u.tolist()
        for x in range(n):
            if u_ < uu[x]:
                bounds.append(x)
                u_ += 1
        off = np.zeros(len(bounds) + 2, dtype=np.int64)
        off[1:-1] = bounds
        off[-1] = n
        return off, i.astype(np.int32)

    # --- reference attributes ------------------------------------------------
    @property
    def trainList(self):
        if self._trainList is None:
            self._trainList = [self.list_items[self.list_off[k]:self.list_off[k + 1]].tolist()
                               for k in range(len(self.list_off) - 1)]
        return self._trainList

    @property
    def trainMatrix(self):
        if self._trainMatrix is None:
            import scipy.sparse as sp
            mat = sp.dok_matrix((self.num_users, self.num_items), dtype=np.float32)
            for a, b in zip(self.pair_user.tolist(), self.pair_item.tolist()):
                mat[a, b] = 1.0
            self._trainMatrix = mat
        return self._trainMatrix

    @property
    def trainSeq(self):
        if self._trainSeq is None:
            seq = defaultdict(list)
            for a, b in zip(self.df["uid"].tolist(), self.df["iid"].tolist()):
                seq[a].append(b)
            self._trainSeq = seq
        return self._trainSeq


class SyntheticDataset(_DatasetBase):
    """Generated dataset with the OriginalDataset API (contiguous users, so the
    trainList quirk is a no-op)."""

    def __init__(self, num_users, num_items, pair_user, pair_item, test_items, name="synthetic"):
        self.name = name
        self.num_users = int(num_users)
        self.num_items = int(num_items)
        self.pair_user = pair_user.astype(np.int32)
        self.pair_item = pair_item.astype(np.int32)
        self.test_items = test_items.astype(np.int32)
        cnt = np.bincount(self.pair_user, minlength=self.num_users)
        self.list_off = np.zeros(self.num_users + 1, dtype=np.int64)
        np.cumsum(cnt, out=self.list_off[1:])
        self.list_items = self.pair_item
        self.testRatings = [[k, int(t)] for k, t in enumerate(self.test_items.tolist())]
        self._sorted_csr = None
        self._df = None

    @property
    def df(self):
        if self._df is None:
            import pandas as pd
            self._df = pd.DataFrame({"uid": self.pair_user, "iid": self.pair_item,
                                     "rating": np.ones(len(self.pair_user), np.int32),
                                     "timestamp": np.arange(len(self.pair_user))})
        return self._df

    @property
    def trainList(self):
        return [self.list_items[self.list_off[k]:self.list_off[k + 1]].tolist()
                for k in range(self.num_users)]

    @property
    def trainMatrix(self):
        import scipy.sparse as sp
        mat = sp.dok_matrix((self.num_users, self.num_items), dtype=np.float32)
        for a, b in zip(self.pair_user.tolist(), self.pair_item.tolist()):
            mat[a, b] = 1.0
        return mat


def synthetic_dataset(num_users: int, num_items: int, n_train: int, seed: int = 2019,
                      min_degree: int = 20, zipf_s: float = 1.0, sigma: float = 1.1,
                      name: str = "synthetic") -> SyntheticDataset:
    """Heavy-tailed user degrees (>= min_degree, mean n_train/num_users), Zipf item
    popularity, one held-out test item per user; pairs sorted by user like the
    reference's *.train.rating files."""
    rng = np.random.default_rng(seed)
    mean_extra = max(n_train / num_users - min_degree, 1.0)
    raw = rng.lognormal(mean=np.log(mean_extra) - sigma * sigma / 2, sigma=sigma, size=num_users)
    deg = min_degree + np.floor(raw).astype(np.int64)
    cap = max(min_degree + 1, int(0.62 * num_items))  # ml-1m: max degree 2,314 of 3,706 items
    deg = np.minimum(deg, cap)
    # rescale to hit n_train exactly (keeping the minimum)
    extra = deg - min_degree
    target_extra = n_train - min_degree * num_users
    if extra.sum() > 0 and target_extra > 0:
        extra = np.floor(extra * (target_extra / extra.sum())).astype(np.int64)
        short = target_extra - extra.sum()
        idx = rng.choice(num_users, size=int(abs(short)), replace=True)
        np.add.at(extra, idx, 1 if short > 0 else 0)
    deg = np.minimum(min_degree + extra, cap)
    # item popularity: Zipf over a random permutation of item ids
    ranks = np.arange(1, num_items + 1, dtype=np.float64)
    pop = ranks ** (-zipf_s)
    pop = pop[rng.permutation(num_items)]
    logw = np.log(pop)
    users, items, tests = [], [], np.empty(num_users, dtype=np.int64)
    chunk = max(1, (1 << 22) // num_items)
    for u0 in range(0, num_users, chunk):
        u1 = min(num_users, u0 + chunk)
        # Efraimidis-Spirakis weighted sampling without replacement (Gumbel top-k)
        keys = logw[None, :] + rng.gumbel(size=(u1 - u0, num_items))
        kmax = int(deg[u0:u1].max()) + 1
        top = np.argpartition(-keys, kmax - 1, axis=1)[:, :kmax]
        order = np.take_along_axis(keys, top, axis=1).argsort(axis=1)[:, ::-1]
        top = np.take_along_axis(top, order, axis=1)
        for r in range(u1 - u0):
            k = int(deg[u0 + r])
            sel = top[r, :k + 1]
            tests[u0 + r] = sel[k]          # the held-out (last) interaction
            perm = rng.permutation(k)
            users.append(np.full(k, u0 + r, dtype=np.int64))
            items.append(sel[:k][perm])
    pu = np.concatenate(users)
    pi = np.concatenate(items)
    return SyntheticDataset(num_users, num_items, pu, pi, tests, name=name)


class DeviceDataset:
    """A dataset that lives only in device memory (config 5: 10M users x 5M items,
    ~200M interactions; host copies would cost minutes): positive pairs sorted
    by user, trainList as a sorted CSR.  Enough of the OriginalDataset surface for
    DeviceSampler (num_users, num_items, device_arrays())."""

    def __init__(self, num_users, num_items, pos_user, pos_item, list_off, list_items, name="synthetic-large"):
        self.name = name
        self.num_users, self.num_items = int(num_users), int(num_items)
        self.pos_user, self.pos_item = pos_user, pos_item
        self.list_off, self.list_items = list_off, list_items

    def device_arrays(self):
        """(pos_user int32, pos_item int32, list_off int64, list_items int32), on device."""
        return self.pos_user, self.pos_item, self.list_off, self.list_items

    def __len__(self):
        return int(self.pos_user.numel())


def synthetic_large(num_users: int = 10_000_000, num_items: int = 5_000_000, per_user: int = 20,
                    zipf_s: float = 1.0, seed: int = 2019, device="cuda") -> DeviceDataset:
    """BASELINE config 5 / SURVEY §8(d) "synthetic large": per_user interactions
    per user (~20, 200M in all), items drawn from a Zipf(zipf_s) popularity over a
    random permutation of the ids, generated on the device (torch, seeded).  Each
    user's list is sorted (the sampler's rejection set); repeats are kept, as a
    rating file may hold them."""
    import torch
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    n = num_users * per_user
    cdf = torch.arange(1, num_items + 1, device=dev, dtype=torch.float64).pow_(-zipf_s).cumsum_(0)
    cdf /= cdf[-1].clone()
    perm = torch.randperm(num_items, device=dev, generator=g).to(torch.int32)
    items = torch.empty(n, dtype=torch.int32, device=dev)
    step = 1 << 24
    for a in range(0, n, step):
        b = min(n, a + step)
        r = torch.rand(b - a, device=dev, dtype=torch.float64, generator=g)
        items[a:b] = perm[torch.searchsorted(cdf, r).clamp_(max=num_items - 1)]
    del cdf, perm
    items = items.view(num_users, per_user).sort(dim=1).values.reshape(-1).contiguous()
    users = torch.arange(num_users, device=dev, dtype=torch.int32).repeat_interleave(per_user)
    off = torch.arange(0, n + 1, per_user, device=dev, dtype=torch.int64)
    return DeviceDataset(num_users, num_items, users, items, off, items, name="synthetic-large")


def ml1m_like(seed: int = 2019) -> SyntheticDataset:
    return synthetic_dataset(**ML1M_SHAPE, seed=seed, name="ml-1m-synthetic")


def pinterest_like(seed: int = 2019) -> SyntheticDataset:
    return synthetic_dataset(**PINTEREST_SHAPE, seed=seed, name="pinterest-20-synthetic")


def yelp_like(seed: int = 2019) -> SyntheticDataset:
    return synthetic_dataset(**YELP_SHAPE, seed=seed, name="yelp-sort-synthetic")


def get_dataset(name: str, path: str = "", seed: int = 2019):
    """Resolve --dataset: a file prefix under <path>data/, or a synthetic shape
    ("ml-1m-synthetic", "pinterest-20-synthetic", "yelp-sort-synthetic", "synthetic:U:I:N")."""
    import os
    if name == "ml-1m-synthetic":
        return ml1m_like(seed)
    if name == "pinterest-20-synthetic":
        return pinterest_like(seed)
    if name == "yelp-sort-synthetic":
        return yelp_like(seed)
    if name.startswith("synthetic:"):
        _, U, I, N = name.split(":")
        return synthetic_dataset(int(U), int(I), int(N), seed=seed)
    prefix = os.path.join(path, "data", name) if not os.path.exists(name + ".train.rating") else name
    return OriginalDataset(prefix)
