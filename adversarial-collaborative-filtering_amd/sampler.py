"""Triplet sampling: ``sampling`` / ``shuffle`` / ``_get_train_batch``
(``APR.py:30-81``).

Reference semantics kept exactly:
  * positives are the ``trainMatrix.keys()`` pairs (first-insertion order);
  * an epoch shuffles their index and keeps ``len // batch_size`` full batches
    (drop-last, ``APR.py:52``);
  * one negative per triplet, uniform on ``[0, num_items)``, redrawn while it is in
    ``trainList[u]`` (``APR.py:76-78``) — ``trainList`` with its misalignment, so a
    negative may equal the positive for users next to a missing uid; it may be item
    0 or the test item.

The reference's stream is not reproducible (forked Pool workers share the numpy
RNG state, ``APR.py:53``), so parity is defined on the distribution; the GPU
sampler (:class:`DeviceSampler`) uses a counter-based RNG keyed by (seed, epoch).
"""
from __future__ import annotations

import numpy as np


def sampling(dataset):
    """APR.py:30-36: (user_input, item_input_pos) lists of the positive pairs."""
    return dataset.pair_user.tolist(), dataset.pair_item.tolist()


def _membership_keys(dataset):
    off, items = dataset.sorted_lists()
    owner = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
    return owner * np.int64(dataset.num_items + 1) + items.astype(np.int64)


def sample_negatives_host(users: np.ndarray, dataset, rng=np.random) -> np.ndarray:
    """Vectorised rejection sampler with the reference's acceptance rule."""
    keys = getattr(dataset, "_member_keys", None)
    if keys is None:
        keys = _membership_keys(dataset)
        dataset._member_keys = keys
    users = np.asarray(users, dtype=np.int64)
    n_lists = dataset.trainlist_len()
    if users.size and (users.min() < 0 or users.max() >= n_lists):
        raise IndexError("user outside trainList (IndexError in APR.py:77)")
    neg = rng.randint(dataset.num_items, size=len(users)).astype(np.int64)
    todo = np.arange(len(users))
    for _ in range(1 << 20):
        k = users[todo] * np.int64(dataset.num_items + 1) + neg[todo]
        pos = np.searchsorted(keys, k)
        pos = np.minimum(pos, len(keys) - 1) if len(keys) else pos
        bad = (keys[pos] == k) if len(keys) else np.zeros(len(todo), bool)
        todo = todo[bad]
        if not len(todo):
            break
        neg[todo] = rng.randint(dataset.num_items, size=len(todo))
    else:
        raise RuntimeError("no admissible negative for some users")
    return neg.astype(np.int32)


def shuffle(samples, batch_size, dataset, model=None, rng=np.random):
    """APR.py:39-61 (dns = model.dns): returns (user_list, item_pos_list,
    user_dns_list, item_dns_list), each a list of [B,1] / [B*dns,1] arrays."""
    user_input, item_input_pos = (np.asarray(s, dtype=np.int32) for s in samples)
    dns = getattr(model, "dns", 1) if model is not None else 1
    index = np.arange(len(user_input))
    rng.shuffle(index)
    num_batch = len(user_input) // batch_size
    index = index[:num_batch * batch_size]
    u = user_input[index]
    i = item_input_pos[index]
    ud = np.repeat(u, dns)
    j = sample_negatives_host(ud, dataset, rng)
    ub = u.reshape(num_batch, batch_size, 1)
    ib = i.reshape(num_batch, batch_size, 1)
    udb = ud.reshape(num_batch, batch_size * dns, 1)
    jb = j.reshape(num_batch, batch_size * dns, 1)
    return list(ub), list(ib), list(udb), list(jb)


class EpochTriplets:
    """One epoch of device-resident triplets (int32, length n_batches*batch_size)."""

    def __init__(self, user, item_pos, item_neg, batch_size: int):
        self.user, self.item_pos, self.item_neg = user, item_pos, item_neg
        self.batch_size = int(batch_size)
        self.n_batches = user.numel() // self.batch_size

    def __len__(self):
        return self.n_batches

    def as_lists(self):
        """The reference's 4-list batches format (host numpy)."""
        B, nb = self.batch_size, self.n_batches
        u = self.user.cpu().numpy().reshape(nb, B, 1)
        i = self.item_pos.cpu().numpy().reshape(nb, B, 1)
        j = self.item_neg.cpu().numpy().reshape(nb, B, 1)
        return list(u), list(i), list(u), list(j)


class DeviceSampler:
    """GPU shuffle + negative sampler over a dataset (acf_sample_epoch).

    ``weights`` (optional, one per item): negatives are proposed from an alias
    table of these weights (acf_sample_epoch_alias; e.g. popularity**0.75)
    instead of uniformly, then accepted by the same trainList rule.  Equal
    weights give the reference's uniform sampler, draw for draw."""

    def __init__(self, dataset, batch_size: int, device, seed: int = 0, weights=None):
        import torch
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.device = torch.device(device)
        self.seed = int(seed)
        if hasattr(dataset, "device_arrays"):  # data.DeviceDataset: already on the device
            self.pos_user, self.pos_item, self.list_off, self.list_items = dataset.device_arrays()
        else:
            off, items = dataset.sorted_lists()
            self.list_off = torch.as_tensor(off, dtype=torch.int64, device=self.device)
            self.list_items = torch.as_tensor(items, dtype=torch.int32, device=self.device)
            self.pos_user = torch.as_tensor(dataset.pair_user, dtype=torch.int32, device=self.device)
            self.pos_item = torch.as_tensor(dataset.pair_item, dtype=torch.int32, device=self.device)
        self.num_items = int(dataset.num_items)
        self.alias = None
        if weights is not None:
            from . import ops
            if len(weights) != self.num_items:
                raise ValueError(f"{len(weights)} weights for {self.num_items} items")
            prob, alias = ops.alias_table(weights)
            self.alias = (torch.as_tensor(prob, device=self.device), torch.as_tensor(alias, device=self.device))

    def epoch(self, epoch: int, check: bool = True) -> EpochTriplets:
        from . import ops
        seed = (self.seed * 0x9E3779B1 + epoch * 0x85EBCA77 + 1) & 0xFFFFFFFFFFFFFFFF
        u, i, j = ops.sample_epoch(self.pos_user, self.pos_item, self.batch_size, self.num_items,
                                   self.list_off, self.list_items, seed, check=check, alias=self.alias)
        return EpochTriplets(u, i, j, self.batch_size)
