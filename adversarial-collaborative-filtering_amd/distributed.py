"""Row-sharded tables across the GPUs of one node (BASELINE.json configs[2]:
"item table row-sharded across 8 x MI355X with RCCL all-gather of negative rows
over xGMI").

Ownership: row r of P (users) and of Q (items), with its Adagrad slot, lives on
rank r % world at local index r // world.  Nothing is replicated.

One chunk of consecutive mini-batches (the same global triplet stream on every
rank) runs as:

1. working set: the unique users / items the chunk touches (sorted);
2. ONE all-gather: each rank contributes the [w | acc] rows it owns of that
   working set (user rows and item rows — positives and sampled negatives);
3. every rank runs the chunk's batches on the compact working-set tables with the
   single-GPU step kernels (remapped indices) — a B = 512 step is far too small to
   split, so it is computed redundantly rather than exchanged per phase;
4. each owner writes its rows back.

The per-row arithmetic and the per-row occurrence order are the ones of the
single-GPU path, so the result is bit-identical to training the full tables on
one device (tests/test_distributed.py checks it with gloo on CPU; on GPUs the
collective is RCCL over xGMI).  Communication per chunk = 2 x d x 4 B x
working-set rows; it buys capacity (tables 1/world per GPU), not speed — the
benchmark's multi-GPU line runs independent replicas instead.
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch
import torch.distributed as dist

# step_fn(P, Q, accP, accQ, u, i, j, batch_size, hp) trains in place on the tables
StepFn = Callable[..., None]


def hip_step(P, Q, accP, accQ, u, i, j, batch_size, hp, _cache={}):
    """Default step: the HIP kernels (plan + hipGraph replay) on device tensors."""
    from . import ops
    nb = u.numel() // batch_size
    key = (P.shape[0], Q.shape[0], P.shape[1], batch_size, P.device)
    ctx = _cache.get(key)
    if ctx is None or not ctx.fits(batch_size, nb):
        ctx = _cache[key] = ops.APRContext(P.shape[0], Q.shape[0], P.shape[1], batch_size,
                                           max(nb, ctx.max_batches if ctx else 0), P.device)
    ctx.plan(u, i, j, batch_size)
    ctx.train_planned((P, Q, accP, accQ), hp, 0, nb, graph=False)


class ShardedTables:
    """This rank's shard of embedding_P / embedding_Q and their Adagrad slots."""

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, device=None, group=None,
                 init_P=None, init_Q=None, acc0: float = 0.1):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.U1, self.I1, self.d = int(num_user_rows), int(num_item_rows), int(dim)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        rows_u = np.arange(self.rank, self.U1, self.world)
        rows_i = np.arange(self.rank, self.I1, self.world)
        f = dict(dtype=torch.float32, device=self.device)
        self.P = torch.empty(len(rows_u), dim, **f)
        self.Q = torch.empty(len(rows_i), dim, **f)
        if init_P is not None:
            self.P.copy_(torch.as_tensor(np.asarray(init_P)[rows_u]))
            self.Q.copy_(torch.as_tensor(np.asarray(init_Q)[rows_i]))
        self.accP = torch.full((len(rows_u), dim), acc0, **f)
        self.accQ = torch.full((len(rows_i), dim), acc0, **f)

    # -- helpers ---------------------------------------------------------------
    def _gather_rows(self, table, acc, rows: np.ndarray):
        """All-gather [w | acc] of `rows` (sorted global ids) from their owners,
        returned in `rows` order."""
        W, G, d = self.world, self.group, self.d
        mine = rows[rows % W == self.rank]
        local = torch.as_tensor(mine // W, dtype=torch.long, device=self.device)
        payload = torch.cat([table[local], acc[local]], 1)
        counts = np.bincount(rows % W, minlength=W)
        cap = int(counts.max()) if len(rows) else 0
        buf = torch.zeros(cap, 2 * d, dtype=torch.float32, device=self.device)
        buf[: len(mine)] = payload
        parts = [torch.empty_like(buf) for _ in range(W)]
        dist.all_gather(parts, buf, group=G)
        out = torch.empty(len(rows), 2 * d, dtype=torch.float32, device=self.device)
        for r in range(W):
            sel = np.flatnonzero(rows % W == r)
            if len(sel):
                out[torch.as_tensor(sel, device=self.device)] = parts[r][: len(sel)]
        return out[:, :d].contiguous(), out[:, d:].contiguous()

    def _write_back(self, table, acc, rows: np.ndarray, w, a):
        W = self.world
        sel = np.flatnonzero(rows % W == self.rank)
        if not len(sel):
            return
        s = torch.as_tensor(sel, device=self.device)
        local = torch.as_tensor(rows[sel] // W, dtype=torch.long, device=self.device)
        table[local] = w[s]
        acc[local] = a[s]

    # -- training ----------------------------------------------------------------
    def train_chunk(self, u, i, j, batch_size: int, hp, step_fn: StepFn = hip_step):
        """Train consecutive batches of the global stream (u, i, j identical on
        every rank).  hp: the step hyper-parameters understood by step_fn."""
        u = np.asarray(u, dtype=np.int64).reshape(-1)
        i = np.asarray(i, dtype=np.int64).reshape(-1)
        j = np.asarray(j, dtype=np.int64).reshape(-1)
        if u.size and (u.min() < 0 or u.max() >= self.U1 or min(i.min(), j.min()) < 0
                       or max(i.max(), j.max()) >= self.I1):
            raise IndexError("triplet index outside the sharded tables")
        ws_u = np.unique(u)
        ws_i = np.unique(np.concatenate([i, j]))
        Pw, aPw = self._gather_rows(self.P, self.accP, ws_u)
        Qw, aQw = self._gather_rows(self.Q, self.accQ, ws_i)
        to_dev = lambda x: torch.as_tensor(x.astype(np.int32), device=self.device)  # noqa: E731
        step_fn(Pw, Qw, aPw, aQw, to_dev(np.searchsorted(ws_u, u)), to_dev(np.searchsorted(ws_i, i)),
                to_dev(np.searchsorted(ws_i, j)), batch_size, hp)
        self._write_back(self.P, self.accP, ws_u, Pw, aPw)
        self._write_back(self.Q, self.accQ, ws_i, Qw, aQw)
        return len(ws_u), len(ws_i)

    def full_tables(self):
        """Assemble the full tables on every rank (checkpoint / evaluation)."""
        outs = []
        for tab, n in ((self.P, self.U1), (self.Q, self.I1), (self.accP, self.U1), (self.accQ, self.I1)):
            cap = (n + self.world - 1) // self.world
            buf = torch.zeros(cap, self.d, dtype=torch.float32, device=self.device)
            buf[: tab.shape[0]] = tab
            parts = [torch.empty_like(buf) for _ in range(self.world)]
            dist.all_gather(parts, buf, group=self.group)
            full = torch.empty(n, self.d, dtype=torch.float32, device=self.device)
            for r in range(self.world):
                cnt = len(range(r, n, self.world))
                full[r::self.world] = parts[r][:cnt]
            outs.append(full)
        return outs
