"""APR training split across the GPUs of one node (BASELINE.json
configs[2] "item table row-sharded across 8 x MI355X" and configs[4] "8 x MI355X").

The reference trains one process on one CPU (``training_batch``, utils.py:106-119,
over the TF1 graph of APR.py:121-195).  Here one global batch of triplets is
split over G ranks (one process per GPU, RCCL over xGMI) and the result is the
single-process step up to fp32 summation order.

Ownership (nothing replicated):
  * user row u of P (and its Adagrad slot) on rank u % G at local row u // G;
  * item row i of Q (and its Adagrad slot) on rank i % G at local row i // G.

Routing: a triplet (u, i, j) runs on its USER's rank, so a user's batch-summed
clean gradient, its delta and its Adagrad step are local.  An item's
occurrences are spread over the ranks, so the batch-global item sums the graph
needs (the delta of APR.py:183-191 and the dedup before SparseApplyAdagrad,
APR.py:193-195) are completed by the item's owner.  One step:

  E1  owners send the current Q rows of each rank's item working set
      (all_to_all; the working set is the rank's unique items of the batch);
  P0  local clean pass (HIP, shard mode): user delta; partial item sums;
  E2  partial item sums -> owners (all_to_all); owners sum them in requester
      order and form delta = eps * l2_normalize(sum);
  E3  deltas -> requesters (all_to_all);
  P1  local adversarial pass: user Adagrad; partial adversarial item sums;
  E4  -> owners (all_to_all); owners: G = clean + reg_adv * adversarial, Adagrad.

BPR (adver = 0): E1, P0 (users updated), E2 + owner Adagrad.

E1 has two forms (``item_exchange``): "all_to_all" (default) sends each rank just
the rows of its working set; "allgather" is the form BASELINE.json's north_star
and configs[2] name -- an RCCL all_gather of every rank's Q shard (the small
pinterest item table replicated for the step), from which each rank takes the
rows its negatives and positives need.  E2-E4 are the same in both.

The working sets and the exchange plans of a whole chunk of steps are built on
device in one go (one host sync per chunk, for the all_to_all split sizes).
Every rank sees the same global triplet stream (the sampler is seeded
identically) and keeps its users' triplets, in stream order.

The local compute is pluggable: :class:`HipLocal` (the product path: the step
kernels in shard mode, include/acf_apr.h) on GPUs; the CPU tests plug in the
oracle's restatement (oracle/shard_oracle.py) to exercise the same routing and
exchanges over gloo.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as dist


class HipLocal:
    """One rank's local passes and owner reductions on the HIP kernels."""

    def __init__(self, sh: "ShardedAPR"):
        from . import ops
        self.ops = ops
        self.sh = sh
        self.ctx = ops.APRContext(sh.P.shape[0], sh.max_items, sh.d, sh.b_max, 1, sh.device)
        self.ctx.set_shard_mode(True, reg_batch=sh.B)
        # the fetched item rows are never updated locally; their Adagrad slots are unused
        self.accQc = torch.full((sh.max_items, sh.d), 0.1, device=sh.device)

    def _tables(self):
        sh = self.sh
        return (sh.P, sh.Qc, sh.accP, self.accQc)

    def plan(self, u_rows, wi, wj):
        self.ctx.plan(u_rows, wi, wj, u_rows.numel(), check=False)

    def clean(self, hp, out):
        self.ctx.shard_pass(self._tables(), hp, 0)
        self.ctx.shard_items_out(out)

    def set_item_delta(self, delta):
        self.ctx.shard_items_delta(delta)

    def adv(self, hp, out):
        self.ctx.shard_pass(self._tables(), hp, 1)
        self.ctx.shard_items_out(out)

    def reduce_delta(self, hp, recv, seg, pos, G0, reply):
        self.ops.shard_reduce_delta(recv, seg, pos, hp, G0, reply)

    def reduce_apply(self, hp, recv, seg, pos, G0, rows, count):
        self.ops.shard_reduce_apply(self.sh.Q, self.sh.accQ, recv, seg, pos, hp, G0, rows, count,
                                    reg_batch=self.sh.B)

    def step_errors(self) -> int:
        return self.ctx.step_errors()


class _Chunk:
    """Device-side routing of one chunk of T global batches for this rank, plus
    the host copies of the split sizes."""


class ShardedAPR:
    """This rank's shard of embedding_P / embedding_Q (+ Adagrad slots) and the
    split APR step.  ``batch_size`` is the GLOBAL batch (the reference's
    ``--batch_size``); each rank processes the triplets of its users.
    ``local_batch``: triplets are routed at sampling time (train_routed), each
    rank holding exactly this many of every global batch (= G x local_batch)."""

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, batch_size: int, device=None,
                 group=None, init_P=None, init_Q=None, acc0: float = 0.1, local=None,
                 local_batch: int | None = None, item_exchange: str = "all_to_all"):
        if item_exchange not in ("all_to_all", "allgather"):
            raise ValueError(f"item_exchange must be 'all_to_all' or 'allgather', got {item_exchange!r}")
        self.item_exchange = item_exchange
        self.group = group
        self.G = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.U1, self.I1, self.d, self.B = int(num_user_rows), int(num_item_rows), int(dim), int(batch_size)
        if self.U1 < self.G or self.I1 < self.G:
            raise ValueError(f"tables of {self.U1} x {self.I1} rows cannot be split over {self.G} ranks")
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._stage = self.device.type == "cuda" and dist.get_backend(group) == "gloo"
        G, r = self.G, self.rank
        f = dict(dtype=torch.float32, device=self.device)
        nu, ni = len(range(r, self.U1, G)), len(range(r, self.I1, G))
        self.P = torch.empty(nu, dim, **f)
        self.Q = torch.empty(ni, dim, **f)
        if init_P is not None:
            self.P.copy_(torch.as_tensor(np.asarray(init_P, np.float32)[r::G]))
            self.Q.copy_(torch.as_tensor(np.asarray(init_Q, np.float32)[r::G]))
        self.accP = torch.full((nu, dim), acc0, **f)
        self.accQ = torch.full((ni, dim), acc0, **f)
        if local_batch is not None and local_batch * self.G != self.B:
            raise ValueError(f"local_batch {local_batch} x {self.G} ranks != batch_size {self.B}")
        self.b_max = int(local_batch) if local_batch is not None else self.B  # triplets of a rank per batch
        self.routed = local_batch is not None
        self.max_items = 2 * self.b_max  # a rank's working set of one batch: <= 2 x its triplets
        self.Qc = torch.zeros(self.max_items, dim, **f)
        self._send = torch.empty(self.max_items, dim, **f)
        self._dlt = torch.empty(self.max_items, dim, **f)
        self._recv = torch.empty(0, dim, **f)
        self._qcap = (self.I1 + G - 1) // G  # rows of the largest Q shard (all_gather slots)
        self._qpad = torch.zeros(self._qcap, dim, **f) if item_exchange == "allgather" else None
        self._qall = torch.empty(G * self._qcap, dim, **f) if item_exchange == "allgather" else None
        self.local = local(self) if local is not None else HipLocal(self)
        self.stats = {"steps": 0, "items_requested": 0, "rows_served": 0, "triplets": 0, "route_s": 0.0}

    # -- collectives ---------------------------------------------------------------
    def _a2a(self, out, inp, out_splits, in_splits):
        if self._stage:  # gloo with device tensors (rehearsal of several ranks on one GPU)
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _gather_q(self):
        """E1, "allgather" form: every rank's Q shard to every rank (RCCL all_gather);
        row i is then at _qall[(i % G) * cap + i // G]."""
        n = self.Q.shape[0]
        self._qpad[:n] = self.Q
        if self._stage:
            parts = [torch.empty(self._qcap, self.d) for _ in range(self.G)]
            dist.all_gather(parts, self._qpad.cpu(), group=self.group)
            self._qall.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(self._qall, self._qpad, group=self.group)

    # -- routing (one chunk of T global batches) -----------------------------------
    def _route(self, u, i, j, T: int) -> _Chunk:
        G, r, I1 = self.G, self.rank, self.I1
        B = self.b_max if self.routed else self.B  # triplets per batch in the stream given
        dev = self.device
        u, i, j = (torch.as_tensor(x, device=dev).reshape(-1)[: T * B].long() for x in (u, i, j))
        if u.numel() != T * B:
            raise ValueError(f"{u.numel()} triplets for {T} batches of {B}")
        # index checks, read with the chunk's host copy below (no extra sync):
        # bit 0 out of range (TF Gather's InvalidArgument), bit 1 another rank's user (routed).
        # Every rank's flags travel with the first exchange, so all ranks raise together
        # (a rank raising alone would leave its peers waiting in the next collective).
        bad = ((u < 0) | (u >= self.U1) | (i < 0) | (i >= I1) | (j < 0) | (j >= I1)).any().long()
        if self.routed:
            bad = bad + 2 * (u % G != r).any().long()
        # clamp so that the routing below stays in range on bad input (it is discarded)
        u, i, j = u.clamp(0, self.U1 - 1), i.clamp(0, I1 - 1), j.clamp(0, I1 - 1)
        c = _Chunk()
        c.T = T
        # this rank's triplets, stream order
        sel = torch.arange(u.numel(), device=dev) if self.routed else torch.nonzero(u % G == r).squeeze(1)
        st = sel // B
        n = sel.numel()
        c.u_rows = (u[sel] // G).to(torch.int32)
        items = torch.cat([i[sel], j[sel]])
        ist = torch.cat([st, st])
        # working set per step: unique items, ordered by (owner, id) so that each
        # owner's rows are one contiguous block of the all_to_all buffers
        uk, inv = torch.unique((ist * G + items % G) * I1 + items, return_inverse=True)
        wstep, wown, wid = uk // (G * I1), (uk // I1) % G, uk % I1
        cnt = torch.bincount(wstep * G + wown, minlength=T * G).view(T, G)
        nloc = torch.bincount(st, minlength=T)
        nW = cnt.sum(1)
        wstart = torch.cumsum(nW, 0) - nW
        widx = (inv - wstart[ist]).to(torch.int32)
        c.wi, c.wj = widx[:n], widx[n:]
        if self.item_exchange == "allgather":  # where each working-set row sits in the gathered table
            c.wslot = ((wid % G) * self._qcap + wid // G).long()
        # the requests of the whole chunk, owner-major, in one exchange
        order = torch.argsort((wown * T + wstep) * I1 + wid)
        req = (wid // G)[order]
        # split sizes (T per owner) + this rank's error flags, to every rank in one exchange
        send = torch.cat([cnt.t(), bad.reshape(1, 1).expand(G, 1)], 1).contiguous()
        recv = torch.empty_like(send)
        self._a2a(recv.view(-1), send.view(-1), [T + 1] * G, [T + 1] * G)
        rc = recv[:, :T]
        host = torch.cat([cnt.reshape(-1), rc.reshape(-1), nloc, recv[:, T]]).cpu().numpy()  # one sync
        flags = host[-G:]
        if flags.any():
            who = [o for o in range(G) if flags[o]]
            if np.bitwise_or.reduce(flags) & 1:
                raise IndexError(f"triplet index outside the sharded tables (rank(s) {who})")
            raise ValueError(f"train_routed: a triplet of another rank's user (rank(s) {who})")
        c.cnt = host[: T * G].reshape(T, G)           # my requests per (step, owner)
        c.rc = host[T * G: 2 * T * G].reshape(G, T)   # requests to me per (requester, step)
        c.nloc = host[2 * T * G: -G]
        rows = torch.empty(int(c.rc.sum()), dtype=req.dtype, device=dev)
        self._a2a(rows, req, c.rc.sum(1).tolist(), c.cnt.sum(0).tolist())
        # received rows in per-step all_to_all order: step, then requester, then id
        c.R = c.rc.sum(0)                                   # rows I serve per step
        c.Rs = np.concatenate([[0], np.cumsum(c.R)])
        pstart = np.cumsum(c.rc, 0) - c.rc                  # [G, T] requester offset inside a step
        blk_start = (c.Rs[:-1][None, :] + pstart).reshape(-1)  # block (requester o, step t) -> position
        blk_len = c.rc.reshape(-1)
        src_pos = np.concatenate([[0], np.cumsum(blk_len)])[:-1]
        k = torch.arange(rows.numel(), device=dev) - torch.as_tensor(np.repeat(src_pos, blk_len), device=dev)
        q = torch.as_tensor(np.repeat(blk_start, blk_len), device=dev) + k
        served = torch.empty_like(rows)
        served[q] = rows
        c.served = served                                   # owner-local rows, step-major
        # owner reduction segments: per (step, row), positions in requester order
        step_of = torch.as_tensor(np.repeat(np.arange(T), c.R), device=dev)
        key = step_of * (self.Q.shape[0] + 1) + served
        skey, spos = torch.sort(key, stable=True)
        head = torch.ones_like(skey, dtype=torch.bool)
        if skey.numel() > 1:
            head[1:] = skey[1:] != skey[:-1]
        starts = torch.nonzero(head).squeeze(1)
        c.seg = torch.cat([starts, torch.tensor([skey.numel()], device=dev)]).to(torch.int32)
        c.pos = (spos - torch.as_tensor(c.Rs[:-1], device=dev)[step_of[spos]]).to(torch.int32)
        c.own_rows = served[spos[starts]].to(torch.int32)
        nseg = torch.bincount(step_of[spos[starts]], minlength=T) if starts.numel() else torch.zeros(T)
        c.Sa = np.concatenate([[0], np.cumsum(nseg.cpu().numpy())]).astype(np.int64)
        c.lo = np.concatenate([[0], np.cumsum(c.nloc)])
        c.nW = c.cnt.sum(1)
        c.w0 = np.concatenate([[0], np.cumsum(c.nW)])  # working-set start of each step (host)
        c.count = None
        self._chunk_items = (i, j)
        return c

    def _counts(self, c: _Chunk, i, j):
        """Occurrences of every owned row of each step in the GLOBAL batch (the
        reg * mean(w^2) gradient counts them, APR.py:153-154)."""
        G, B, T = self.G, self.B, c.T
        items = torch.cat([i, j])
        st = torch.cat([torch.arange(T * B, device=self.device) // B] * 2)
        mine = items % G == self.rank
        nrow = self.Q.shape[0] + 1
        cnt = torch.bincount(st[mine] * nrow + items[mine] // G, minlength=T * nrow)
        seg_step = torch.as_tensor(np.repeat(np.arange(T), np.diff(c.Sa)), device=self.device)
        return cnt[seg_step * nrow + c.own_rows.long()].to(torch.int32)

    # -- one step ------------------------------------------------------------------
    def _step(self, c: _Chunk, t: int, hp):
        d = self.d
        cnt, rc = c.cnt[t].tolist(), c.rc[:, t].tolist()
        b, nw, R = int(c.nloc[t]), int(c.nW[t]), int(c.R[t])
        if self._recv.shape[0] < R:
            self._recv = torch.empty(max(R, 2 * self._recv.shape[0]), d, dtype=torch.float32, device=self.device)
        lo = int(c.lo[t])
        served = c.served[c.Rs[t]: c.Rs[t] + R]
        seg = c.seg[c.Sa[t]: c.Sa[t + 1] + 1]
        own_rows = c.own_rows[c.Sa[t]: c.Sa[t + 1]]
        count = None if c.count is None else c.count[c.Sa[t]: c.Sa[t + 1]]
        nseg = seg.numel() - 1
        recv, reply = self._recv[:R], self._recv_reply(R)
        part = self._send[:nw]
        # E1: current item rows of my working set from their owners
        if self.item_exchange == "allgather":
            self._gather_q()
            w0 = int(c.w0[t])
            torch.index_select(self._qall, 0, c.wslot[w0: w0 + nw], out=self.Qc[:nw])
        else:
            self._a2a(self.Qc[:nw], self.Q.index_select(0, served.long()), cnt, rc)
        if b:
            self.local.plan(c.u_rows[lo: lo + b], c.wi[lo: lo + b], c.wj[lo: lo + b])
            self.local.clean(hp, part)
        # E2: partial clean item sums -> owners
        self._a2a(recv, part, rc, cnt)
        G0 = self._g0(nseg)
        if hp.adver:
            self.local.reduce_delta(hp, recv, seg, c.pos, G0, reply)
            # E3: deltas -> requesters
            self._a2a(self._dlt[:nw], reply, cnt, rc)
            if b:
                self.local.set_item_delta(self._dlt[:nw])
                self.local.adv(hp, part)
            # E4: partial adversarial item sums -> owners, who apply Adagrad
            self._a2a(recv, part, rc, cnt)
            self.local.reduce_apply(hp, recv, seg, c.pos, G0, own_rows, count)
        else:
            self.local.reduce_apply(hp, recv, seg, c.pos, None, own_rows, count)
        st = self.stats
        st["steps"] += 1
        st["items_requested"] += nw
        st["rows_served"] += R
        st["triplets"] += b

    def _recv_reply(self, R):
        buf = getattr(self, "_reply", None)
        if buf is None or buf.shape[0] < R:
            self._reply = buf = torch.empty(max(R, 1), self.d, dtype=torch.float32, device=self.device)
        return buf[:R]

    def _g0(self, n):
        buf = getattr(self, "_g0buf", None)
        if buf is None or buf.shape[0] < n:
            self._g0buf = buf = torch.empty(max(n, 1), self.d, dtype=torch.float32, device=self.device)
        return buf[:n]

    # -- public --------------------------------------------------------------------
    def train(self, u, i, j, hp, chunk: int = 64) -> int:
        """Train consecutive global batches of the stream (u, i, j), identical on
        every rank (length a multiple of the batch size; train_routed: this rank's
        triplets only, local_batch per batch).  Returns the batches run."""
        bs = self.b_max if self.routed else self.B
        n = len(u) // bs
        for c0 in range(0, n, chunk):
            T = min(chunk, n - c0)
            s = slice(c0 * bs, (c0 + T) * bs)
            t0 = time.perf_counter()
            c = self._route(u[s], i[s], j[s], T)
            self.stats["route_s"] += time.perf_counter() - t0
            if hp.reg:  # the owners count their rows in the GLOBAL batch
                if self.routed:
                    raise ValueError("reg != 0 needs the global stream on every rank (train, not train_routed)")
                c.count = self._counts(c, *self._chunk_items)
            for t in range(T):
                self._step(c, t, hp)
        return n

    def train_routed(self, u, i, j, hp, chunk: int = 64) -> int:
        """As train, for triplets routed at sampling time: this rank's users only,
        local_batch of them per global batch (the sampler runs per rank)."""
        if not self.routed:
            raise ValueError("train_routed needs ShardedAPR(local_batch=...)")
        return self.train(u, i, j, hp, chunk)

    def step_errors(self) -> int:
        return self.local.step_errors() if hasattr(self.local, "step_errors") else 0

    def full_tables(self):
        """The full tables on every rank (checkpoints, evaluation, tests)."""
        outs = []
        for tab, n in ((self.P, self.U1), (self.Q, self.I1), (self.accP, self.U1), (self.accQ, self.I1)):
            cap = (n + self.G - 1) // self.G
            cdev = torch.device("cpu") if self._stage else self.device
            buf = torch.zeros(cap, self.d, dtype=torch.float32, device=cdev)
            buf[: tab.shape[0]] = tab
            parts = [torch.empty_like(buf) for _ in range(self.G)]
            dist.all_gather(parts, buf, group=self.group)
            full = torch.empty(n, self.d, dtype=torch.float32, device=cdev)
            for r in range(self.G):
                full[r::self.G] = parts[r][: len(range(r, n, self.G))]
            outs.append(full.to(self.device))
        return outs
