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

Static step layout.  Every exchange buffer has a fixed shape: G blocks of C rows
(C = the chunk's largest per-peer request count, rounded up and only ever
grown), block o holding what this rank exchanges with rank o, plus one trash
row.  The routing of a chunk of T steps (one host sync, for the counts) writes
per-step index maps into persistent buffers at fixed per-step offsets:
``wsrc`` (working-set entry -> its row of the exchange blocks: the passes
write the item sums there and read the deltas from there), ``srv`` (exchange
row -> owned row), and the owner's
segments ``seg`` / ``pos`` / ``own`` (rows padded with empty segments on a
trash row of the Q storage).  A step therefore has no host-side sizes, so a
chunk's steps are captured as hipGraphs once and replayed:

  * world 1: the exchanges are the identity (no collective), the whole chunk is
    ONE graph;
  * world > 1: a chunk is captured as SEGMENTS cut at every collective, the
    fixed-size RCCL all_to_all / all_gather calls host-issued between the
    segment replays (the default since r06), with the plans in line while
    capturing (r04's pipelined plan straddled the cuts: the capture failed --
    the "allocator assertion" of r04).  ``capture_collectives=True``
    (or ACF_SHARD_RCCL_GRAPH=1) captures the collectives INSIDE the graph too,
    after a one-off capture + replay of an all_reduce at construction that every
    rank must pass, so a chunk is again ONE graph with no host round trip per
    exchange.  That form is rehearsed only as a one-rank RCCL self-exchange on
    one GPU (RCCL refuses two ranks on one GPU), never at world > 1 on several
    GPUs, so it is opt-in.  A graph holding captured RCCL work keeps
    the communicator busy, so the graphs are dropped before the process group
    goes: ``close()``, the with-block, the object's collection or, failing all
    three, the interpreter's exit (a weakref.finalize; tools/rccl_capture_probe.py
    checks the orders).  The recorded collectives of a segment capture hold the
    tensors and the group, never the object, so a dropped object is collected in
    both forms.
    ``force_collectives`` routes the
    exchanges through the process group even at world 1 (an RCCL self-exchange):
    the one-GPU rehearsal of the captured collectives
    (tests/test_gpu_distributed.py).

The working sets and the exchange plans of a whole chunk of steps are built on
device in one go.  Every rank sees the same global triplet stream (the sampler
is seeded identically) and keeps its users' triplets, in stream order.

The local compute is pluggable: :class:`HipLocal` (the product path: the step
kernels in shard mode, include/acf_apr.h) on GPUs; the CPU tests plug in the
oracle's restatement (oracle/shard_oracle.py) to exercise the same routing and
exchanges over gloo.
"""
from __future__ import annotations

import os
import time
import warnings
import weakref

import numpy as np
import torch
import torch.distributed as dist


def _drop_graphs(graphs: dict, device) -> None:
    """ShardedAPR's finalizer: wait for the device, then release the captured step
    graphs (it holds no reference to the ShardedAPR itself)."""
    if device is not None and graphs:
        torch.cuda.synchronize(device)
    graphs.clear()


class HipLocal:
    """One rank's local passes and owner reductions on the HIP kernels.  Two
    step contexts (plan buffers + pass scratch) alternate by step parity, so the
    plan of step t + 1 runs beside step t (ShardedAPR._step, r04)."""

    graphable = True  # every call is a fixed-shape launch sequence (no host sync)
    pipelined = True  # plan_into / use: the next step's plan beside this step
    # (r06) plan_chunk / use_batch: a chunk of equal local batches (the hash
    # plan) planned at once, each step one batch of it -- one plan's launches per
    # chunk instead of one plan beside every step
    chunk_planned = True
    # ... for local batches larger than this: every size (configs[2]'s 512-triplet
    # batches too: 0.055 -> 0.045 ms per step, profiles/r06/shard_chunk_small_ab.json)
    chunk_min = 0

    def __init__(self, sh: "ShardedAPR"):
        from . import ops
        self.ops = ops
        self.sh = sh
        self.ctxs = [ops.APRContext(sh.P.shape[0], sh.max_items, sh.d, sh.b_max, 1, sh.device) for _ in range(2)]
        for c in self.ctxs:
            c.set_shard_mode(True, reg_batch=sh.B)
        self.ctx = self.ctxs[0]  # the context the passes below use
        self.cctx, self._cT = None, 0  # the chunk plan's context (plan_chunk), sized for _cT steps
        # the fetched item rows are never updated locally; their Adagrad slots are unused
        self.accQc = torch.full((sh.max_items, sh.d), 0.1, device=sh.device)

    def _tables(self):
        sh = self.sh
        return (sh.P, sh.Qc, sh.accP, self.accQc)

    def use(self, k: int) -> None:
        self.ctx = self.ctxs[k]

    def plan_into(self, k: int, u_rows, wi, wj):
        self.ctxs[k].plan(u_rows, wi, wj, u_rows.numel(), check=False)

    def plan(self, u_rows, wi, wj):
        self.ctx.plan(u_rows, wi, wj, u_rows.numel(), check=False)

    def plan_chunk(self, u_rows, wi, wj):
        """[T, b] local rows of T steps, planned as ONE T-batch plan (shard mode,
        T > 1: the triplet-centric hash plan, whose batches are independent); the
        passes then take batch t of it (use_batch)."""
        sh, (T, b) = self.sh, tuple(u_rows.shape)
        if self.cctx is None or self._cT < T:
            self.cctx = None  # free the smaller one first
            self.cctx = self.ops.APRContext(sh.P.shape[0], sh.max_items, sh.d, sh.b_max, T, sh.device)
            self.cctx.set_shard_mode(True, reg_batch=sh.B)
            self._cT = T
        self.ctx = self.cctx
        self.cctx.plan(u_rows.reshape(-1), wi.reshape(-1), wj.reshape(-1), b, check=False)

    def use_batch(self, t: int) -> None:
        self.cctx.set_shard_batch(t)

    def chunk_ok(self) -> bool:
        """Chunk plans are triplet-centric (hash) plans: fusion must be on (a
        fusion-off plan is the sort plan, whose shard passes take one batch), and
        the step contexts' plan mode the default (mode 1 asks for the sort plan)."""
        return getattr(self.ctxs[0], "fusion", True) and getattr(self.ctxs[0], "plan_mode", 0) == 0

    def clean(self, hp, out, rows):
        """pass 0; working-set entry w's partial clean sum -> out[rows[w]]"""
        self.ctx.shard_pass_export(self._tables(), hp, 0, out, rows)

    def set_item_delta(self, src, rows):
        """the owners' delta of working-set entry w <- src[rows[w]]"""
        self.ctx.shard_items_mapped(1, src, rows)

    def adv(self, hp, out, rows):
        self.ctx.shard_pass_export(self._tables(), hp, 1, out, rows)

    def reduce_delta(self, hp, recv, seg, pos, G0, reply):
        self.ops.shard_reduce_delta(recv, seg, pos, hp, G0, reply)

    def reduce_apply(self, hp, recv, seg, pos, G0, rows, count):
        # rows of padded segments name the trash row ni of the Q storage
        self.ops.shard_reduce_apply(self.sh._Qst, self.sh._aQst, recv, seg, pos, hp, G0, rows, count,
                                    reg_batch=self.sh.B)

    def step_errors(self) -> int:
        e = self.ctxs[0].step_errors() | self.ctxs[1].step_errors()
        return e | (self.cctx.step_errors() if self.cctx is not None else 0)


class _Chunk:
    """Host copies of one chunk's counts (the device maps live in ShardedAPR._maps[mset])."""


class _Buffers:
    """Persistent per-chunk maps and per-step exchange buffers (fixed addresses, so
    captured step graphs stay valid from one chunk to the next)."""


def _a2a_op(G, force, stage, group, out, inp, out_splits=None, in_splits=None) -> None:
    """One all_to_all_single of `inp` into `out` (a copy at world 1 unless forced;
    host-staged over gloo for device tensors: the one-GPU rehearsal of several ranks)."""
    if G == 1 and not force:
        out.copy_(inp)
    elif stage:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _hp_key(hp) -> tuple:
    return tuple(sorted((k, v) for k, v in vars(hp).items() if isinstance(v, (int, float, bool, str))))


class _SegmentRecorder:
    """Captures a step sequence as hipGraph segments cut at every collective."""

    def __init__(self, stream, pool):
        self.stream, self.pool = stream, pool
        self.segs = []  # [(graph, collective or None)]
        self._g = None

    def begin(self):
        self._g = torch.cuda.CUDAGraph()
        # thread-local: the process group's watchdog thread may query its events meanwhile
        self._g.capture_begin(pool=self.pool, capture_error_mode="thread_local")

    def cut(self, fn):
        self._g.capture_end()
        self.segs.append((self._g, fn))
        self.begin()

    def end(self):
        self._g.capture_end()
        self.segs.append((self._g, None))
        self._g = None

    def abort(self):
        """End a capture that failed half-way (the segments are dropped)."""
        if self._g is not None:
            try:
                self._g.capture_end()
            except RuntimeError:
                pass
            self._g = None
        self.segs = []

    def replay(self):
        for g, fn in self.segs:
            g.replay()
            if fn is not None:
                fn()


class ShardedAPR:
    """This rank's shard of embedding_P / embedding_Q (+ Adagrad slots) and the
    split APR step.  ``batch_size`` is the GLOBAL batch (the reference's
    ``--batch_size``); each rank processes the triplets of its users.
    ``local_batch``: triplets are routed at sampling time (train_routed), each
    rank holding exactly this many of every global batch (= G x local_batch).
    ``graph``: capture a chunk's steps as hipGraphs (None = whenever the local
    passes are the HIP ones on a GPU and the collectives are RCCL)."""

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, batch_size: int, device=None,
                 group=None, init_P=None, init_Q=None, acc0: float = 0.1, local=None,
                 local_batch: int | None = None, item_exchange: str = "all_to_all", graph: bool | None = None,
                 capture_collectives: bool | None = None, force_collectives: bool = False):
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
        # exchanges through the process group even at world 1 (RCCL self-exchange: rehearsal)
        self._force = bool(force_collectives) and not self._stage
        G, r = self.G, self.rank
        f = dict(dtype=torch.float32, device=self.device)
        nu, ni = len(range(r, self.U1, G)), len(range(r, self.I1, G))
        self.ni = ni
        self.P = torch.empty(nu, dim, **f)
        # Q / accQ storage carries one trash row (index ni) for the padded owner segments
        self._Qst = torch.zeros(ni + 1, dim, **f)
        self._aQst = torch.full((ni + 1, dim), acc0, **f)
        self.Q, self.accQ = self._Qst[:ni], self._aQst[:ni]
        if init_P is not None:
            self.P.copy_(torch.as_tensor(np.asarray(init_P, np.float32)[r::G]))
            self.Q.copy_(torch.as_tensor(np.asarray(init_Q, np.float32)[r::G]))
        self.accP = torch.full((nu, dim), acc0, **f)
        if local_batch is not None and local_batch * self.G != self.B:
            raise ValueError(f"local_batch {local_batch} x {self.G} ranks != batch_size {self.B}")
        self.b_max = int(local_batch) if local_batch is not None else self.B  # triplets of a rank per batch
        self.routed = local_batch is not None
        self.max_items = 2 * self.b_max  # a rank's working set of one batch: <= 2 x its triplets
        self.Qc = torch.zeros(self.max_items, dim, **f)
        self._qcap = (self.I1 + G - 1) // G  # rows of the largest Q shard (all_gather slots)
        gq = item_exchange == "allgather" and (G > 1 or self._force)
        self._qpad = torch.zeros(self._qcap, dim, **f) if gq else None
        self._qall = torch.empty(G * self._qcap, dim, **f) if gq else None
        # the local passes see this object through a weak proxy: no reference cycle,
        # so dropping the last reference runs the finalizer at once (see close)
        me = weakref.proxy(self)
        self.local = local(me) if local is not None else HipLocal(me)
        can_graph = (self.device.type == "cuda" and not self._stage and getattr(self.local, "graphable", False))
        self.graph = (True if graph is None else bool(graph)) and can_graph
        if capture_collectives is None:  # default off (r06): opt in with ACF_SHARD_RCCL_GRAPH=1
            capture_collectives = os.environ.get("ACF_SHARD_RCCL_GRAPH", "0") == "1"
        multi = self.G > 1 or self._force  # exchanges that are collectives
        self._multi = multi
        self._cap_coll = bool(capture_collectives) and self.graph and multi
        self._C = 0   # per-peer block rows of the exchange buffers (only grows)
        self._T = 0   # steps the per-chunk maps hold
        self._buf = None
        self._maps = None
        self._graphs = {}
        # the captured graphs (which may hold RCCL work) are dropped before the
        # process group goes: by close() / the with-block, else when this object is
        # collected, else at interpreter exit (weakref.finalize runs its atexit hook
        # before torch's process-group destructors)
        self._finalizer = weakref.finalize(self, _drop_graphs, self._graphs,
                                           self.device if self.device.type == "cuda" else None)
        self._pool = None
        self._cap_stream = None
        self._rec = None  # the segment recorder while capturing
        self.stats = {"steps": 0, "items_requested": 0, "rows_served": 0, "triplets": 0, "route_s": 0.0,
                      "graph_replays": 0}
        if self._cap_coll:  # here, where every rank is: the check is itself a collective
            self._cap_coll = self._collectives_capturable()
        # without the collectives inside (the check failed, or capture_collectives
        # off), a chunk's steps are captured as SEGMENTS cut at every collective,
        # which runs host-issued between the segment replays (_SegmentRecorder); the
        # segments are captured with the plans in line (_run_steps): r04's pipelined
        # plan forked a side stream across a cut -- unjoined work in the segment,
        # the capture failed and the RCCL call after it met a broken capture state
        # (tools/segment_capture_probe.py)
    # -- buffers -------------------------------------------------------------------
    def _ensure(self, T: int, C: int) -> None:
        if C <= self._C and T <= self._T:
            return
        if self.device.type == "cuda":  # the old buffers may still be in use by enqueued steps
            torch.cuda.synchronize(self.device)
        if C > self._C:  # headroom: chunk-to-chunk growth should not re-capture
            self._C = max(64, -(-int(C * 1.0625) // 64) * 64)
        self._T = max(self._T, T)
        self._graphs.clear()
        G, C, T, M, d = self.G, self._C, self._T, self.max_items, self.d
        GC = G * C
        dev = self.device
        li = dict(dtype=torch.int64, device=dev)
        ii = dict(dtype=torch.int32, device=dev)
        fl = dict(dtype=torch.float32, device=dev)
        maps = []
        for _ in range(2):  # chunk k routes into set k % 2 while chunk k - 1 runs on the other
            m = _Buffers()
            m.u_rows = torch.zeros(T, self.b_max, **ii)
            m.wi = torch.zeros(T, self.b_max, **ii)
            m.wj = torch.zeros(T, self.b_max, **ii)
            m.wsrc = torch.empty(T, M, **li)        # working-set entry -> its row of the exchange blocks
            m.srv = torch.empty(T, GC + 1, **li)    # exchange row -> owned Q row (trash: ni)
            m.wq = torch.empty(T, M, **li) if G == 1 else None  # world 1: working-set entry -> Q row
            m.wslot = torch.zeros(T, M, **li) if self.item_exchange == "allgather" else None
            # seg / own / count: flat storage with one dump element at the end (routing
            # scatters the entries it does not want there instead of compacting)
            m.seg_flat = torch.empty(T * (GC + 1) + 1, **ii)
            m.seg = m.seg_flat[:-1].view(T, GC + 1)
            m.dump_at = T * (GC + 1)
            m.pos = torch.zeros(T, GC, **ii)
            m.own_flat = torch.empty(T * GC + 1, **ii)
            m.own = m.own_flat[:-1].view(T, GC)
            m.dump_own = T * GC
            m.count_flat = torch.zeros(T * GC + 1, **ii)
            m.count = m.count_flat[:-1].view(T, GC)
            maps.append(m)
        self._maps = maps
        b = _Buffers()  # per-step exchange scratch (steps run one after another on one stream)
        b.S1 = torch.empty(GC + 1, d, **fl)
        b.R1 = torch.empty(GC + 1, d, **fl)
        b.S = torch.zeros(GC + 1, d, **fl)
        b.R = torch.empty(GC + 1, d, **fl)
        b.G0 = torch.empty(GC, d, **fl)
        b.reply = torch.zeros(GC + 1, d, **fl)
        b.R3 = torch.zeros(GC + 1, d, **fl)
        self._buf = b

    # -- collectives ---------------------------------------------------------------
    def _collective(self, fn) -> None:
        if self._rec is not None and not self._cap_coll:  # the collective runs between segment replays
            self._rec.cut(fn)
        else:  # eager, or captured into the graph with the local work
            fn()

    def _collectives_capturable(self) -> bool:
        """One-off check, at construction (every rank is there), that this process
        group's collectives can be captured into a graph and replayed (RCCL): an
        all_reduce captured on the capture stream, then -- only if every rank
        captured it -- replayed twice and checked.  Every rank takes the same
        decision (the graphs must hold the same collectives); on any error the
        chunks keep the collectives between graph segments."""
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
            self._cap_stream = torch.cuda.Stream(self.device)

        def agree(ok: bool) -> bool:
            flag = torch.tensor([1 if ok else 0], device=self.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            return bool(flag.item())

        x = torch.ones(64, device=self.device)
        g = torch.cuda.CUDAGraph()  # its own memory pool: the step graphs' pool stays untouched
        ok = True
        try:
            torch.cuda.synchronize(self.device)
            self._cap_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._cap_stream):
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    x.mul_(1.0)  # a node besides the collective (a one-rank RCCL all_reduce may record none)
                    dist.all_reduce(x, group=self.group)
                finally:
                    g.capture_end()
        except Exception as e:  # noqa: BLE001
            warnings.warn(f"ShardedAPR: collectives cannot be captured ({e!r}); they stay between graph segments")
            ok = False
        if not agree(ok):
            return False
        try:
            x.fill_(1.0)
            g.replay()
            g.replay()
            torch.cuda.synchronize(self.device)
            ok = bool((x == float(self.G) ** 2).all())
        except Exception as e:  # noqa: BLE001
            warnings.warn(f"ShardedAPR: a captured collective did not replay ({e!r}); collectives stay eager")
            ok = False
        del g
        return agree(ok)

    def _a2a(self, out, inp, out_splits=None, in_splits=None):
        _a2a_op(self.G, self._force, self._stage, self.group, out, inp, out_splits, in_splits)

    def _exchange(self, out, inp):
        """Fixed-size exchange of G blocks of C rows (block o to / from rank o);
        the identity at world 1.  Returns the tensor holding the received rows."""
        if self.G == 1 and not self._force:
            return inp
        n = self.G * self._C
        # the closure holds the tensors and the group, never self: a segment
        # recorder keeps it, and the finalizer's graphs must not keep this object
        # alive
        G, force, stage, group, o, x = self.G, self._force, self._stage, self.group, out[:n], inp[:n]
        self._collective(lambda: _a2a_op(G, force, stage, group, o, x))
        return out

    def _gather_q(self):
        """E1, "allgather" form: every rank's Q shard to every rank (RCCL all_gather);
        row i is then at _qall[(i % G) * cap + i // G].  World 1: Q itself."""
        if self.G == 1 and not self._force:
            return self._Qst
        self._qpad[: self.ni] = self.Q
        G, stage, group, qall, qpad, cap, d = self.G, self._stage, self.group, self._qall, self._qpad, self._qcap, self.d

        def gather():  # no reference to self (see _exchange)
            if stage:
                parts = [torch.empty(cap, d) for _ in range(G)]
                dist.all_gather(parts, qpad.cpu(), group=group)
                qall.copy_(torch.cat(parts))
            else:
                dist.all_gather_into_tensor(qall, qpad, group=group)
        self._collective(gather)
        return self._qall

    # -- routing (one chunk of T global batches) -----------------------------------
    def _route(self, u, i, j, T: int, mset: int = 0) -> _Chunk:
        G, r, I1, ni = self.G, self.rank, self.I1, self.ni
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
        c.mset = mset
        # this rank's triplets, stream order
        sel = torch.arange(u.numel(), device=dev) if self.routed else torch.nonzero(u % G == r).squeeze(1)
        st = sel // B
        n = sel.numel()
        items = torch.cat([i[sel], j[sel]])
        ist = torch.cat([st, st])
        # Working set per step: the unique items, ordered by (owner, id) so that each
        # owner's rows are one contiguous block.  No step below waits on the device
        # before the one host copy of the counts: a unique is a sort + head flags,
        # counts are scatter-adds, and arrays keep their full length (entries past
        # the U uniques are don't-cares, sliced off once U is known on the host).
        # 32-bit sort keys whenever the key range fits (half the radix passes).
        k32 = T * G * I1 < 2 ** 31
        wkey = (ist * G + items % G) * I1 + items
        sk, perm = torch.sort(wkey.to(torch.int32) if k32 else wkey)
        sk = sk.long()
        hd = torch.ones_like(sk, dtype=torch.bool)
        if sk.numel() > 1:
            hd[1:] = sk[1:] != sk[:-1]
        uid = torch.cumsum(hd, 0) - 1                       # unique index of each sorted occurrence
        inv = torch.empty_like(uid)
        inv[perm] = uid                                     # occurrence -> unique index
        uk = torch.zeros_like(sk).scatter_(0, uid, sk)      # unique keys first (same value per segment)
        valid = torch.arange(sk.numel(), device=dev) <= uid[-1:]
        wstep, wown, wid = uk // (G * I1), (uk // I1) % G, uk % I1
        ones = torch.ones_like(wstep)
        cnt = torch.zeros(T * G + 1, dtype=torch.long, device=dev).scatter_add_(
            0, torch.where(valid, wstep * G + wown, T * G), ones)[: T * G].view(T, G)
        nloc = (torch.full((T,), B, dtype=torch.long, device=dev) if self.routed else
                torch.zeros(T, dtype=torch.long, device=dev).scatter_add_(0, st, torch.ones_like(st)))
        nW = cnt.sum(1)
        wstart = torch.cumsum(nW, 0) - nW
        widx = (inv - wstart[ist]).to(torch.int32)
        wk = torch.arange(uk.numel(), device=dev) - wstart[wstep]        # entry inside its step's set
        kblk = wk - (torch.cumsum(cnt, 1) - cnt)[wstep, wown]             # entry inside its owner block
        # the requests of the whole chunk, owner-major (valid entries first), in one exchange
        if G == 1:  # the working sets are already in (owner, step, id) order
            req = wid
        else:
            okey = torch.where(valid, (wown * T + wstep) * I1 + wid, T * G * I1)
            req = (wid // G)[torch.argsort(okey.to(torch.int32) if k32 and T * G * I1 < 2 ** 31 - 1 else okey)]
        # split sizes (T per owner) + this rank's error flags + its largest request count
        # (the exchange blocks' C must be the same on every rank), to every rank in one exchange
        send = torch.cat([cnt.t(), bad.reshape(1, 1).expand(G, 1), cnt.max().reshape(1, 1).expand(G, 1)],
                         1).contiguous()
        recv = torch.empty_like(send)
        self._a2a(recv.view(-1), send.view(-1), [T + 2] * G, [T + 2] * G)
        rc = recv[:, :T]
        host = torch.cat([cnt.reshape(-1), rc.reshape(-1), nloc, recv[:, T + 1], recv[:, T]]).cpu().numpy()  # one sync
        flags = host[-G:]
        cmax = int(host[-2 * G: -G].max())  # the largest request count of any rank and step
        if flags.any():
            who = [o for o in range(G) if flags[o]]
            if np.bitwise_or.reduce(flags) & 1:
                raise IndexError(f"triplet index outside the sharded tables (rank(s) {who})")
            raise ValueError(f"train_routed: a triplet of another rank's user (rank(s) {who})")
        c.cnt = host[: T * G].reshape(T, G)           # my requests per (step, owner)
        c.rc = host[T * G: 2 * T * G].reshape(G, T)   # requests to me per (requester, step)
        c.nloc = host[2 * T * G: -2 * G]
        U = int(c.cnt.sum())                          # my working-set entries over the chunk
        self._ensure(T, max(cmax, 1))
        bf, C, M = self._maps[mset], self._C, self.max_items
        GC = G * C
        # local triplets at a fixed stride of b_max per step
        lo = torch.cumsum(nloc, 0) - nloc
        slot = st * self.b_max + (torch.arange(n, device=dev) - lo[st])
        bf.u_rows[:T].view(-1)[slot] = (u[sel] // G).to(torch.int32)
        bf.wi[:T].view(-1)[slot] = widx[:n]
        bf.wj[:T].view(-1)[slot] = widx[n:]
        # requester maps: working-set entry <-> row of the exchange blocks
        wstep, wown, wid, wk, kblk = wstep[:U], wown[:U], wid[:U], wk[:U], kblk[:U]
        xrow = wown * C + kblk
        bf.wsrc[:T].fill_(GC)
        bf.wsrc[:T].view(-1)[wstep * M + wk] = xrow
        if bf.wslot is not None:  # where each working-set row sits in the gathered table
            bf.wslot[:T].view(-1)[wstep * M + wk] = (wid % G) * self._qcap + wid // G if G > 1 else wid
        # rows I serve, received in (requester o, step t, k) order
        Rn = int(c.rc.sum())
        rows = torch.empty(Rn, dtype=req.dtype, device=dev)
        self._a2a(rows, req[:U], c.rc.sum(1).tolist(), c.cnt.sum(0).tolist())
        Rt = c.rc.sum(0)                                              # rows I serve per step (host)
        Rstart = np.concatenate([[0], np.cumsum(Rt)])
        # the host-side counts this routing needs on the device, in ONE upload
        meta = torch.as_tensor(np.concatenate([c.rc.reshape(-1), Rstart[:-1], Rt]).astype(np.int64), device=dev)
        blk_len, rstart_d, rt_d = meta[: G * T], meta[G * T: G * T + T], meta[G * T + T:]
        blk = torch.repeat_interleave(torch.arange(G * T, device=dev), blk_len, output_size=Rn)
        o_e, t_e = blk // T, blk % T
        k_e = torch.arange(Rn, device=dev) - (torch.cumsum(blk_len, 0) - blk_len)[blk]
        bf.srv[:T].fill_(ni)
        bf.srv[:T].view(-1)[t_e * (GC + 1) + o_e * C + k_e] = rows
        if bf.wq is not None:  # world 1: E1 in one gather (the exchange is the identity)
            torch.gather(bf.srv[:T], 1, bf.wsrc[:T], out=bf.wq[:T])
        # owner reduction segments: per (step, row), positions in requester order;
        # non-head entries write to the maps' dump element (no compaction, no sync)
        key = (t_e * (ni + 1) + rows) * G + o_e
        if G == 1:  # the requests are the working sets, already in (step, row) order: no sort
            skey, sp = key, torch.arange(Rn, device=dev)
        else:
            skey, sp = torch.sort(key.to(torch.int32) if T * (ni + 1) * G < 2 ** 31 else key)
            skey = skey.long()
        srow = skey // G
        head = torch.ones_like(srow, dtype=torch.bool)
        if srow.numel() > 1:
            head[1:] = srow[1:] != srow[:-1]
        ts = t_e[sp]
        hcum = torch.zeros(Rn + 1, dtype=torch.long, device=dev)
        hcum[1:] = torch.cumsum(head.long(), 0)                       # heads before each position
        segstart = hcum[rstart_d]                                     # first segment of each step
        p_in = torch.arange(Rn, device=dev) - rstart_d[ts]
        s_in = hcum[1:] - 1 - segstart[ts]
        bf.pos[:T].view(-1)[ts * GC + p_in] = (o_e * C + k_e)[sp].to(torch.int32)
        bf.seg[:T].copy_(rt_d.to(torch.int32)[:, None].expand(T, GC + 1))
        dump = bf.dump_at
        bf.seg_flat[torch.where(head, ts * (GC + 1) + s_in, dump)] = p_in.to(torch.int32)
        bf.own[:T].fill_(ni)
        c.own_rows = srow % (ni + 1)
        c.own_flat = torch.where(head, ts * GC + s_in, bf.dump_own)
        bf.own_flat[c.own_flat] = c.own_rows.to(torch.int32)
        c.has_count = False
        c.R = Rt                                          # rows I serve per step
        c.nW = c.cnt.sum(1)
        self._chunk_items = (i, j)
        return c

    def _counts(self, c: _Chunk, i, j) -> None:
        """Occurrences of every owned row of each step in the GLOBAL batch (the
        reg * mean(w^2) gradient counts them, APR.py:153-154)."""
        G, B, T = self.G, self.B, c.T
        items = torch.cat([i, j])
        st = torch.cat([torch.arange(T * B, device=self.device) // B] * 2)
        nrow = self.ni + 1
        # other ranks' items count into the trash row ni of their step (never read)
        local = torch.where(items % G == self.rank, items // G, self.ni)
        cnt = torch.zeros(T * nrow, dtype=torch.long, device=self.device).scatter_add_(
            0, st * nrow + local, torch.ones_like(st))
        m = self._maps[c.mset]
        seg_step = torch.clamp(c.own_flat // (G * self._C), max=T - 1)
        m.count[:T].zero_()
        m.count_flat[c.own_flat] = cnt[seg_step * nrow + c.own_rows].to(torch.int32)
        c.has_count = True

    # -- one step ------------------------------------------------------------------
    def _pipelined(self) -> bool:
        """The next step's plan beside this step: the local passes support it.  In
        a whole-chunk capture (collectives inside the graph, or none: world 1) the
        side-stream plan is a branch of the captured graph, forked and joined by
        events; a segment capture plans in line instead (_run_steps)."""
        return getattr(self.local, "pipelined", False)

    def _plan_step(self, m, t: int, nb: list, pipe: bool) -> None:
        """The plan of step t (nb[t] local triplets): in line, or -- pipelined -- the
        one made beside step t - 1 (step 0's in line), then step t + 1's forked
        onto the side stream once step t - 1 has released its context."""
        b = nb[t]
        if not pipe:
            self.local.plan(m.u_rows[t, :b], m.wi[t, :b], m.wj[t, :b])
            return
        main = torch.cuda.current_stream(self.device)
        k = t & 1
        if t == 0 or self._planned[k] is None:
            self.local.plan_into(k, m.u_rows[t, :b], m.wi[t, :b], m.wj[t, :b])
        else:
            main.wait_event(self._planned[k])
        self._planned[k] = None
        self.local.use(k)
        T = len(nb)
        if t + 1 < T and nb[t + 1]:
            k1 = k ^ 1
            side = self._plan_stream
            fork = self._free[k1]
            if fork is None:  # nothing used that context yet in this chunk: fork from here
                fork = torch.cuda.Event()
                fork.record(main)
            side.wait_event(fork)
            with torch.cuda.stream(side):
                b1 = nb[t + 1]
                self.local.plan_into(k1, m.u_rows[t + 1, :b1], m.wi[t + 1, :b1], m.wj[t + 1, :b1])
                ev = torch.cuda.Event()
                ev.record(side)
            self._planned[k1] = ev

    def _release(self, t: int, pipe: bool) -> None:
        """Step t's last use of its context: the plan of step t + 2 may overwrite it."""
        if pipe:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._free[t & 1] = ev

    def _step(self, m, t: int, nb: list, hp, count: bool, pipe: bool = False, chunk: bool = False) -> None:
        """Step t of a chunk routed into map set m (fixed shapes: every size is the buffers')."""
        b = nb[t]
        bf = self._buf
        # E1: current item rows of my working set from their owners
        if self.item_exchange == "allgather":
            torch.index_select(self._gather_q(), 0, m.wslot[t], out=self.Qc)
        elif m.wq is not None and not self._force:
            torch.index_select(self._Qst, 0, m.wq[t], out=self.Qc)
        else:
            torch.index_select(self._Qst, 0, m.srv[t], out=bf.S1)
            torch.index_select(self._exchange(bf.R1, bf.S1), 0, m.wsrc[t], out=self.Qc)
        rows = m.wsrc[t, : 2 * b]  # working-set entry -> its exchange row
        if b:
            if chunk:  # batch t of the chunk's plan (_run_steps)
                self.local.use_batch(t)
            else:
                self._plan_step(m, t, nb, pipe)
            self.local.clean(hp, bf.S, rows)
            if not hp.adver:
                self._release(t, pipe)
        # E2: partial clean item sums -> owners
        recv = self._exchange(bf.R, bf.S)
        cnt = m.count[t] if count else None
        if hp.adver:
            self.local.reduce_delta(hp, recv, m.seg[t], m.pos[t], bf.G0, bf.reply)
            # E3: deltas -> requesters
            dl = self._exchange(bf.R3, bf.reply)
            if b:
                self.local.set_item_delta(dl, rows)
                self.local.adv(hp, bf.S, rows)
                self._release(t, pipe)
            # E4: partial adversarial item sums -> owners, who apply Adagrad
            recv = self._exchange(bf.R, bf.S)
            self.local.reduce_apply(hp, recv, m.seg[t], m.pos[t], bf.G0, m.own[t], cnt)
        else:
            self.local.reduce_apply(hp, recv, m.seg[t], m.pos[t], None, m.own[t], cnt)

    def _run(self, c: _Chunk, hp) -> None:
        T = c.T
        bs = set(int(x) for x in c.nloc)
        key = None
        if self.graph and len(bs) == 1 and min(bs) > 0:
            key = (c.mset, T, min(bs), self._C, c.has_count, _hp_key(hp))
        rec = self._graphs.get(key) if key is not None else None
        if rec is not None:
            rec.replay()
            self.stats["graph_replays"] += 1
            return
        m = self._maps[c.mset]
        self._run_steps(m, [int(x) for x in c.nloc[:T]], hp, c.has_count)
        if key is not None:  # capture for the next chunk of this shape (capturing runs nothing)
            try:
                self._graphs[key] = self._capture(m, T, min(bs), hp, c.has_count)
            except RuntimeError as e:  # the chunk ran eagerly; later chunks stay eager
                warnings.warn(f"ShardedAPR: step capture failed ({e}); continuing without graphs")
                self.graph = False

    def _run_steps(self, m, nb: list, hp, count: bool) -> None:
        """The steps of a chunk, each step's plan beside the previous step where
        the local passes allow it (_pipelined)."""
        # never across a segment cut (see the constructor): plans in line while
        # capturing segments; eager runs and whole-step graphs keep the pipeline
        # (world 1 without forced collectives has no cut: one graph, pipelined)
        segments = self._rec is not None and not self._cap_coll and self._multi
        # (r06) equal local batches: the whole chunk in ONE plan, in line at its
        # start (the one-batch plans beside every step cost ~150 us of GPU time per
        # configs[4] step; at configs[2] k_shard_plan's ~22 us per step)
        chunk = (getattr(self.local, "chunk_planned", False) and len(nb) > 1 and len(set(nb)) == 1
                 and nb[0] > getattr(self.local, "chunk_min", 1024) and self.local.chunk_ok())
        pipe = self.device.type == "cuda" and self._pipelined() and not segments and not chunk
        if pipe and getattr(self, "_plan_stream", None) is None:
            self._plan_stream = torch.cuda.Stream(self.device)
        self._planned, self._free = [None, None], [None, None]
        if chunk:
            T, b = len(nb), nb[0]
            self.local.plan_chunk(m.u_rows[:T, :b], m.wi[:T, :b], m.wj[:T, :b])
        for t in range(len(nb)):
            self._step(m, t, nb, hp, count, pipe, chunk)
        self._planned, self._free = [None, None], [None, None]

    def _capture(self, m, T: int, b: int, hp, count: bool) -> _SegmentRecorder:
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
            self._cap_stream = torch.cuda.Stream(self.device)
        main = torch.cuda.current_stream(self.device)
        rec = _SegmentRecorder(self._cap_stream, self._pool)
        torch.cuda.synchronize(self.device)
        self._cap_stream.wait_stream(main)
        with torch.cuda.stream(self._cap_stream):
            self._rec = rec
            try:
                rec.begin()
                self._run_steps(m, [b] * T, hp, count)
                rec.end()
            except BaseException:
                rec.abort()
                raise
            finally:
                self._rec = None
        main.wait_stream(self._cap_stream)
        return rec

    # -- public --------------------------------------------------------------------
    def train(self, u, i, j, hp, chunk: int = 64) -> int:
        """Train consecutive global batches of the stream (u, i, j), identical on
        every rank (length a multiple of the batch size; train_routed: this rank's
        triplets only, local_batch per batch).  Returns the batches run.

        On a GPU the routing of chunk k + 1 runs on a side stream while chunk k's
        steps run on the caller's stream (the two chunks use the two map sets).
        That overlap is complete only at world 1: above it, the routing's count
        and row all_to_alls go through the same process group as chunk k's step
        collectives, so they queue behind them (and the routing's host copy of
        the counts waits for most of chunk k); the split-step figures of DESIGN
        §7 are world-1 measurements."""
        bs = self.b_max if self.routed else self.B
        n = len(u) // bs
        spans = [(c0, min(chunk, n - c0)) for c0 in range(0, n, chunk)]
        cuda = self.device.type == "cuda"
        main = torch.cuda.current_stream(self.device) if cuda else None
        if cuda and getattr(self, "_route_stream", None) is None:
            self._route_stream = torch.cuda.Stream(self.device)
        side = self._route_stream if cuda else None
        done = [None, None]  # event after the last chunk enqueued on map set k % 2

        def route(k):
            c0, T = spans[k]
            s = slice(c0 * bs, (c0 + T) * bs)
            t0 = time.perf_counter()
            if cuda:
                if k == 0:  # the triplets come from the caller's stream
                    side.wait_stream(main)
                if done[k % 2] is not None:  # the set's previous chunk has run
                    side.wait_event(done[k % 2])
                with torch.cuda.stream(side):
                    c = self._route(u[s], i[s], j[s], T, k % 2)
                    if hp.reg:
                        self._reg_counts(c)
                    c.ready = torch.cuda.Event()
                    c.ready.record(side)
            else:
                c = self._route(u[s], i[s], j[s], T, k % 2)
                if hp.reg:
                    self._reg_counts(c)
            self.stats["route_s"] += time.perf_counter() - t0
            return c

        c = route(0) if spans else None
        for k in range(len(spans)):
            if cuda:
                main.wait_event(c.ready)
            self._run(c, hp)
            if cuda:
                done[k % 2] = torch.cuda.Event()
                done[k % 2].record(main)
            st = self.stats
            st["steps"] += c.T
            st["items_requested"] += int(c.nW.sum())
            st["rows_served"] += int(c.R.sum())
            st["triplets"] += int(c.nloc.sum())
            if k + 1 < len(spans):
                c = route(k + 1)
        return n

    def _reg_counts(self, c: _Chunk) -> None:
        # the owners count their rows in the GLOBAL batch
        if self.routed:
            raise ValueError("reg != 0 needs the global stream on every rank (train, not train_routed)")
        self._counts(c, *self._chunk_items)

    def train_routed(self, u, i, j, hp, chunk: int = 64) -> int:
        """As train, for triplets routed at sampling time: this rank's users only,
        local_batch of them per global batch (the sampler runs per rank)."""
        if not self.routed:
            raise ValueError("train_routed needs ShardedAPR(local_batch=...)")
        return self.train(u, i, j, hp, chunk)

    def step_errors(self) -> int:
        return self.local.step_errors() if hasattr(self.local, "step_errors") else 0

    def close(self) -> None:
        """Drop the captured step graphs (before the process group is destroyed: a
        graph holding captured RCCL collectives keeps the communicator busy).  Also
        run by the with-block, when the object is collected, and at exit."""
        self._finalizer()

    def __enter__(self) -> "ShardedAPR":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

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
