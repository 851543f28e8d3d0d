"""Torch-tensor front end of the C-ABI.

PyTorch provides device memory and the current HIP stream; every computation runs
in ``libacf_apr.so``.  Arguments are validated here the way TF validated feeds
(dtype/shape/device errors raise ``TypeError``/``ValueError`` before any launch);
index ranges are validated on device by the plan / sampler (``NativeIndexError``).
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass

import torch

from . import _native
from ._native import HParams, Tables, call

CLIP_LO = -80.0   # APR.py:148
CLIP_HI = 1e8


class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL = _Null()


def _on(device: torch.device):
    """torch.cuda.device(device) unless it is already current (a few us saved per call)."""
    return _NULL if torch.cuda.current_device() == device.index else torch.cuda.device(device)


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_RAW = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _raw_stream(device: torch.device) -> int:
    """The current stream of `device` as an integer handle (torch's raw accessor:
    no Stream object per call)."""
    return _RAW(device.index) if _RAW is not None else _stream_ptr(device)


def _require(t: torch.Tensor, name: str, dtype: torch.dtype, device: torch.device | None = None,
             ndim: int | None = None) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must live on a HIP device (got {t.device}); there is no CPU path")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t.data_ptr()


def _idx(t, name, device) -> torch.Tensor:
    """Accept [N] or [N,1] int tensors/arrays (the placeholders are [None,1])."""
    if (isinstance(t, torch.Tensor) and t.dtype == torch.int32 and t.dim() == 1 and t.device == device
            and t.is_contiguous()):
        return t
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    t = t.reshape(-1)
    if t.dtype != torch.int32:
        t = t.to(torch.int32)
    return t.to(device, non_blocking=True).contiguous()


class StepWaitError(RuntimeError):
    """A streamed step gave up waiting for a row (ACF_SPIN_LIMIT
    polls): the tables of that call hold stale rows and must not be trusted."""

    def __init__(self, bits: int):
        self.bits = int(bits)
        super().__init__(f"step error word {bits:#x}: a step kernel gave up waiting for a row version; "
                         "the tables of this call are not trustworthy")


@dataclass
class StepHParams:
    """Hyper-parameters of one MF graph (APR.py:86-97)."""
    lr: float = 0.05
    eps: float = 0.5
    reg: float = 0.0
    reg_adv: float = 1.0
    adver: int = 0
    adv: str = "grad"        # "grad" | "random" (APR.py:170-191)
    seed: int = 0
    zero_delta: int = 0
    clip_lo: float = CLIP_LO
    clip_hi: float = CLIP_HI

    def to_c(self) -> HParams:
        key = (self.lr, self.eps, self.reg, self.reg_adv, self.adver, self.adv, self.seed, self.zero_delta,
               self.clip_lo, self.clip_hi)
        c = self.__dict__.get("_c")
        if c is not None and c[0] == key:
            return c[1]
        if self.adv not in ("grad", "random"):
            raise ValueError(f"adv must be 'grad' or 'random', got {self.adv!r}")
        h = HParams(self.lr, self.eps, self.reg, self.reg_adv, self.clip_lo, self.clip_hi,
                    int(bool(self.adver)), 0 if self.adv == "grad" else 1,
                    int(self.seed) & 0xFFFFFFFFFFFFFFFF, int(bool(self.zero_delta)), 0)
        self.__dict__["_c"] = (key, h)
        return h


class APRContext:
    """Owns an ``acf_apr_ctx``: plan workspace, per-batch scratch, graph cache."""

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, max_batch_size: int,
                 max_batches: int, device: torch.device):
        self.device = torch.device(device)
        self.U1, self.I1, self.d = int(num_user_rows), int(num_item_rows), int(dim)
        self.max_batch_size, self.max_batches = int(max_batch_size), int(max_batches)
        self._ptr = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("acf_apr_create", ctypes.byref(self._ptr), self.U1, self.I1, self.d,
                 self.max_batch_size, self.max_batches)
        self.batch_size = 0
        self.n_batches = 0
        self._staged = None
        self._tb_key, self._tb = None, None

    def __del__(self):
        try:
            if self._ptr:
                _native.load().acf_apr_destroy(self._ptr)
                self._ptr = ctypes.c_void_p()
        except Exception:
            pass

    def fits(self, batch_size: int, n_batches: int) -> bool:
        return batch_size <= self.max_batch_size and n_batches <= self.max_batches

    def plan(self, user, item_pos, item_neg, batch_size: int, check: bool = True) -> int:
        """Stage triplets and build the dedup plan; returns the number of batches."""
        u = _idx(user, "user", self.device)
        i = _idx(item_pos, "item_pos", self.device)
        j = _idx(item_neg, "item_neg", self.device)
        if not (u.numel() == i.numel() == j.numel()):
            raise ValueError(f"triplet lengths differ: {u.numel()}, {i.numel()}, {j.numel()}")
        if batch_size <= 0 or u.numel() % batch_size:
            raise ValueError(f"{u.numel()} triplets is not a multiple of batch_size {batch_size}")
        nb = u.numel() // batch_size
        if not self.fits(batch_size, nb):
            raise ValueError(f"plan of {nb} x {batch_size} exceeds context capacity "
                             f"{self.max_batches} x {self.max_batch_size}")
        with torch.cuda.device(self.device):
            call("acf_apr_plan", self._ptr, u.data_ptr(), i.data_ptr(), j.data_ptr(), batch_size, nb,
                 int(check), _stream_ptr(self.device))
        self._staged = (u, i, j)  # keep alive until the stream has consumed them
        self.batch_size, self.n_batches = batch_size, nb
        return nb

    def _tables(self, P, Q, accP, accQ) -> Tables:
        # the same storage, shape, strides and dtype as the last validated call (the
        # device cannot differ at the same address)
        key = (P.data_ptr(), Q.data_ptr(), accP.data_ptr(), accQ.data_ptr(), P.shape, Q.shape, accP.shape,
               accQ.shape, P.stride(), Q.stride(), accP.stride(), accQ.stride(), P.dtype, Q.dtype, accP.dtype,
               accQ.dtype)
        if self._tb_key == key:
            return self._tb
        for t, n, rows in ((P, "embedding_P", self.U1), (Q, "embedding_Q", self.I1),
                           (accP, "accumulator_P", self.U1), (accQ, "accumulator_Q", self.I1)):
            _require(t, n, torch.float32, self.device, 2)
            if tuple(t.shape) != (rows, self.d):
                raise ValueError(f"{n} has shape {tuple(t.shape)}, expected {(rows, self.d)}")
        self._tb = Tables(P.data_ptr(), Q.data_ptr(), accP.data_ptr(), accQ.data_ptr())
        self._tb_key = key
        return self._tb

    def train_range(self, tables, hp: StepHParams, user: torch.Tensor, item_pos: torch.Tensor,
                    item_neg: torch.Tensor, batch_size: int, first_batch: int, n_batches: int,
                    graph: bool = True, check: bool = False, _checked: bool = False) -> None:
        """plan + train_planned of batches [first_batch, first_batch + n_batches) of
        device int32 triplet streams, in ONE C call (acf_apr_train); the range is
        addressed in place (no slicing).  (_checked: the caller, PlanPipeline.run,
        has validated the three streams and the range.)"""
        B, nb = int(batch_size), int(n_batches)
        if not _checked:
            for t, n in ((user, "user"), (item_pos, "item_pos"), (item_neg, "item_neg")):
                if t.dtype != torch.int32 or t.device != self.device or not t.is_contiguous() or t.dim() != 1:
                    raise ValueError(f"{n} must be a contiguous 1-D int32 tensor on {self.device}")
                if (first_batch + nb) * B > t.numel() or first_batch < 0:
                    raise ValueError(f"batches [{first_batch}, {first_batch + nb}) outside {n}")
        if not self.fits(B, nb):
            raise ValueError(f"plan of {nb} x {B} exceeds context capacity {self.max_batches} x "
                             f"{self.max_batch_size}")
        tb, h = self._tables(*tables), hp.to_c()
        off = first_batch * B * 4
        with _on(self.device):
            call("acf_apr_train", self._ptr, ctypes.byref(tb), ctypes.byref(h), user.data_ptr() + off,
                 item_pos.data_ptr() + off, item_neg.data_ptr() + off, B, nb, int(check), int(bool(graph)),
                 torch.cuda.current_stream(self.device).cuda_stream)
        self._staged = (user, item_pos, item_neg)
        self.batch_size, self.n_batches = B, nb

    def delta_update(self, tables, hp: StepHParams, batch: int) -> None:
        tb, h = self._tables(*tables), hp.to_c()
        with torch.cuda.device(self.device):
            call("acf_apr_delta_update", self._ptr, ctypes.byref(tb), ctypes.byref(h), batch,
                 _stream_ptr(self.device))

    def optimizer_step(self, tables, hp: StepHParams, batch: int) -> None:
        tb, h = self._tables(*tables), hp.to_c()
        with torch.cuda.device(self.device):
            call("acf_apr_optimizer_step", self._ptr, ctypes.byref(tb), ctypes.byref(h), batch,
                 _stream_ptr(self.device))

    def train_planned(self, tables, hp: StepHParams, first: int = 0, n: int | None = None,
                      graph: bool = True) -> None:
        n = self.n_batches - first if n is None else n
        tb, h = self._tables(*tables), hp.to_c()
        with torch.cuda.device(self.device):
            call("acf_apr_train_planned", self._ptr, ctypes.byref(tb), ctypes.byref(h), first, n,
                 int(bool(graph)), _stream_ptr(self.device))

    def set_slot_mapping(self, mode: str | int) -> None:
        """'auto' | 'wave' (one wavefront per unique row) | 'group' (one lane-group per row)."""
        m = {"auto": 0, "wave": 1, "group": 2}.get(mode, mode)
        call("acf_apr_set_slot_mapping", self._ptr, int(m))

    def set_plan_mode(self, mode: str | int) -> None:
        """'auto' (batch-local plan where it applies: one-wave-per-slot plans of
        batches <= 1,024) | 'sort' (always the device-wide sort plan).  Both
        write identical plans; 'sort' is for A/B and the equivalence test."""
        m = {"auto": 0, "sort": 1}.get(mode, mode)
        call("acf_apr_set_plan_mode", self._ptr, int(m))
        self.plan_mode = int(m)

    PLAN_KINDS = {-1: None, 0: "sort", 1: "batch", 2: "shard", 3: "hash"}

    def plan_kind(self) -> str | None:
        """The planner the last plan() used: 'sort' (device-wide radix sort),
        'batch' (batch-local, B <= 1,024), 'shard' (one-workgroup shard plan) or
        'hash' (triplet-centric plans); None before any plan."""
        return self.PLAN_KINDS[_native.load().acf_apr_plan_kind(self._ptr)]

    def set_fusion(self, on: bool) -> None:
        """Fuse triplets whose three rows occur once in their batch (default on;
        identical results either way).  Applies to train_planned / time_kernels;
        for large batches (one lane-group per slot) set it before plan(): a plan
        made with fusion on is triplet-centric and updates every row in place, and
        training it with fusion off raises."""
        call("acf_apr_set_fusion", self._ptr, int(bool(on)))
        self.fusion = bool(on)

    def time_kernels(self, tables, hp: StepHParams, first: int = 0, n: int | None = None):
        """Per-kernel-kind device time (ms) and launch counts over planned batches,
        measured with start/stop events attached to each launch of the sequence
        train_planned runs (tables are trained exactly as by it).  Kinds: clean
        (phase 1, or the fused BPR step), adv (phase 2 + Adagrad), flush
        (end-of-call write-back), stream (the whole range in one launch,
        k_stream), hot (the hot-slot combine of large-batch plans)."""
        n = self.n_batches - first if n is None else n
        tb, h = self._tables(*tables), hp.to_c()
        ms = (ctypes.c_double * 6)()
        cnt = (ctypes.c_int32 * 6)()
        with torch.cuda.device(self.device):
            call("acf_apr_time_kernels", self._ptr, ctypes.byref(tb), ctypes.byref(h), first, n, ms, cnt,
                 _stream_ptr(self.device))
        # (slot 3 was the overlapped step k_ovl, removed in r05)
        return {k: (ms[x], cnt[x]) for x, k in enumerate(("clean", "adv", "flush", None, "stream", "hot")) if k}

    def set_stream(self, on: bool) -> None:
        """Streamed APR steps (default on; identical results either way): one
        launch runs the whole batch range through tagged row versions."""
        call("acf_apr_set_stream", self._ptr, int(bool(on)))

    def set_failsafe(self, on: bool) -> None:
        """Verified streamed steps (default on): a streamed call stays asynchronous
        and is queued; if a hand-off wait gave up (k_stream needs all its waves
        resident), the call applied nothing and gated the later streamed calls of
        its group, and the next settling point (resolve(), step_errors(),
        stream_recoveries(), losses(), a re-plan of this context, ...) replays
        them in order on the two-kernel schedule -- exact.  Off: a give-up is
        reported by step_errors() and that call is not applied."""
        call("acf_apr_set_failsafe", self._ptr, int(bool(on)))

    def resolve(self) -> None:
        """Settle the queued streamed calls of this context's group (blocking)."""
        call("acf_apr_resolve", self._ptr)

    def share_failsafe(self, peer: "APRContext") -> None:
        """Verify this context's streamed calls together with peer's (contexts
        training the same tables on one stream)."""
        call("acf_apr_share_failsafe", self._ptr, peer._ptr)

    def set_spin_limit(self, polls: int) -> None:
        """Version polls before a k_stream wait gives up (default 65,536; tests use
        0 to force the replay)."""
        call("acf_apr_set_spin_limit", self._ptr, int(polls))

    def stream_recoveries(self) -> int:
        """Streamed calls replayed on the two-kernel schedule so far."""
        out = ctypes.c_int64(0)
        call("acf_apr_stream_recoveries", self._ptr, ctypes.byref(out))
        return int(out.value)

    # -- shard mode (distributed.ShardedAPR; include/acf_apr.h "shard mode") --------
    def set_shard_mode(self, on: bool, reg_batch: int = 0) -> None:
        """Item rows are this rank's partial sums (one lane-group per slot, no
        fusion, one-batch plans); reg_batch = the global batch of the reg mean."""
        call("acf_apr_set_shard_mode", self._ptr, int(bool(on)), int(reg_batch))
        self.batch_size = self.n_batches = 0

    def set_shard_batch(self, t: int) -> None:
        """The plan's batch the next shard passes step (a triplet-centric shard
        plan may hold a chunk of steps; 0 otherwise)."""
        call("acf_apr_set_shard_batch", self._ptr, int(t))

    def shard_pass(self, tables, hp: StepHParams, pass_: int) -> None:
        """pass 0: clean sums (users: delta; items: partial sums); pass 1 (APR):
        adversarial sums, user Adagrad + write-back."""
        tb, h = self._tables(*tables), hp.to_c()
        with torch.cuda.device(self.device):
            call("acf_apr_shard_pass", self._ptr, ctypes.byref(tb), ctypes.byref(h), int(pass_),
                 _stream_ptr(self.device))

    def shard_pass_export(self, tables, hp: StepHParams, pass_: int, buf: torch.Tensor, rows: torch.Tensor) -> None:
        """shard_pass, with working-set entry w's partial item sum also written to
        buf[rows[w]] by the pass's own launches (the split step's exchange rows)."""
        tb, h = self._tables(*tables), hp.to_c()
        _require(buf, "buf", torch.float32, self.device, 2)
        _require(rows, "rows", torch.int64, self.device, 1)
        with torch.cuda.device(self.device):
            call("acf_apr_shard_pass_export", self._ptr, ctypes.byref(tb), ctypes.byref(h), int(pass_),
                 buf.data_ptr(), rows.data_ptr(), rows.numel(), _stream_ptr(self.device))

    def shard_items_out(self, out: torch.Tensor) -> None:
        """The item slots' partial sums (working-set order) -> out [n_items, d]."""
        _require(out, "out", torch.float32, self.device, 2)
        with torch.cuda.device(self.device):
            call("acf_apr_shard_items", self._ptr, 0, out.data_ptr(), out.shape[0], _stream_ptr(self.device))

    def shard_items_delta(self, delta: torch.Tensor) -> None:
        """The owners' deltas [n_items, d] (working-set order) -> the item slots."""
        _require(delta, "delta", torch.float32, self.device, 2)
        with torch.cuda.device(self.device):
            call("acf_apr_shard_items", self._ptr, 1, delta.data_ptr(), delta.shape[0], _stream_ptr(self.device))

    def shard_items_mapped(self, dir_: int, buf: torch.Tensor, rows: torch.Tensor) -> None:
        """Working-set entry w <-> row rows[w] of buf, for w < rows.numel(): dir 0
        writes the item slots' partial sums there, dir 1 takes the owners'
        deltas from there (the split step's exchange rows)."""
        _require(buf, "buf", torch.float32, self.device, 2)
        _require(rows, "rows", torch.int64, self.device, 1)
        with torch.cuda.device(self.device):
            call("acf_apr_shard_items_mapped", self._ptr, int(dir_), buf.data_ptr(), rows.data_ptr(), rows.numel(),
                 _stream_ptr(self.device))

    def step_errors(self) -> int:
        """Read and clear the step error words (bit 0: an overlapped step gave up
        waiting for a row, or an unverified streamed call gave up -- set_failsafe)."""
        out = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            call("acf_apr_step_errors", self._ptr, ctypes.byref(out), _stream_ptr(self.device))
        return int(out.value)

    def losses(self):
        """Per-triplet (clean, adversarial) softplus terms of the last steps."""
        n = self.batch_size * self.n_batches
        lc = torch.empty(n, dtype=torch.float32, device=self.device)
        la = torch.empty(n, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            call("acf_apr_copy_losses", self._ptr, lc.data_ptr(), la.data_ptr(),
                 _stream_ptr(self.device))
        return lc, la

    def delta_tables(self):
        """Dense delta_P / delta_Q of the last delta_update (zeros elsewhere)."""
        dP = torch.zeros(self.U1, self.d, dtype=torch.float32, device=self.device)
        dQ = torch.zeros(self.I1, self.d, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            call("acf_apr_delta_scatter", self._ptr, dP.data_ptr(), dQ.data_ptr(),
                 _stream_ptr(self.device))
        return dP, dQ


class PlanPipeline:
    """training_batch's epoch loop with the dedup plan off the critical path.

    A long triplet stream is trained in chunks of ``chunk`` batches.  The plan of
    chunk c+1 (sort / dedup / records — it reads triplets only, never the tables)
    runs on a side stream while chunk c trains on the caller's stream; two
    contexts alternate so a plan never overwrites records still in use.  Chunks
    are independent calls of train_planned (each ends with its flush), so the
    result is the one of planning and training the chunks in sequence.

    overlap=False plans on the caller's stream instead.  overlap=None (default)
    decides per run: concurrent planning for large batches (B >= 4,096: the
    device-wide sort plan, ~40 us per batch); in line for smaller ones, whose
    batch-local plan (two launches per chunk) costs less than the
    events and stream hand-offs of planning beside the step, and never shares
    the device with the persistent k_stream.  A run of a single chunk always
    plans in line.
    """

    def __init__(self, num_user_rows: int, num_item_rows: int, dim: int, batch_size: int,
                 chunk: int, device: torch.device, overlap: bool | None = True):
        self.device = torch.device(device)
        self.overlap = None if overlap is None else bool(overlap)
        self._ov = bool(overlap)  # the current run's choice
        self.batch_size, self.chunk = int(batch_size), int(chunk)
        self.ctx = [APRContext(num_user_rows, num_item_rows, dim, batch_size, chunk, self.device)
                    for _ in range(2)]
        self.ctx[1].share_failsafe(self.ctx[0])  # one verification queue for both (acf_apr.h)
        # default priority: a high-priority plan stream halved the configs[4] rate
        # (608M -> 313M triplets/s at d = 64, tools/large_prio.py, r03)
        # (the steps on a high-priority stream instead, the plan filling what they
        # leave idle, was 1.8x slower at configs[4]: 775M -> 424M triplets/s, r04)
        self.side = torch.cuda.Stream(self.device)
        self._free = [None, None]  # event: the last training on ctx[k] has been issued before it
        self._memo = None  # the last single-chunk call, validated (_repeat)

    def set_fusion(self, on: bool) -> None:
        for c in self.ctx:
            c.set_fusion(on)

    def set_stream(self, on: bool) -> None:
        for c in self.ctx:
            c.set_stream(on)

    def step_errors(self) -> int:
        e = 0
        for c in self.ctx:
            e |= c.step_errors()
        return e

    def set_failsafe(self, on: bool) -> None:
        for c in self.ctx:
            c.set_failsafe(on)

    def set_spin_limit(self, polls: int) -> None:
        for c in self.ctx:
            c.set_spin_limit(polls)

    def stream_recoveries(self) -> int:
        return sum(c.stream_recoveries() for c in self.ctx)

    def resolve(self) -> None:
        self.ctx[0].resolve()

    def set_slot_mapping(self, mode) -> None:
        for c in self.ctx:
            c.set_slot_mapping(mode)

    def set_plan_mode(self, mode) -> None:
        for c in self.ctx:
            c.set_plan_mode(mode)

    def _remember(self, tables, hp, user, item_pos, item_neg, first_batch, n_arg, n_batches, graph) -> None:
        c = self.ctx[0]
        P, Q, aP, aQ = tables
        tb, h = c._tables(P, Q, aP, aQ), hp.to_c()
        off = first_batch * self.batch_size * 4
        args = (c._ptr, ctypes.byref(tb), ctypes.byref(h), user.data_ptr() + off, item_pos.data_ptr() + off,
                item_neg.data_ptr() + off, self.batch_size, n_batches, 0, int(bool(graph)))
        self._memo = (user, item_pos, item_neg, hp, first_batch, n_arg, graph, P, Q, aP, aQ, dict(hp.__dict__),
                      (P.data_ptr(), Q.data_ptr(), aP.data_ptr(), aQ.data_ptr(), user.data_ptr(),
                       item_pos.data_ptr(), item_neg.data_ptr()),
                      _native.load().acf_apr_train, args, c, tb, h)

    def _plan(self, k, u, i, j, b, n, check):
        B, c = self.batch_size, self.ctx[k % 2]
        s = slice(b * B, (b + n) * B)
        if not self._ov:
            c.plan(u[s], i[s], j[s], B, check=check)
            return None
        with torch.cuda.stream(self.side):
            if self._free[k % 2] is not None:
                self.side.wait_event(self._free[k % 2])
            c.plan(u[s], i[s], j[s], B, check=check)
            ev = torch.cuda.Event()
            ev.record(self.side)
        return ev

    def _repeat(self, tables, hp, user, item_pos, item_neg, first_batch, n_batches, graph) -> bool:
        """The exact call the last run made (same tensor objects, storage, shapes
        and hyper-parameters; one chunk): issue it straight to the C-ABI with the
        arguments validated then.  Saves the per-call validation (~10 us of host
        time in front of the first kernel of a short call)."""
        m = self._memo
        if not (m[0] is user and m[1] is item_pos and m[2] is item_neg and m[3] is hp and m[4] == first_batch
                and m[5] == n_batches and m[6] == graph):
            return False
        P, Q, aP, aQ = tables
        # the same tensor objects on the same storage (a storage swap moves data_ptr)
        # and the same hyper-parameters; the launches go to the device's current
        # stream, which selects the device
        if not (P is m[7] and Q is m[8] and aP is m[9] and aQ is m[10] and hp.__dict__ == m[11]
                and m[12] == (P.data_ptr(), Q.data_ptr(), aP.data_ptr(), aQ.data_ptr(), user.data_ptr(),
                              item_pos.data_ptr(), item_neg.data_ptr())):
            return False
        fn, args, ctx = m[13], m[14], m[15]
        rc = fn(*args, _raw_stream(self.device))
        if rc:
            _native.call_failed(rc, "acf_apr_train")
        ctx._staged = (user, item_pos, item_neg)
        return True

    def run(self, tables, hp: StepHParams, user, item_pos, item_neg, first_batch: int = 0,
            n_batches: int | None = None, graph: bool = True, check: bool = False) -> None:
        """Train batches [first_batch, first_batch + n_batches) of the stream."""
        if self._memo is not None and not check and self._repeat(tables, hp, user, item_pos, item_neg, first_batch,
                                                                 n_batches, graph):
            return
        self._memo = None
        n_arg = n_batches  # the memo compares the caller's own argument (None or a count)
        B = self.batch_size
        u, i, j = (_idx(x, n, self.device) for x, n in ((user, "user"), (item_pos, "item_pos"),
                                                       (item_neg, "item_neg")))
        total = min(u.numel(), i.numel(), j.numel()) // B
        n_batches = total - first_batch if n_batches is None else int(n_batches)
        if first_batch < 0 or n_batches <= 0 or first_batch + n_batches > total:
            raise ValueError(f"batches [{first_batch}, {first_batch + n_batches}) outside the "
                             f"{total} batches of the stream")
        main = torch.cuda.current_stream(self.device)
        chunks = [(b, min(self.chunk, first_batch + n_batches - b))
                  for b in range(first_batch, first_batch + n_batches, self.chunk)]
        self._ov = (self.overlap if self.overlap is not None else B >= 4096) and len(chunks) > 1
        if not self._ov:  # plan + train per chunk in one C call each, on the caller's stream
            for k, (b, n) in enumerate(chunks):
                self.ctx[k % 2].train_range(tables, hp, u, i, j, B, b, n, graph=graph, check=check, _checked=True)
            self._staged = (u, i, j)
            if len(chunks) == 1 and not check and u is user and i is item_pos and j is item_neg:
                self._remember(tables, hp, user, item_pos, item_neg, first_batch, n_arg, n_batches, graph)
            return
        ready = torch.cuda.Event()
        ready.record(main)  # triplets produced on the caller's stream
        self.side.wait_event(ready)
        planned = self._plan(0, u, i, j, *chunks[0], check)
        for k, (b, n) in enumerate(chunks):
            if planned is not None:
                main.wait_event(planned)
            self.ctx[k % 2].train_planned(tables, hp, 0, n, graph=graph)
            done = torch.cuda.Event()
            done.record(main)
            self._free[k % 2] = done
            if k + 1 < len(chunks):
                planned = self._plan(k + 1, u, i, j, *chunks[k + 1], check)
        self._staged = (u, i, j)


def settle_tables() -> None:
    """Settle every queued (lazily verified) streamed call of the process
    (acf_apr_resolve_all): a failed one is replayed before anything reads the
    tables.  The readers outside a context's group call it first: the forward,
    evaluation, dns selection, Session fetches of the tables and checkpoints."""
    call("acf_apr_resolve_all")


def bpr_forward(P, Q, user, item_pos, item_neg, batch_size: int, clip_lo=CLIP_LO, clip_hi=CLIP_HI,
                want_scores: bool = False):
    """training_loss_acc's forward (utils.py:159-175): per-batch loss sum and #correct."""
    settle_tables()
    dev = P.device
    _require(P, "embedding_P", torch.float32, None, 2)
    _require(Q, "embedding_Q", torch.float32, dev, 2)
    if P.shape[1] != Q.shape[1]:
        raise ValueError("embedding_P and embedding_Q dims differ")
    u, i, j = (_idx(x, n, dev) for x, n in ((user, "user"), (item_pos, "item_pos"), (item_neg, "item_neg")))
    n = u.numel()
    if batch_size <= 0 or n % batch_size or i.numel() != n or j.numel() != n:
        raise ValueError("triplets must be equal-length multiples of batch_size")
    nb = n // batch_size
    _check_range(u, P.shape[0], "user")
    _check_range(i, Q.shape[0], "item")
    _check_range(j, Q.shape[0], "item")
    bl = torch.empty(nb, dtype=torch.float32, device=dev)
    bc = torch.empty(nb, dtype=torch.int32, device=dev)
    op = torch.empty(n, dtype=torch.float32, device=dev) if want_scores else None
    on = torch.empty(n, dtype=torch.float32, device=dev) if want_scores else None
    with torch.cuda.device(dev):
        call("acf_bpr_forward", P.data_ptr(), Q.data_ptr(), P.shape[0], Q.shape[0], P.shape[1],
             u.data_ptr(), i.data_ptr(), j.data_ptr(), batch_size, nb, clip_lo, clip_hi,
             bl.data_ptr(), bc.data_ptr(), op.data_ptr() if op is not None else None,
             on.data_ptr() if on is not None else None, _stream_ptr(dev))
    return bl, bc, op, on


_RANGE_OK: dict = {}  # (address, length, version, bound, device) -> weakref of the checked tensor


def _check_range(idx: torch.Tensor, rows: int, name: str) -> None:
    """IndexError unless every index lies in [0, rows).  The check reads the
    extremes back to the host (a device sync), so a tensor that passed is
    remembered by (address, length, in-place version, bound): an evaluation plan
    re-uses the same user / test tensors every epoch and pays the check once.
    The cache holds weak references only: an entry never extends a
    tensor's lifetime and leaves the cache when the tensor is freed."""
    key = (idx.data_ptr(), idx.numel(), idx._version, rows, idx.device)
    ref = _RANGE_OK.get(key)
    if ref is not None and ref() is idx:
        return
    if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= rows):
        raise _native.NativeIndexError(_native.ACF_E_RANGE, "range check",
                                       f"{name} index outside [0, {rows})")

    def _evict(r, k=key):
        if _RANGE_OK.get(k) is r:
            del _RANGE_OK[k]
    _RANGE_OK[key] = weakref.ref(idx, _evict)


EVAL_KERNELS = {"auto": 0, "mfma": 1, "valu": 2}


def _unique_exclusions(off: torch.Tensor, ex: torch.Tensor, n_users: int) -> torch.Tensor:
    """Each user's exclusion list as a SET (the reference's set(trainList[u]),
    utils.py:188-195): a repeated entry of a list is replaced by -1, which every
    sweep ignores (never a candidate).  The MFMA sweep applies a list as a bitmap
    (set semantics) and the VALU sweep subtracts once per entry, so without this a
    duplicate made them disagree.  Sort + compare on the device, no
    host sync; the lengths stay as given."""
    if ex.numel() < 2:
        return ex
    # each list's segment id by a search over the offsets (no assumption that
    # off[0] == 0 or off[-1] == len(ex); entries outside every list get -1 and
    # are left alone)
    pos = torch.arange(ex.numel(), device=ex.device, dtype=off.dtype)
    seg = torch.searchsorted(off[1:].contiguous(), pos, right=True)
    seg = torch.where((pos >= off[0]) & (seg < n_users), seg, torch.full_like(seg, -1))
    wide = int(2 ** 31)
    key = seg * wide + ex.long().clamp(-1, wide - 2) + 1
    skey, perm = torch.sort(key)
    dup = torch.zeros(ex.numel(), dtype=torch.bool, device=ex.device)
    dup[perm[1:]] = skey[1:] == skey[:-1]
    return torch.where(dup, torch.full_like(ex, -1), ex)


def eval_positions_all(P, Q, users, test_items, num_candidates: int, excl_off, excl_items, kernel: str = "auto",
                       unique_lists: bool = False):
    """_eval_by_user positions over all items minus the exclusion lists.  kernel:
    'auto' | 'mfma' | 'valu' (acf_eval_positions_all_kernel; same positions).
    A list may repeat an item: it is excluded once (set semantics); callers whose
    lists are already duplicate-free (EvalPlan: np.union1d) pass unique_lists=True
    to skip the device-side dedup."""
    settle_tables()
    dev = P.device
    _require(P, "embedding_P", torch.float32, None, 2)
    _require(Q, "embedding_Q", torch.float32, dev, 2)
    u, t = _idx(users, "users", dev), _idx(test_items, "test_items", dev)
    off = torch.as_tensor(excl_off).to(device=dev, dtype=torch.int64).contiguous()
    ex = _idx(excl_items, "excl_items", dev) if len(excl_items) else torch.zeros(1, dtype=torch.int32, device=dev)
    if off.numel() != u.numel() + 1:
        raise ValueError("excl_off must have len(users) + 1 entries")
    if kernel not in EVAL_KERNELS:
        raise ValueError(f"kernel must be one of {sorted(EVAL_KERNELS)}, got {kernel!r}")
    _check_range(u, P.shape[0], "user")
    _check_range(t, Q.shape[0], "test item")
    if num_candidates > Q.shape[0]:
        raise ValueError("num_candidates exceeds item rows")
    if not unique_lists and len(excl_items):
        ex = _unique_exclusions(off, ex, u.numel())
    pos = torch.empty(u.numel(), dtype=torch.int32, device=dev)
    with _on(dev):
        call("acf_eval_positions_all_kernel", P.data_ptr(), Q.data_ptr(), P.shape[0], Q.shape[0], P.shape[1],
             u.data_ptr(), t.data_ptr(), u.numel(), int(num_candidates), off.data_ptr(), ex.data_ptr(),
             pos.data_ptr(), EVAL_KERNELS[kernel], _stream_ptr(dev))
    return pos


def eval_positions_list(P, Q, users, test_items, cand_off, cand_items):
    """_eval_by_user positions over explicit candidate lists ("sample" mode)."""
    settle_tables()
    dev = P.device
    _require(P, "embedding_P", torch.float32, None, 2)
    _require(Q, "embedding_Q", torch.float32, dev, 2)
    u, t = _idx(users, "users", dev), _idx(test_items, "test_items", dev)
    off = torch.as_tensor(cand_off).to(device=dev, dtype=torch.int64).contiguous()
    c = _idx(cand_items, "cand_items", dev) if len(cand_items) else torch.zeros(1, dtype=torch.int32, device=dev)
    _check_range(u, P.shape[0], "user")
    _check_range(t, Q.shape[0], "item")
    _check_range(c, Q.shape[0], "item")
    pos = torch.empty(u.numel(), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        call("acf_eval_positions_list", P.data_ptr(), Q.data_ptr(), P.shape[0], Q.shape[0], P.shape[1],
             u.data_ptr(), t.data_ptr(), u.numel(), off.data_ptr(), c.data_ptr(), pos.data_ptr(),
             _stream_ptr(dev))
    return pos


def alias_table(weights):
    """(prob, alias) float32 / int32 numpy arrays of Vose's alias table for
    sampling k with probability weights[k] / sum(weights) (acf_alias_build)."""
    import numpy as np
    w = np.ascontiguousarray(np.asarray(weights, dtype=np.float32).reshape(-1))
    prob = np.empty(w.size, np.float32)
    alias = np.empty(w.size, np.int32)
    call("acf_alias_build", w.ctypes.data, w.size, prob.ctypes.data, alias.ctypes.data)
    return prob, alias


def sample_epoch(pos_user, pos_item, batch_size: int, num_items: int, list_off, list_items,
                 seed: int, max_tries: int = 1 << 20, check: bool = True, alias=None):
    """Device-side shuffle + negative sampling for one epoch (APR.py:39-81).
    alias: None (uniform proposals, APR.py:76) or a (prob, alias) pair of device
    tensors from alias_table (acf_sample_epoch_alias)."""
    dev = pos_user.device
    pu = _idx(pos_user, "pos_user", dev)
    pi = _idx(pos_item, "pos_item", dev)
    off = torch.as_tensor(list_off).to(device=dev, dtype=torch.int64).contiguous()
    li = _idx(list_items, "list_items", dev) if len(list_items) else torch.zeros(1, dtype=torch.int32, device=dev)
    n_out = (pu.numel() // batch_size) * batch_size
    ou = torch.empty(n_out, dtype=torch.int32, device=dev)
    op = torch.empty(n_out, dtype=torch.int32, device=dev)
    on = torch.empty(n_out, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        if alias is None:
            call("acf_sample_epoch", pu.data_ptr(), pi.data_ptr(), pu.numel(), batch_size, int(num_items),
                 off.numel() - 1, off.data_ptr(), li.data_ptr(), int(seed) & 0xFFFFFFFFFFFFFFFF,
                 int(max_tries), int(check), ou.data_ptr(), op.data_ptr(), on.data_ptr(), _stream_ptr(dev))
        else:
            prob, al = alias
            _require(prob, "alias prob", torch.float32, dev, 1)
            _require(al, "alias", torch.int32, dev, 1)
            if prob.numel() != num_items or al.numel() != num_items:
                raise ValueError(f"alias table has {prob.numel()} columns, expected num_items = {num_items}")
            call("acf_sample_epoch_alias", pu.data_ptr(), pi.data_ptr(), pu.numel(), batch_size, int(num_items),
                 off.numel() - 1, off.data_ptr(), li.data_ptr(), prob.data_ptr(), al.data_ptr(),
                 int(seed) & 0xFFFFFFFFFFFFFFFF, int(max_tries), int(check), ou.data_ptr(), op.data_ptr(),
                 on.data_ptr(), _stream_ptr(dev))
    return ou, op, on


def dns_select(P, Q, user, cand, dns: int):
    """utils.py:121-133: argmax-score negative among dns candidates per triplet."""
    settle_tables()
    dev = P.device
    _require(P, "embedding_P", torch.float32, None, 2)
    _require(Q, "embedding_Q", torch.float32, dev, 2)
    u = _idx(user, "user", dev)
    c = _idx(cand, "cand", dev)
    if c.numel() != u.numel() * dns:
        raise ValueError("cand must hold dns candidates per triplet")
    _check_range(u, P.shape[0], "user")
    _check_range(c, Q.shape[0], "item")
    out = torch.empty(u.numel(), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        call("acf_dns_select", P.data_ptr(), Q.data_ptr(), P.shape[0], Q.shape[0], P.shape[1],
             u.data_ptr(), c.data_ptr(), u.numel(), int(dns), out.data_ptr(), _stream_ptr(dev))
    return out


def shard_reduce_delta(recv, seg, pos, hp: StepHParams, G0, reply) -> None:
    """Owner side of the APR delta (APR.py:183-191): per owned row s, the partial
    clean sums recv[pos[seg[s]:seg[s+1]]] in order -> G0[s]; eps * l2_normalize
    of it -> reply[pos[...]] (include/acf_apr.h acf_shard_reduce_delta)."""
    n = seg.numel() - 1
    if n <= 0:
        return
    dev = recv.device
    for t, nm, dt in ((recv, "recv", torch.float32), (G0, "G0", torch.float32), (reply, "reply", torch.float32),
                      (seg, "seg", torch.int32), (pos, "pos", torch.int32)):
        _require(t, nm, dt, dev)
    h = hp.to_c()
    with torch.cuda.device(dev):
        call("acf_shard_reduce_delta", recv.data_ptr(), seg.data_ptr(), pos.data_ptr(), n, recv.shape[1],
             ctypes.byref(h), G0.data_ptr(), reply.data_ptr(), _stream_ptr(dev))


def shard_reduce_apply(Q, accQ, recv, seg, pos, hp: StepHParams, G0, rows, count=None, reg_batch: int = 0) -> None:
    """Owner side of the item Adagrad (APR.py:193-195): per owned row s,
    G0[s] + reg_adv * sum of its partial adversarial rows (BPR: the sum of its
    partial clean rows), then sparse Adagrad on Q[rows[s]], accQ[rows[s]]."""
    n = seg.numel() - 1
    if n <= 0:
        return
    dev = recv.device
    for t, nm, dt in ((Q, "Q", torch.float32), (accQ, "accQ", torch.float32), (recv, "recv", torch.float32),
                      (seg, "seg", torch.int32), (pos, "pos", torch.int32), (rows, "rows", torch.int32)):
        _require(t, nm, dt, dev)
    h = hp.to_c()
    with torch.cuda.device(dev):
        call("acf_shard_reduce_apply", Q.data_ptr(), accQ.data_ptr(), recv.data_ptr(), seg.data_ptr(),
             pos.data_ptr(), n, Q.shape[1], ctypes.byref(h), 0 if G0 is None else G0.data_ptr(),
             rows.data_ptr(), 0 if count is None else count.data_ptr(), int(reg_batch), _stream_ptr(dev))
