"""``MF`` — drop-in for the reference's APR/BPR-MF graph (``APR.py:85-202``).

The reference builds a TF1 graph and drives it with ``sess.run``.  This class keeps
that surface: the same constructor and attributes, ``build_graph()``, placeholder
handles (``user_input``, ``item_input_pos``, ``item_input_neg``) and fetch handles
(``update_P``, ``update_Q``, ``optimizer``, ``loss``, ``output``, ``output_neg``,
``embedding_P``, ``embedding_Q`` …), and :class:`Session` runs those fetches.
Under it, the tables are fp32 tensors on a HIP device and every fetch is a call
into ``libacf_apr.so``:

  ``sess.run([update_P, update_Q], fd)``  -> ``acf_apr_delta_update``
  ``sess.run(optimizer, fd)``             -> ``acf_apr_optimizer_step``
  ``sess.run([loss, output, output_neg])``-> ``acf_bpr_forward``
  ``sess.run(output, {user, item_pos})``  -> scores P[u]·Q[i]

For whole epochs ``train.training_batch`` bypasses the per-call plan and runs the
entire epoch from one plan through a cached hipGraph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


class _Handle:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"<acf handle {self.name}>"


def default_device():
    import os
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the APR path runs only on MI355X (gfx950); "
                           "there is no CPU fallback")
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))


class MF:
    """MF(num_users, num_items, args) — APR.py:86-97.  Tables have num_users + 1 /
    num_items + 1 rows like APR.py:108,111 (twin=True: evaluation_adv.py:120,123
    sizes them num_users / num_items)."""

    def __init__(self, num_users, num_items, args, twin: bool = False):
        self.num_items = num_items
        self.num_users = num_users
        self.embedding_size = args.embed_size
        self.learning_rate = args.lr
        self.reg = args.reg
        self.dns = args.dns
        self.adv = args.adv
        self.eps = args.eps
        self.adver = args.adver
        self.reg_adv = args.reg_adv
        self.epochs = args.epochs
        self.twin = twin
        self.seed = getattr(args, "seed", None)
        self.built = False

    # -- graph ----------------------------------------------------------------
    def _create_placeholders(self):
        self.user_input = _Handle("user_input")
        self.item_input_pos = _Handle("item_input_pos")
        self.item_input_neg = _Handle("item_input_neg")

    def _create_variables(self, device=None, generator=None):
        self.device = torch.device(device) if device is not None else default_device()
        extra = 0 if self.twin else 1
        self.num_user_rows = self.num_users + extra
        self.num_item_rows = self.num_items + extra
        d = self.embedding_size
        g = generator
        if g is None and self.seed is not None:
            g = torch.Generator().manual_seed(int(self.seed))
        # tf.truncated_normal(stddev=0.01): normal redrawn beyond 2 sigma (APR.py:107-112)
        P = torch.empty(self.num_user_rows, d, dtype=torch.float32)
        Q = torch.empty(self.num_item_rows, d, dtype=torch.float32)
        torch.nn.init.trunc_normal_(P, 0.0, 0.01, -0.02, 0.02, generator=g)
        torch.nn.init.trunc_normal_(Q, 0.0, 0.01, -0.02, 0.02, generator=g)
        self.embedding_P = P.to(self.device)
        self.embedding_Q = Q.to(self.device)
        # AdagradOptimizer slots, initial_accumulator_value = 0.1 (APR.py:195)
        self.accumulator_P = torch.full_like(self.embedding_P, 0.1)
        self.accumulator_Q = torch.full_like(self.embedding_Q, 0.1)
        self.h = None  # the ones-vector of APR.py:119 is the row reduction in the kernels

    def _create_fetches(self):
        for name in ("update_P", "update_Q", "optimizer", "loss", "loss_adv", "output", "output_neg",
                     "output_adv", "output_neg_adv", "opt_loss", "result"):
            setattr(self, name, _Handle(name))

    def build_graph(self, device=None, generator=None):
        """APR.py:197-202."""
        self._create_placeholders()
        self._create_variables(device, generator)
        self._create_fetches()
        self._ctx = None
        self._pipe = None
        self._delta_feed = None
        self.built = True
        return self

    # -- state ----------------------------------------------------------------
    @property
    def tables(self):
        """The four tables for a READER: every queued streamed call is settled
        first (its lazy verification, ops.settle_tables)."""
        ops.settle_tables()
        return self.launch_tables

    @property
    def launch_tables(self):
        """The four tables for a training LAUNCH, without settling: a launch on
        them is ordered after the queued calls on the stream, and the native
        failure-safe gate covers the rest (settling here blocked the
        host on every queued call at each epoch)."""
        return (self.embedding_P, self.embedding_Q, self.accumulator_P, self.accumulator_Q)

    def hparams(self, adver=None) -> ops.StepHParams:
        return ops.StepHParams(lr=self.learning_rate, eps=self.eps, reg=self.reg,
                               reg_adv=self.reg_adv, adver=int(self.adver if adver is None else adver),
                               adv=self.adv, seed=int(self.seed or 0))

    def context(self, batch_size: int, n_batches: int) -> ops.APRContext:
        ctx = self._ctx
        if ctx is None or not ctx.fits(batch_size, n_batches):
            cap_b = max(batch_size, ctx.max_batch_size if ctx else 0)
            cap_n = max(n_batches, ctx.max_batches if ctx else 0)
            self._ctx = ctx = ops.APRContext(self.num_user_rows, self.num_item_rows,
                                             self.embedding_size, cap_b, cap_n, self.device)
        return ctx

    def pipeline(self, batch_size: int, chunk: int = 512) -> ops.PlanPipeline:
        """Epoch trainer: chunks of `chunk` batches, next chunk planned while one trains."""
        p = self._pipe
        if p is None or p.batch_size != batch_size or p.chunk != chunk:
            # concurrent planning for large batches only (device-wide sort plan); small
            # batches plan in line (batch-local plan, two launches per chunk)
            self._pipe = p = ops.PlanPipeline(self.num_user_rows, self.num_item_rows,
                                              self.embedding_size, batch_size, chunk, self.device,
                                              overlap=None)
        return p

    def reset_optimizer(self):
        """A fresh MF in the reference means fresh Adagrad slots (run_adv_ori.py:108)."""
        self.accumulator_P.fill_(0.1)
        self.accumulator_Q.fill_(0.1)

    def load_embeddings(self, P, Q):
        self.embedding_P.copy_(torch.as_tensor(np.asarray(P), dtype=torch.float32))
        self.embedding_Q.copy_(torch.as_tensor(np.asarray(Q), dtype=torch.float32))

    # -- single-batch entry points (one sess.run each) -------------------------
    def _plan_feed(self, u, i, j):
        u = ops._idx(u, "user_input", self.device)
        B = u.numel()
        ctx = self.context(B, 1)
        ctx.plan(u, i, j, B)
        return ctx

    def delta_update(self, u, i, j):
        """sess.run([update_P, update_Q], feed) — utils.py:117-118."""
        ctx = self._plan_feed(u, i, j)
        ctx.delta_update(self.launch_tables, self.hparams(adver=1), 0)
        self._delta_feed = (u, i, j)

    def optimizer_step(self, u, i, j):
        """sess.run(optimizer, feed) — utils.py:119."""
        ctx = self._ctx
        same = (self._delta_feed is not None and ctx is not None and ctx.n_batches == 1
                and all(a is b for a, b in zip(self._delta_feed, (u, i, j))))
        if self.adver and not same:
            self.delta_update(u, i, j)
            ctx = self._ctx
        elif not self.adver:
            ctx = self._plan_feed(u, i, j)
        ctx.optimizer_step(self.launch_tables, self.hparams(), 0)
        self._delta_feed = None

    def scores(self, users, items):
        """model.output for arbitrary (user, item) pairs: P[u]·Q[i] ([n,1])."""
        u = ops._idx(users, "user_input", self.device)
        i = ops._idx(items, "item_input_pos", self.device)
        n = u.numel()
        if n == 0:
            return np.zeros((0, 1), np.float32)
        _, _, op, _ = ops.bpr_forward(self.embedding_P, self.embedding_Q, u, i, i, n, want_scores=True)
        return op.cpu().numpy().reshape(-1, 1)


class Session:
    """Minimal ``tf.Session`` stand-in for the fetches the APR path uses."""

    def __init__(self, model: MF):
        self.model = model

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def run(self, fetches, feed_dict=None):
        m = self.model
        single = not isinstance(fetches, (list, tuple))
        fl = [fetches] if single else list(fetches)
        # variables are fetched by value, like TF returns their numpy arrays (utils.py:92)
        names = [f.name if isinstance(f, _Handle) else
                 ("embedding_P" if f is m.embedding_P else "embedding_Q" if f is m.embedding_Q else f)
                 if isinstance(f, torch.Tensor) else f for f in fl]
        fd = {k.name if isinstance(k, _Handle) else k: v for k, v in (feed_dict or {}).items()}
        u, i, j = fd.get("user_input"), fd.get("item_input_pos"), fd.get("item_input_neg")
        out = {}
        if any(isinstance(n, str) and n in ("update_P", "update_Q") for n in names):
            # build_graph always creates the adversarial ops (APR.py:197-202), so a BPR
            # graph runs them too: delta is computed, and its optimizer never reads it
            m.delta_update(u, i, j)
            out["update_P"] = out["update_Q"] = None
        if "optimizer" in names:
            m.optimizer_step(u, i, j)
            out["optimizer"] = None
        if any(isinstance(n, str) and n in ("loss", "output_neg") for n in names) or (
                "output" in names and j is not None):
            uu = ops._idx(u, "user_input", m.device)
            n = uu.numel()
            bl, bc, op, on = ops.bpr_forward(m.embedding_P, m.embedding_Q, uu, i, j, n, want_scores=True)
            out["loss"] = float(bl.cpu()[0])
            out["output"] = op.cpu().numpy().reshape(-1, 1)
            out["output_neg"] = on.cpu().numpy().reshape(-1, 1)
        elif "output" in names:
            out["output"] = m.scores(u, i)
        if "embedding_P" in names or "embedding_Q" in names:
            ops.settle_tables()
        if "embedding_P" in names:
            out["embedding_P"] = m.embedding_P.cpu().numpy()
        if "embedding_Q" in names:
            out["embedding_Q"] = m.embedding_Q.cpu().numpy()
        for k, n in enumerate(names):
            if isinstance(n, torch.Tensor):  # any other tensor: its value
                names[k] = "_t%d" % k
                out[names[k]] = n.detach().cpu().numpy()
        missing = [n for n in names if n not in out]
        if missing:
            raise NotImplementedError(f"fetch(es) {missing} not supported by the APR session")
        res = [out[n] for n in names]
        return res[0] if single else res
