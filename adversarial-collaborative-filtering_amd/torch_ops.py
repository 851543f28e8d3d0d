"""``torch.ops.acf.*``: the APR hot path as PyTorch custom ops.

``lib/libacf_torch.so`` (csrc/acf_torch.cpp) registers ``TORCH_LIBRARY(acf, m)``
over the C-ABI of ``libacf_apr.so`` (include/acf_apr.h), with the operator set
SURVEY.md §8(b) proposes:

- ``bpr_apr_step(P, Q, accP, accQ, u, i, j, lr, eps, reg, reg_adv, adver, clip_lo, clip_hi)
  -> (loss_clean, loss_adv, n_correct)``: one training_batch iteration
  (utils.py:114-119, APR.py:143-195), tables updated in place;
- ``apr_train(..., batch_size, ...) -> (loss_clean[n], loss_adv[n])``: n/batch_size
  consecutive batches (the streamed step);
- decomposed, one TF op each: ``gather_bpr_fwd_bwd`` (APR.py:121-150,183),
  ``row_segment_sum`` (IndexedSlices dedup, APR.py:183-187,195), ``l2norm_perturb``
  (APR.py:186-191), ``sparse_adagrad_apply`` (APR.py:193-195);
- evaluation: ``score_rank`` / ``score_rank_all`` (_eval_by_user, utils.py:211-254);
- ``release_contexts() -> int``: frees the cached step contexts (plan workspace and
  the streamed step's version buffers) that ``apr_train`` / ``bpr_apr_step`` keep per
  (device, table shape, batch shape).

There is no CPU kernel: calling an op on CPU tensors raises (no fallback).
"""
from __future__ import annotations

import os
import threading

import torch

from . import build_native

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libacf_torch.so")
OPS = ("bpr_apr_step", "apr_train", "gather_bpr_fwd_bwd", "row_segment_sum", "l2norm_perturb",
       "sparse_adagrad_apply", "score_rank", "score_rank_all",
       "release_contexts")
_lock = threading.Lock()
_loaded = False


def load():
    """Load the op library (once) and return the ``torch.ops.acf`` namespace."""
    global _loaded
    with _lock:
        if not _loaded:
            if not os.path.exists(LIB):
                raise ImportError(f"{LIB} not found: build it with __graft_entry__.build() "
                                  "(build_native.build_torch_ops); there is no CPU fallback")
            build_native.verify("torch", LIB)  # built from these sources (ImportError otherwise)
            torch.ops.load_library(LIB)
            _loaded = True
    return torch.ops.acf
