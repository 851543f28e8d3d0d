"""Multi-threaded CPU restatement of the reference's training step, for the CPU
baseline only (TEST / BASELINE INFRASTRUCTURE: bench.py's cpu_baseline leg and
tests/test_oracle.py import it; the product path never does).

The reference (APR.py:101-195 on TF1, CPU) cannot run here (TensorFlow is
absent), so its work is mirrored op for op in torch-CPU fp32 with every host
thread, the way TF's CPU kernels use its intra-op pool:

  per batch (utils.py:114-119)
    clean gathers + BPR loss + grads            APR.py:121-150
    dense mode: grads densified to [rows, d], EVERY row l2-normalised and the
      full delta tables assigned                APR.py:183-191 (the reference's work)
    sparse mode: the same on the touched rows only (mathematically identical)
    adversarial gathers on P + delta, loss, grads  APR.py:130-165
    IndexedSlices concat (clean pos, clean neg, adv pos, adv neg), dedup by
      summation, SparseApplyAdagrad              APR.py:193-195
  BPR phase (adver = 0): the clean terms and Adagrad only.

Numerics agree with oracle/apr_oracle.c to fp32 rounding (tests/test_oracle.py).
"""
from __future__ import annotations

import os

import torch


def _bpr(P, Q, u, i, j, lo=-80.0, hi=1e8):
    p, qi, qj = P[u], Q[i], Q[j]
    x = (p * qi).sum(1) - (p * qj).sum(1)
    xc = x.clamp(lo, hi)
    g = torch.where((x >= lo) & (x <= hi), -torch.sigmoid(-xc), torch.zeros_like(x))
    loss = torch.nn.functional.softplus(-xc)
    return p, qi, qj, g, loss


def apr_step(P, Q, accP, accQ, u, i, j, lr=0.05, eps=0.5, reg_adv=1.0, adver=True, dense=True):
    """One training_batch iteration in place (reg = 0, the run_adv_ori default)."""
    p, qi, qj, g, _ = _bpr(P, Q, u, i, j)
    gu = torch.cat([g[:, None] * qi, -g[:, None] * qj])          # P slices: pos, neg
    gq = torch.cat([g[:, None] * p, -g[:, None] * p])             # Q slices: pos, neg
    iu, iq = torch.cat([u, u]), torch.cat([i, j])
    if adver:
        if dense:  # the reference's densify / normalise-every-row / assign
            dP = torch.zeros_like(P).index_add_(0, iu, gu)
            dQ = torch.zeros_like(Q).index_add_(0, iq, gq)
            dP = eps * dP * torch.rsqrt(dP.square().sum(1, keepdim=True).clamp_min(1e-12))
            dQ = eps * dQ * torch.rsqrt(dQ.square().sum(1, keepdim=True).clamp_min(1e-12))
            pa, qia, qja = P[u] + dP[u], Q[i] + dQ[i], Q[j] + dQ[j]
        else:  # touched rows only
            ru, inv_u = torch.unique(iu, return_inverse=True)
            rq, inv_q = torch.unique(iq, return_inverse=True)
            su = torch.zeros(len(ru), P.shape[1]).index_add_(0, inv_u, gu)
            sq = torch.zeros(len(rq), Q.shape[1]).index_add_(0, inv_q, gq)
            su = eps * su * torch.rsqrt(su.square().sum(1, keepdim=True).clamp_min(1e-12))
            sq = eps * sq * torch.rsqrt(sq.square().sum(1, keepdim=True).clamp_min(1e-12))
            n = len(u)
            pa, qia, qja = p + su[inv_u[:n]], qi + sq[inv_q[:n]], qj + sq[inv_q[n:]]
        xa = (pa * qia).sum(1) - (pa * qja).sum(1)
        ga = -torch.sigmoid(-xa.clamp(-80.0, 1e8)) * ((xa >= -80.0) & (xa <= 1e8))
        gu = torch.cat([gu, reg_adv * ga[:, None] * qia, -reg_adv * ga[:, None] * qja])
        gq = torch.cat([gq, reg_adv * ga[:, None] * pa, -reg_adv * ga[:, None] * pa])
        iu, iq = torch.cat([iu, u, u]), torch.cat([iq, i, j])
    for W, A, idx, val in ((P, accP, iu, gu), (Q, accQ, iq, gq)):
        rows, inv = torch.unique(idx, return_inverse=True)
        G = torch.zeros(len(rows), W.shape[1]).index_add_(0, inv, val)
        a = A[rows] + G * G
        A[rows] = a
        W[rows] = W[rows] - lr * G * torch.rsqrt(a)


def threads() -> int:
    """The host threads this job may use (OMP_NUM_THREADS on the GPU box, else all)."""
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"
