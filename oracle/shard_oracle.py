"""CPU restatement of one rank's passes of the split APR step — TEST INFRASTRUCTURE ONLY.

Plugged into ``distributed.ShardedAPR(local=OracleShardLocal)`` by the gloo tests
(tests/test_distributed.py) so that the product routing and all_to_all
exchanges run on CPU with the arithmetic of the HIP shard passes
(include/acf_apr.h "shard mode").  The product package never imports it.

Arithmetic follows APR.py:121-195 with TF op semantics, as oracle/apr_oracle.py:
rounded products summed per row in occurrence order (a triplet's positive
branch, then its negative branch), clip gradient on lo <= x <= hi, TF's
SoftplusGrad, l2_normalize with epsilon 1e-12, Adagrad acc += g^2,
w -= lr * g * rsqrt(acc).  Items: this rank's partial sums, completed by the
owner (reduce_delta / reduce_apply) in requester order.
"""
from __future__ import annotations

import numpy as np

from apr_oracle import _l2_normalize, _sigmoid_grad

f32 = np.float32


def _bpr_coef(x, lo, hi):
    r = np.clip(x, f32(lo), f32(hi))
    mask = ((x >= lo) & (x <= hi)).astype(f32)
    return (_sigmoid_grad(r) * mask).astype(f32)


def _sums(u, wi, wj, p, qi, qj, g, nU, nW, d):
    """Per-row sums of the rounded contributions, occurrence order."""
    GP = np.zeros((nU, d), f32)
    GQ = np.zeros((nW, d), f32)
    for b in range(len(u)):
        GP[u[b]] = GP[u[b]] + (g[b] * qi[b]).astype(f32)
        GP[u[b]] = GP[u[b]] - (g[b] * qj[b]).astype(f32)
        GQ[wi[b]] = GQ[wi[b]] + (g[b] * p[b]).astype(f32)
        GQ[wj[b]] = GQ[wj[b]] - (g[b] * p[b]).astype(f32)
    return GP, GQ


def _adagrad(W, A, rows, G, lr):
    for r in rows:
        A[r] = (A[r] + G[r] * G[r]).astype(f32)
        W[r] = (W[r] - (f32(lr) * G[r]) * (f32(1) / np.sqrt(A[r]))).astype(f32)


class OracleShardLocal:
    """Same interface as distributed.HipLocal, on the CPU shard tensors."""

    def __init__(self, sh):
        self.sh = sh

    def plan(self, u_rows, wi, wj):
        self.u = u_rows.numpy().astype(np.int64)
        self.wi = wi.numpy().astype(np.int64)
        self.wj = wj.numpy().astype(np.int64)
        self.nW = int(max(self.wi.max(), self.wj.max())) + 1 if len(self.u) else 0

    def _rows(self, dP=None, dQ=None):
        P, Qc = self.sh.P.numpy(), self.sh.Qc.numpy()
        p, qi, qj = P[self.u], Qc[self.wi], Qc[self.wj]
        if dP is not None:
            p = (p + dP[self.u]).astype(f32)
            qi = (qi + dQ[self.wi]).astype(f32)
            qj = (qj + dQ[self.wj]).astype(f32)
        x = ((p * qi).astype(f32).sum(1, dtype=f32) - (p * qj).astype(f32).sum(1, dtype=f32)).astype(f32)
        return p, qi, qj, x

    def clean(self, hp, out, rows):
        """working-set entry w's partial clean sum -> out[rows[w]]"""
        sh, d = self.sh, self.sh.d
        p, qi, qj, x = self._rows()
        g = _bpr_coef(x, hp.clip_lo, hp.clip_hi)
        GP, GQ = _sums(self.u, self.wi, self.wj, p, qi, qj, g, sh.P.shape[0], rows.numel(), d)
        self.GPc, self.users, self.p0 = GP, np.unique(self.u), p
        if hp.adver:  # the delta follows the clean loss only (APR.py:180-191)
            self.dP = np.zeros_like(GP) if hp.zero_delta else (_l2_normalize(GP) * f32(hp.eps)).astype(f32)
        else:
            if hp.reg:
                self._reg(GP, p, hp)
            _adagrad(sh.P.numpy(), sh.accP.numpy(), self.users, GP, hp.lr)
        out.numpy()[rows.numpy()] = GQ

    def _reg(self, GP, p, hp):
        coef = f32(2.0 * hp.reg / (self.sh.B * self.sh.d)) * f32(2 if hp.adver else 1)
        for b in range(len(self.u)):
            GP[self.u[b]] = GP[self.u[b]] + (coef * p[b]).astype(f32)

    def set_item_delta(self, src, rows):
        """the owners' delta of working-set entry w <- src[rows[w]]"""
        self.dQ = src.numpy()[rows.numpy()].copy()

    def adv(self, hp, out, rows):
        sh, d = self.sh, self.sh.d
        p, qi, qj, x = self._rows(self.dP, self.dQ)
        g = _bpr_coef(x, hp.clip_lo, hp.clip_hi)
        GP, GQ = _sums(self.u, self.wi, self.wj, p, qi, qj, g, sh.P.shape[0], rows.numel(), d)
        G = (self.GPc + f32(hp.reg_adv) * GP).astype(f32)
        if hp.reg:
            self._reg(G, self.p0, hp)
        _adagrad(sh.P.numpy(), sh.accP.numpy(), self.users, G, hp.lr)
        out.numpy()[rows.numpy()] = GQ

    # -- owner side ------------------------------------------------------------------
    @staticmethod
    def _seg_sums(recv, seg, pos):
        R, seg, pos = recv.numpy(), seg.numpy(), pos.numpy()
        out = np.zeros((len(seg) - 1, R.shape[1]), f32)
        for s in range(len(seg) - 1):
            for q in range(seg[s], seg[s + 1]):
                out[s] = (out[s] + R[pos[q]]).astype(f32)
        return out, seg, pos

    def reduce_delta(self, hp, recv, seg, pos, G0, reply):
        S, seg, pos = self._seg_sums(recv, seg, pos)
        G0.numpy()[:] = S
        dl = np.zeros_like(S) if hp.zero_delta else (_l2_normalize(S) * f32(hp.eps)).astype(f32)
        rep = reply.numpy()
        for s in range(len(seg) - 1):
            for q in range(seg[s], seg[s + 1]):
                rep[pos[q]] = dl[s]

    def reduce_apply(self, hp, recv, seg, pos, G0, rows, count):
        S, seg, _ = self._seg_sums(recv, seg, pos)
        G = (G0.numpy() + f32(hp.reg_adv) * S).astype(f32) if hp.adver else S
        # the storage with the trash row that padded segments name (distributed.py)
        Q, A, rows = self.sh._Qst.numpy(), self.sh._aQst.numpy(), rows.numpy()
        if hp.reg:
            coef = f32(2.0 * hp.reg / (self.sh.B * self.sh.d)) * f32(2 if hp.adver else 1)
            cnt = count.numpy()
            for s in range(len(rows)):
                G[s] = (G[s] + (coef * f32(cnt[s])) * Q[rows[s]]).astype(f32)
        for s, r in enumerate(rows):
            A[r] = (A[r] + G[s] * G[s]).astype(f32)
            Q[r] = (Q[r] - (f32(hp.lr) * G[s]) * (f32(1) / np.sqrt(A[r]))).astype(f32)
