"""Golden vectors of the CPU oracle on tiny shapes.

These pin the oracle against regressions (they are the oracle's own outputs,
cross-checked at generation time against the dense numpy TF-graph restatement
and torch autograd — see tests/test_oracle.py).  Shapes: U+1 = 64, I+1 = 48,
d in {8, 64}, B = 32, 3 batches, BPR and APR graphs, reg 0 and 0.01, with
forced i == j triplets (possible through the reference's trainList quirk).

Usage:  python tests/golden/make_oracle_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
from apr_oracle import COracle, HParams, tf_graph_step  # noqa: E402

CASES = [(d, adver, reg) for d in (8, 64) for adver in (0, 1) for reg in (0.0, 0.01)]


def make_case(o, d, adver, reg, seed):
    rng = np.random.default_rng(seed)
    U1, I1, B, nb = 64, 48, 32, 3
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    j[::11] = i[::11]
    hp = HParams(adver=adver, reg=reg)
    out = {"P0": P.copy(), "Q0": Q.copy(), "u": u, "i": i, "j": j}
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    tP, tQ, taP, taQ = P.copy(), Q.copy(), aP.copy(), aQ.copy()
    losses, deltas = [], []
    for t in range(nb):
        s = slice(t * B, (t + 1) * B)
        lc, la, dP, dQ = o.apr_batch(P, Q, aP, aQ, u[s], i[s], j[s], hp, want_delta=True)
        tf_graph_step(tP, tQ, taP, taQ, u[s], i[s], j[s], hp)
        losses.append(lc)
        if adver:
            out[f"dP{t}"], out[f"dQ{t}"] = dP, dQ
    # generation-time cross-check against the dense TF-graph restatement
    for a, b in ((P, tP), (Q, tQ), (aP, taP), (aQ, taQ)):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)
    out.update(P=P, Q=Q, accP=aP, accQ=aQ, loss_clean=np.concatenate(losses))
    return out


def main():
    o = COracle()
    arrays = {}
    for n, (d, adver, reg) in enumerate(CASES):
        for k, v in make_case(o, d, adver, reg, 100 + n).items():
            arrays[f"d{d}_a{adver}_r{reg}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "oracle_tiny.npz"), **arrays)
    print("wrote", os.path.join(HERE, "oracle_tiny.npz"))


if __name__ == "__main__":
    main()
