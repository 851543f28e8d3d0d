"""BASELINE configs[4] at its exact shape on one GPU: 10M users x 5M items,
d = 128, ~200M Zipf interactions (data.synthetic_large), batches of 65,536
triplets with alias-table negatives from the device sampler, through the
default large-batch step (triplet-centric list kernels, hot-slot pieces).
The oracle runs on the touched rows only (one APR step never reads or writes
another row), remapped to compact tables."""
import numpy as np
import pytest
import torch

from apr_oracle import HParams

pytestmark = pytest.mark.gpu


def test_config5_batches_match_oracle(ops, acf, oracle, dev, fp32_parity):
    B, d, nb = 65536, 128, 2
    big = acf.synthetic_large(device=dev)
    U1, I1 = big.num_users + 1, big.num_items + 1
    ep = acf.DeviceSampler(big, B, dev, seed=7, weights=np.ones(big.num_items, np.float32)).epoch(0)
    u, i, j = (x[: nb * B].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
    del ep, big
    g = torch.Generator(device=dev).manual_seed(5)
    tabs = [torch.randn(U1, d, device=dev, generator=g) * 0.1, torch.randn(I1, d, device=dev, generator=g) * 0.1,
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    uu = torch.unique(u.long())
    ii = torch.unique(torch.cat([i, j]).long())
    before = [tabs[0][uu].cpu().numpy(), tabs[1][ii].cpu().numpy()]
    probe_u = torch.randint(0, U1, (4096,), device=dev, generator=g)
    probe_u = probe_u[~torch.isin(probe_u, uu)]
    probe = tabs[0][probe_u].clone()
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(u, i, j, B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    lc, la = ctx.losses()
    assert ctx.step_errors() == 0
    # the oracle on compact tables of the touched rows
    un, inn = uu.cpu().numpy(), ii.cpu().numpy()
    cu = np.searchsorted(un, u.cpu().numpy()).astype(np.int32)
    ci = np.searchsorted(inn, i.cpu().numpy()).astype(np.int32)
    cj = np.searchsorted(inn, j.cpu().numpy()).astype(np.int32)
    P, Q = before
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    lcw, law = [], []
    for t in range(nb):
        s = slice(t * B, (t + 1) * B)
        a, b_, _, _ = oracle.apr_batch(P, Q, aP, aQ, cu[s], ci[s], cj[s], HParams(adver=1))
        lcw.append(a)
        law.append(b_)
    got = [tabs[0][uu], tabs[1][ii], tabs[2][uu], tabs[3][ii]]
    for x, w, n in zip(got, (P, Q, aP, aQ), ("P", "Q", "accP", "accQ")):
        fp32_parity(x, w, n)
    n_terms = max(2 * np.bincount(cu).max(), np.bincount(np.concatenate([ci, cj])).max())
    rtol = max(1e-5, 2 * n_terms * 2.0 ** -24)  # Higham bound for the hot rows' sums
    np.testing.assert_allclose(lc.cpu().numpy(), np.concatenate(lcw), rtol=rtol, atol=1e-6)
    np.testing.assert_allclose(la.cpu().numpy(), np.concatenate(law), rtol=rtol, atol=1e-6)
    assert torch.equal(tabs[0][probe_u], probe)  # untouched rows unchanged
