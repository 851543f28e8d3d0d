"""HIP path vs the CPU oracle (oracle/apr_oracle.c) on identical inputs.

Tolerance: fp32, rtol 1e-5 / atol 1e-6 on tables of magnitude O(0.1-1) — the
bar north_star sets ("within 1e-5 fp32").  Differences come only from the order
of the per-row dot-product sums (wavefront butterfly vs sequential).
"""
import importlib

import numpy as np
import pytest
import torch

from apr_oracle import HParams
from conftest import PKG

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-5, 1e-6


def _problem(seed, U1, I1, d, B, nb, scale=0.3, dup_items=False):
    rng = np.random.default_rng(seed)
    P = (rng.standard_normal((U1, d)) * scale).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * scale).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    if dup_items:  # the trainList quirk lets j == i happen; force some
        j[::7] = i[::7]
    return P, Q, u, i, j


def _gpu_tables(P, Q, dev):
    return [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
            torch.full(P.shape, 0.1, device=dev), torch.full(Q.shape, 0.1, device=dev)]


def _oracle_run(oracle, P, Q, u, i, j, B, hp, dense=False):
    rP, rQ = P.copy(), Q.copy()
    aP, aQ = np.full(P.shape, 0.1, np.float32), np.full(Q.shape, 0.1, np.float32)
    lcs, las, deltas = [], [], []
    for t in range(len(u) // B):
        s = slice(t * B, (t + 1) * B)
        lc, la, dP, dQ = oracle.apr_batch(rP, rQ, aP, aQ, u[s], i[s], j[s], hp, dense=dense, want_delta=True)
        lcs.append(lc)
        las.append(la)
        deltas.append((dP, dQ))
    return (rP, rQ, aP, aQ), np.concatenate(lcs), np.concatenate(las), deltas


def _close(got, want, name):
    got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else got
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=ATOL, err_msg=name)


@pytest.mark.parametrize("d", [8, 32, 64, 128, 256, 512])
@pytest.mark.parametrize("adver", [0, 1])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("mapping", ["wave", "group"])
def test_train_planned_matches_oracle(ops, oracle, dev, d, adver, graph, mapping):
    U1, I1, B, nb = 61, 47, 64, 4
    P, Q, u, i, j = _problem(d * 10 + adver, U1, I1, d, B, nb, dup_items=True)
    hp_c = HParams(adver=adver)
    want, lc_w, la_w, _ = _oracle_run(oracle, P, Q, u, i, j, B, hp_c)
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_slot_mapping(mapping)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=adver), graph=graph)
    lc, la = ctx.losses()
    torch.cuda.synchronize()
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        _close(g, w, n)
    _close(lc, lc_w, "loss_clean")
    if adver:
        _close(la, la_w, "loss_adv")


@pytest.mark.parametrize("reg", [0.0, 0.01])
@pytest.mark.parametrize("d", [16, 64])
def test_split_calls_and_delta_match_oracle(ops, oracle, dev, reg, d):
    """sess.run([update_P, update_Q]) then sess.run(optimizer), batch by batch."""
    U1, I1, B, nb = 33, 29, 48, 3
    P, Q, u, i, j = _problem(5 + d, U1, I1, d, B, nb)
    hp_c = HParams(adver=1, reg=reg)
    want, _, _, deltas = _oracle_run(oracle, P, Q, u, i, j, B, hp_c)
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    hp = ops.StepHParams(adver=1, reg=reg)
    for t in range(nb):
        ctx.delta_update(tabs, hp, t)
        dP, dQ = ctx.delta_tables()
        _close(dP, deltas[t][0], f"delta_P batch {t}")
        _close(dQ, deltas[t][1], f"delta_Q batch {t}")
        ctx.optimizer_step(tabs, hp, t)
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        _close(g, w, n)


def test_dense_oracle_equals_sparse_path(ops, oracle, dev):
    """The reference's dense full-table delta work vs touched-rows-only: same result."""
    U1, I1, d, B, nb = 90, 70, 64, 32, 3
    P, Q, u, i, j = _problem(11, U1, I1, d, B, nb)
    dense, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1), dense=True)
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    for g, w, n in zip(tabs, dense, ("P", "Q", "accP", "accQ")):
        _close(g, w, n)


def test_zero_delta_dns_branch(ops, oracle, dev):
    U1, I1, d, B = 20, 25, 32, 16
    P, Q, u, i, j = _problem(3, U1, I1, d, B, 2)
    want, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1, zero_delta=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, 2, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    hp = ops.StepHParams(adver=1, zero_delta=1)
    ctx.train_planned(tabs, hp, graph=False)
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        _close(g, w, n)


def test_random_delta_has_norm_eps(ops, dev):
    U1, I1, d, B = 30, 30, 64, 32
    P, Q, u, i, j = _problem(4, U1, I1, d, B, 1)
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, 1, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    hp = ops.StepHParams(adver=1, adv="random", eps=0.5, seed=9)
    ctx.delta_update(tabs, hp, 0)
    dP, dQ = ctx.delta_tables()
    touched_u = np.unique(u)
    norms = torch.linalg.vector_norm(dP[torch.tensor(touched_u, device=dev)], dim=1).cpu().numpy()
    np.testing.assert_allclose(norms, 0.5, rtol=1e-5)
    untouched = np.setdiff1d(np.arange(U1), touched_u)
    assert float(dP[torch.tensor(untouched, device=dev)].abs().max()) == 0.0 if len(untouched) else True


@pytest.mark.parametrize("stream", [False, True])
@pytest.mark.parametrize("d", [16, 64])
def test_random_delta_matches_oracle(ops, oracle, dev, stream, d):
    """adv = "random" (APR.py:170-177) against the oracle's restatement of the
    same counter-based draw: delta rows of the split calls, then whole calls
    (k_stream or two kernels per step; fused triplets on) over 4 batches.  A
    fresh context's first call reads call counter 1, its second call 2."""
    U1, I1, B, nb = 50, 40, 64, 4
    P, Q, u, i, j = _problem(8 + d, U1, I1, d, B, nb, dup_items=True)
    hp = ops.StepHParams(adver=1, adv="random", seed=77)
    # split calls, batch 0: delta tables
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    tabs = _gpu_tables(P, Q, dev)
    ctx.delta_update(tabs, hp, 0)
    dP, dQ = ctx.delta_tables()
    rP, rQ = P.copy(), Q.copy()
    aP, aQ = np.full(P.shape, 0.1, np.float32), np.full(Q.shape, 0.1, np.float32)
    _, _, wdP, wdQ = oracle.apr_batch(rP, rQ, aP, aQ, u[:B], i[:B], j[:B],
                                      HParams(adver=1, adv="random", seed=77, call=1, t=0), want_delta=True)
    _close(dP, wdP, "random delta_P")
    _close(dQ, wdQ, "random delta_Q")
    # whole calls: a fresh context, two calls over the same 4 batches (counter 1, then 2)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_stream(stream)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    tabs = _gpu_tables(P, Q, dev)
    rP, rQ = P.copy(), Q.copy()
    aP, aQ = np.full(P.shape, 0.1, np.float32), np.full(Q.shape, 0.1, np.float32)
    for call in (1, 2):
        ctx.train_planned(tabs, hp)
        oracle.apr_train(rP, rQ, aP, aQ, u, i, j, B, HParams(adver=1, adv="random", seed=77, call=call))
        for g, w, n in zip(tabs, (rP, rQ, aP, aQ), ("P", "Q", "accP", "accQ")):
            _close(g, w, f"call {call} {n}")
    assert ctx.step_errors() == 0


def test_random_delta_redrawn_every_call(ops, dev):
    """The same batch stepped twice draws different noise (truncated_normal is
    re-evaluated by every sess.run in the reference)."""
    U1, I1, d, B = 30, 30, 32, 32
    P, Q, u, i, j = _problem(4, U1, I1, d, B, 1)
    ctx = ops.APRContext(U1, I1, d, B, 1, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    hp = ops.StepHParams(adver=1, adv="random", seed=9)
    tabs = _gpu_tables(P, Q, dev)
    draws = []
    for _ in range(2):
        ctx.delta_update(tabs, hp, 0)
        draws.append(ctx.delta_tables()[0].clone())
        ctx.optimizer_step(tabs, hp, 0)
    rows = torch.tensor(np.unique(u), device=dev)
    assert not torch.equal(draws[0][rows], draws[1][rows])
    np.testing.assert_allclose(torch.linalg.vector_norm(draws[1][rows], dim=1).cpu().numpy(), 0.5, rtol=1e-5)


def test_forward_matches_oracle(ops, oracle, dev):
    U1, I1, d, B, nb = 100, 80, 64, 50, 6
    P, Q, u, i, j = _problem(21, U1, I1, d, B, nb)
    bl_w, bc_w, op_w, on_w = oracle.bpr_forward(P, Q, u, i, j, B)
    Pt, Qt = torch.tensor(P, device=dev), torch.tensor(Q, device=dev)
    bl, bc, op, on = ops.bpr_forward(Pt, Qt, torch.tensor(u, device=dev), torch.tensor(i, device=dev),
                                     torch.tensor(j, device=dev), B, want_scores=True)
    _close(op, op_w, "output")
    _close(on, on_w, "output_neg")
    np.testing.assert_allclose(bl.cpu().numpy(), bl_w, rtol=1e-5)
    # acc counts compare sign(x+ - x-); allow a flip only where |x| is at rounding level
    x = op_w - on_w
    unsure = (np.abs(x) < 1e-5).reshape(nb, B).sum(1)
    assert np.all(np.abs(bc.cpu().numpy() - bc_w) <= unsure)


def test_eval_positions_exact(ops, oracle, dev):
    """Integer-valued tables: every score is exact, so ties (>=) are decided the
    same way as the reference; positions must match bit for bit."""
    rng = np.random.default_rng(0)
    U1, I1, d = 50, 200, 16
    P = rng.integers(-3, 4, (U1, d)).astype(np.float32)
    Q = rng.integers(-3, 4, (I1, d)).astype(np.float32)
    users = np.arange(0, 45, dtype=np.int32)
    tests = rng.integers(0, I1, len(users)).astype(np.int32)
    lists = [np.unique(np.append(rng.integers(0, 180, rng.integers(0, 40)), t)).astype(np.int32)
             for t in tests]
    lists = [l_[l_ < 180] for l_ in lists]
    off = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(l_) for l_ in lists], out=off[1:])
    excl = np.concatenate(lists)
    want = oracle.eval_positions_all(P, Q, users, tests, 180, off, excl)
    got = ops.eval_positions_all(torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                                 torch.tensor(users, device=dev), torch.tensor(tests, device=dev), 180,
                                 off, excl)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    cand = rng.integers(0, I1, len(users) * 100).astype(np.int32)
    coff = np.arange(0, len(users) * 100 + 1, 100, dtype=np.int64)
    want = oracle.eval_positions_list(P, Q, users, tests, coff, cand)
    got = ops.eval_positions_list(torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                                  torch.tensor(users, device=dev), torch.tensor(tests, device=dev), coff, cand)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_eval_positions_random_tables(ops, oracle, dev):
    rng = np.random.default_rng(1)
    U1, I1, d = 300, 1000, 64
    P = rng.standard_normal((U1, d)).astype(np.float32)
    Q = rng.standard_normal((I1, d)).astype(np.float32)
    users = np.arange(U1, dtype=np.int32)
    tests = rng.integers(0, I1, U1).astype(np.int32)
    lists = [np.unique(np.append(rng.integers(0, I1 - 1, 30), t)).astype(np.int32) for t in tests]
    lists = [l_[l_ < I1 - 1] for l_ in lists]
    off = np.zeros(U1 + 1, np.int64)
    np.cumsum([len(l_) for l_ in lists], out=off[1:])
    excl = np.concatenate(lists)
    want = oracle.eval_positions_all(P, Q, users, tests, I1 - 1, off, excl)
    got = ops.eval_positions_all(torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                                 torch.tensor(users, device=dev), torch.tensor(tests, device=dev), I1 - 1,
                                 off, excl).cpu().numpy()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("d", [16, 64, 100, 256])
def test_eval_mfma_exact_near_ties(ops, oracle, dev, d):
    """The MFMA sweep (k_eval_mfma) gives the oracle's positions exactly, also where
    candidates score within the f32 error band of the test item (rescored with the
    sequential dot): near-copies of each user's test row, exact copies (real ties),
    and ragged tile edges (users and candidates not multiples of 64 / 128)."""
    rng = np.random.default_rng(d)
    U1, I1 = 150, 700
    P = rng.standard_normal((U1, d)).astype(np.float32)
    Q = rng.standard_normal((I1, d)).astype(np.float32)
    users = rng.permutation(U1)[:133].astype(np.int32)
    tests = rng.integers(0, 600, len(users)).astype(np.int32)
    for k, t in enumerate(tests[:60]):  # near-ties and exact ties of the test row
        row = 600 + k
        Q[row] = Q[t] * np.float32(1 + (k % 5 - 2) * 1e-7) if k % 3 else Q[t]
    num_cand = 677
    lists = [np.unique(np.append(rng.integers(0, num_cand, 20), t)).astype(np.int32) for t in tests]
    off = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(x) for x in lists], out=off[1:])
    excl = np.concatenate(lists)
    want = oracle.eval_positions_all(P, Q, users, tests, num_cand, off, excl)
    args = (torch.tensor(P, device=dev), torch.tensor(Q, device=dev), torch.tensor(users, device=dev),
            torch.tensor(tests, device=dev), num_cand, off, excl)
    got = ops.eval_positions_all(*args).cpu().numpy()
    np.testing.assert_array_equal(got, want)
    for kernel in ("mfma", "valu"):
        np.testing.assert_array_equal(ops.eval_positions_all(*args, kernel=kernel).cpu().numpy(), want)


def test_eval_exclusions_unsorted_and_out_of_range(ops, oracle, dev):
    """The MFMA sweep applies the exclusion lists as a set (utils.py:209-214):
    unsorted lists and entries outside [0, num_candidates) give the positions of
    the sorted, in-range lists; the VALU sweep agrees."""
    rng = np.random.default_rng(21)
    U1, I1, d, num_cand = 300, 900, 64, 777
    P = rng.standard_normal((U1, d)).astype(np.float32)
    Q = rng.standard_normal((I1, d)).astype(np.float32)
    users = rng.permutation(U1)[:211].astype(np.int32)
    tests = rng.integers(0, num_cand, len(users)).astype(np.int32)
    lists = [np.unique(np.append(rng.integers(0, I1, 40), t)).astype(np.int32) for t in tests]
    clean = [x[x < num_cand] for x in lists]
    off = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(x) for x in clean], out=off[1:])
    want = oracle.eval_positions_all(P, Q, users, tests, num_cand, off, np.concatenate(clean))
    shuffled = [rng.permutation(x) for x in lists]
    off2 = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(x) for x in shuffled], out=off2[1:])
    args = (torch.tensor(P, device=dev), torch.tensor(Q, device=dev), torch.tensor(users, device=dev),
            torch.tensor(tests, device=dev), num_cand, off2, np.concatenate(shuffled))
    for kernel in ("auto", "mfma", "valu"):
        np.testing.assert_array_equal(ops.eval_positions_all(*args, kernel=kernel).cpu().numpy(), want)
    with pytest.raises(ValueError):
        ops.eval_positions_all(*args, kernel="gemm")


def test_eval_exclusions_duplicated_entries(ops, oracle, dev):
    """A list that repeats an item (and the test item) excludes it once, as the
    reference's set(trainList[u]) does (utils.py:188-195): the MFMA and VALU
    sweeps give the positions of the duplicate-free lists."""
    rng = np.random.default_rng(22)
    U1, I1, d, num_cand = 200, 600, 64, 600
    P = rng.standard_normal((U1, d)).astype(np.float32)
    Q = rng.standard_normal((I1, d)).astype(np.float32)
    users = rng.permutation(U1)[:150].astype(np.int32)
    tests = rng.integers(0, num_cand, len(users)).astype(np.int32)
    lists = [np.unique(np.append(rng.integers(0, num_cand, 30), t)).astype(np.int32) for t in tests]
    off = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(x) for x in lists], out=off[1:])
    want = oracle.eval_positions_all(P, Q, users, tests, num_cand, off, np.concatenate(lists))
    dup = [rng.permutation(np.concatenate([x, x[: 1 + k % len(x)], [t, t]])).astype(np.int32)
           for k, (x, t) in enumerate(zip(lists, tests))]
    off2 = np.zeros(len(users) + 1, np.int64)
    np.cumsum([len(x) for x in dup], out=off2[1:])
    args = (torch.tensor(P, device=dev), torch.tensor(Q, device=dev), torch.tensor(users, device=dev),
            torch.tensor(tests, device=dev), num_cand, off2, np.concatenate(dup))
    for kernel in ("auto", "mfma", "valu"):
        np.testing.assert_array_equal(ops.eval_positions_all(*args, kernel=kernel).cpu().numpy(), want)


def test_sampler_properties(ops, acf, dev):
    ds = acf.synthetic_dataset(500, 300, 20000, seed=3)
    s = acf.DeviceSampler(ds, 128, dev, seed=1)
    ep = s.epoch(0)
    n_out = (len(ds.pair_user) // 128) * 128
    u, i, j = (t.cpu().numpy() for t in (ep.user, ep.item_pos, ep.item_neg))
    assert len(u) == n_out
    off, items = ds.sorted_lists()
    # every negative in range and not in the user's list; positives are real pairs
    assert j.min() >= 0 and j.max() < ds.num_items
    for k in range(0, n_out, 37):
        lst = items[off[u[k]]:off[u[k] + 1]]
        assert j[k] not in lst and i[k] in lst
    # a permutation of the positives (drop-last): no positive used twice
    key = u.astype(np.int64) * ds.num_items + i
    assert len(np.unique(key)) == n_out
    # deterministic per (seed, epoch), different across epochs
    ep2 = s.epoch(0)
    assert torch.equal(ep.item_neg, ep2.item_neg)
    assert not torch.equal(ep.user, s.epoch(1).user)
    # uniformity of negatives (chi-square-ish): counts per item within 6 sigma
    counts = np.bincount(j, minlength=ds.num_items)
    allowed = ds.num_items - np.diff(off).mean()
    exp = n_out / allowed
    assert counts.max() < exp + 6 * np.sqrt(exp) + 10


def test_dns_select(ops, dev):
    rng = np.random.default_rng(2)
    P = rng.standard_normal((10, 32)).astype(np.float32)
    Q = rng.standard_normal((40, 32)).astype(np.float32)
    u = rng.integers(0, 10, 64).astype(np.int32)
    cand = rng.integers(0, 40, 64 * 5).astype(np.int32)
    got = ops.dns_select(torch.tensor(P, device=dev), torch.tensor(Q, device=dev), torch.tensor(u, device=dev),
                         torch.tensor(cand, device=dev), 5).cpu().numpy()
    sc = np.einsum("nd,nkd->nk", P[u], Q[cand.reshape(64, 5)])
    want = cand.reshape(64, 5)[np.arange(64), sc.argmax(1)]
    np.testing.assert_array_equal(got, want)


def test_out_of_range_index_raises(ops, dev):
    from importlib import import_module
    native = import_module("adversarial-collaborative-filtering_amd._native")
    ctx = ops.APRContext(10, 10, 8, 4, 1, dev)
    bad = torch.tensor([0, 1, 2, 10], dtype=torch.int32, device=dev)
    ok = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device=dev)
    with pytest.raises(native.NativeIndexError):
        ctx.plan(ok, bad, ok, 4)
    with pytest.raises(native.NativeIndexError):
        ctx.plan(bad, ok, ok, 4)
    # a failed plan leaves the context unplanned
    with pytest.raises(native.NativeError):
        ctx.optimizer_step(_gpu_tables(np.zeros((10, 8), np.float32), np.zeros((10, 8), np.float32), dev),
                           ops.StepHParams(), 0)


def test_full_size_ml1m_epoch_deterministic(ops, acf, dev):
    """ml-1m-shaped epoch (1,941 batches of 512, d=64): graph replay and eager
    launches give the same bits; two runs give the same bits; everything finite."""
    ds = acf.ml1m_like(seed=2019)
    s = acf.DeviceSampler(ds, 512, dev, seed=0)
    ep = s.epoch(0)
    assert ep.n_batches == 1941
    U1, I1, d = ds.num_users + 1, ds.num_items + 1, 64
    g = torch.Generator().manual_seed(0)
    P0 = torch.nn.init.trunc_normal_(torch.empty(U1, d), 0, 0.01, -0.02, 0.02, generator=g)
    Q0 = torch.nn.init.trunc_normal_(torch.empty(I1, d), 0, 0.01, -0.02, 0.02, generator=g)
    results = []
    ctx = ops.APRContext(U1, I1, d, 512, 1941, dev)
    ctx.plan(ep.user, ep.item_pos, ep.item_neg, 512)
    for graph in (True, False, True):
        tabs = [P0.to(dev), Q0.to(dev), torch.full((U1, d), 0.1, device=dev),
                torch.full((I1, d), 0.1, device=dev)]
        ctx.train_planned(tabs, ops.StepHParams(adver=1), graph=graph)
        torch.cuda.synchronize()
        results.append([t.clone() for t in tabs])
    for a, b in zip(results[0], results[1]):
        assert torch.equal(a, b)
    for a, b in zip(results[0], results[2]):
        assert torch.equal(a, b)
    P, Q, aP, aQ = results[0]
    assert torch.isfinite(P).all() and torch.isfinite(Q).all()
    assert float(aP.min()) >= 0.1 and float(aQ.min()) >= 0.1
    # every touched row moved, untouched rows did not
    moved = (P != P0.to(dev)).any(1).cpu().numpy()
    touched = np.zeros(U1, bool)
    touched[ep.user.cpu().numpy()] = True
    assert np.array_equal(moved, touched)


@pytest.mark.parametrize("adver", [0, 1])
@pytest.mark.parametrize("mapping", ["wave", "group"])
def test_piecewise_calls_equal_one_call(ops, oracle, dev, adver, mapping):
    """train_planned over [0,2)+[2,5) and per-batch optimizer_step == one call,
    and all match the oracle (exercises the deferred flush across calls)."""
    U1, I1, d, B, nb = 40, 35, 64, 32, 5
    P, Q, u, i, j = _problem(17 + adver, U1, I1, d, B, nb, dup_items=True)
    want, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=adver))
    hp = ops.StepHParams(adver=adver)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_slot_mapping(mapping)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    a = _gpu_tables(P, Q, dev)
    ctx.train_planned(a, hp, 0, 2, graph=True)
    ctx.train_planned(a, hp, 2, 3, graph=False)
    b = _gpu_tables(P, Q, dev)
    for t in range(nb):
        if adver:
            ctx.delta_update(b, hp, t)
        ctx.optimizer_step(b, hp, t)
    torch.cuda.synchronize()
    for x, y, w, n in zip(a, b, want, ("P", "Q", "accP", "accQ")):
        assert torch.equal(x, y), n
        _close(x, w, n)


@pytest.mark.parametrize("mapping", ["wave", "group"])
def test_hot_rows_many_occurrences(ops, oracle, dev, mapping, fp32_parity):
    """A few rows with hundreds of occurrences per batch (overflow records,
    many rounds per wave / group) still match the oracle."""
    U1, I1, d, B, nb = 12, 9, 64, 1024, 2
    P, Q, u, i, j = _problem(23, U1, I1, d, B, nb)
    want, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_slot_mapping(mapping)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        fp32_parity(g, w, n)


@pytest.mark.parametrize("mapping", ["wave", "group"])
@pytest.mark.parametrize("shape", ["hot", "large"])
def test_single_step_strict(ops, oracle, dev, mapping, shape):
    """One step of the shapes the multi-step tests hold to fp32_parity (hundreds
    of occurrences per row; B = 8,192 on 200k x 100k tables), losses included, at
    rtol max(1e-5, 2 n u) / atol 1e-6: n = the most terms any row sums (its
    occurrences, x2 for a user's pos and neg branch), u = 2^-24.  Two orders of
    an n-term fp32 sum may differ by 2 gamma_n = 2 n u relative to sum |terms|
    (Higham); at n ~ 230 (the hot shape) that is 2.7e-5, above a flat 1e-5."""
    if shape == "hot":
        U1, I1, d, B = 12, 9, 64, 1024
        P, Q, u, i, j = _problem(23, U1, I1, d, B, 1)
    else:
        U1, I1, d, B = 200_000, 100_000, 64, 8192
        rng = np.random.default_rng(5)
        P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
        Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
        u = rng.integers(0, U1, B).astype(np.int32)
        i = (rng.zipf(1.3, B) % I1).astype(np.int32)
        j = rng.integers(0, I1, B).astype(np.int32)
    want, lc_w, la_w, _ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, 1, dev)
    ctx.set_slot_mapping(mapping)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    lc, la = ctx.losses()
    n_terms = max(2 * np.bincount(u).max(), np.bincount(np.concatenate([i, j])).max())
    rtol = max(RTOL, 2 * n_terms * 2.0 ** -24)
    for g, w, n in zip(tabs + [lc, la], list(want) + [lc_w, la_w], ("P", "Q", "accP", "accQ", "lc", "la")):
        np.testing.assert_allclose(g.cpu().numpy(), w, rtol=rtol, atol=ATOL, err_msg=f"{n} (rtol {rtol:.1e})")


def test_replan_reuses_graph(ops, oracle, dev):
    """A cached graph stays valid after a new plan (plan generation is read on device)."""
    U1, I1, d, B, nb = 50, 40, 32, 64, 3
    P, Q, u, i, j = _problem(31, U1, I1, d, B, 2 * nb)
    want, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    hp = ops.StepHParams(adver=1)
    for c in range(2):
        s = slice(c * nb * B, (c + 1) * nb * B)
        ctx.plan(torch.tensor(u[s], device=dev), torch.tensor(i[s], device=dev),
                 torch.tensor(j[s], device=dev), B)
        ctx.train_planned(tabs, hp, 0, nb, graph=True)
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        _close(g, w, n)


@pytest.mark.parametrize("d", [64, 128])
def test_large_batch_auto_mapping_matches_oracle(ops, oracle, dev, d, fp32_parity):
    """B = 8,192 (auto -> one lane-group per slot) on 200k x 100k tables."""
    U1, I1, B, nb = 200_000, 100_000, 8192, 2
    rng = np.random.default_rng(d)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = (rng.zipf(1.3, nb * B) % I1).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    want, *_ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        fp32_parity(g, w, n)


def _zipf_large(seed, U1, I1, d, B, nb, s=1.1):
    """Config-5-shaped batches: uniform users and negatives, Zipf
    positives, so a batch of 65,536 holds items with thousands of occurrences."""
    rng = np.random.default_rng(seed)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = ((rng.zipf(s, nb * B) - 1) % I1).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    return P, Q, u, i, j


@pytest.mark.parametrize("d,adver", [(64, 1), (128, 1), (64, 0)])
def test_hot_slots_large_batch_match_oracle(ops, oracle, dev, d, adver, fp32_parity):
    """B = 65,536 with Zipf positives: slots with more than ACF_HOT_MIN (8)
    occurrences run as pieces + a combine of the pieces (inside k_tri_combine, or
    for the clean pass at the head of k_tri_cadv; the top item has ~3,000
    occurrences per batch).  Tables and losses vs the oracle, and the hot path
    really ran (kind 'hot' launches)."""
    U1, I1, B, nb = 300_000, 200_000, 65536, 2
    P, Q, u, i, j = _zipf_large(d + adver, U1, I1, d, B, nb)
    assert np.bincount(i[:B]).max() > 1000
    want, lc_w, la_w, _ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=adver))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    t = ctx.time_kernels(tabs, ops.StepHParams(adver=adver))
    # one combine launch per pass, hot slots combined inside; (r06) on the hash plan
    # the clean pass's combine rides in the adversarial launch (k_tri_cadv)
    assert ctx.plan_kind() == "hash"
    assert t["hot"][1] == nb  # APR: the adversarial combine; BPR: its one combine
    assert t["adv"][1] == (nb if adver else 0)
    lc, la = ctx.losses()
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        fp32_parity(g, w, n)
    n_terms = max(2 * np.bincount(u).max(), np.bincount(np.concatenate([i, j])).max())
    rtol = max(RTOL, 2 * n_terms * 2.0 ** -24)  # Higham bound, as test_single_step_strict
    np.testing.assert_allclose(lc.cpu().numpy(), lc_w, rtol=rtol, atol=ATOL)
    if adver:
        np.testing.assert_allclose(la.cpu().numpy(), la_w, rtol=rtol, atol=ATOL)
    assert ctx.step_errors() == 0


def test_hot_slots_deterministic(ops, dev):
    """The hot lists are appended with atomics (their order varies run to run);
    each slot's pieces are still summed in piece order, so two runs give
    identical bits, graph or eager."""
    U1, I1, d, B, nb = 200_000, 100_000, 64, 32768, 3
    P, Q, u, i, j = _zipf_large(3, U1, I1, d, B, nb)
    runs = []
    for graph in (False, True, True):
        tabs = _gpu_tables(P, Q, dev)
        ctx = ops.APRContext(U1, I1, d, B, nb, dev)
        ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
        ctx.train_planned(tabs, ops.StepHParams(adver=1), graph=graph)
        lc, la = ctx.losses()
        runs.append(tabs + [lc.clone(), la.clone()])
    for other in runs[1:]:
        for x, y in zip(runs[0], other):
            assert torch.equal(x, y)


@pytest.mark.parametrize("B,adver", [(32768, 1), (32768, 0), (4096, 1)])
def test_hash_plan_matches_sort_plan(ops, dev, B, adver):
    """The hash plan (k_hplan_*: triplet-centric plans, the default) against the
    device-wide sort plan: identical bits through the triplet-centric step, whole
    range and piecewise (both planners), on Zipf positives whose top items have
    thousands of occurrences per batch (the workgroup bitmap ranks), tens (the
    wave ranks) and up to 8 (the per-thread network)."""
    U1, I1, d, nb = 200_000, 100_000, 64, 3
    P, Q, u, i, j = _zipf_large(11 + B + adver, U1, I1, d, B, nb)
    cnt = np.bincount(np.concatenate([i[:B], j[:B]]))
    assert cnt.max() > 64 and ((cnt > 8) & (cnt <= 64)).any() and ((cnt > 1) & (cnt <= 8)).any()
    hp = ops.StepHParams(adver=adver, reg=0.01)
    uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
    runs = []
    for mode, pieces in (("sort", [(0, nb)]), ("auto", [(0, nb)]), ("auto", [(0, 1), (1, nb - 1)]),
                         ("sort", [(0, 1), (1, nb - 1)])):
        ctx = ops.APRContext(U1, I1, d, B, nb, dev)
        ctx.set_plan_mode(mode)
        ctx.plan(uu, ii, jj, B)
        assert ctx.plan_kind() == ("hash" if mode == "auto" else "sort")
        tabs = _gpu_tables(P, Q, dev)
        for first, n in pieces:
            ctx.train_planned(tabs, hp, first, n, graph=first == 0)
        lc, la = ctx.losses()
        assert ctx.step_errors() == 0
        runs.append(tabs + [lc.clone(), la.clone()])
    torch.cuda.synchronize()
    names = ("P", "Q", "accP", "accQ", "loss_clean", "loss_adv")
    for other in runs[1:]:
        for x, y, n in zip(runs[0], other, names):
            if n == "loss_adv" and not adver:
                continue
            assert torch.equal(x, y), n


def test_hash_plan_crowded_partition_rounds(ops, dev):
    """A batch whose users all hash into ONE partition of the hash plan (the top
    partition bits of k_hplan's Fibonacci hash equal): ~2,000 distinct users there,
    more than a partition round holds (3/4 of its LDS buckets), so the partition
    is split into rounds by further hash bits.  The bits equal the sort plan's."""
    U1, I1, d, B, nb = 300_000, 50_000, 32, 4096, 2
    pb = 5  # hplan_pbits(4096, 384): 12,288 occurrences / 384 -> 32 partitions
    rows = np.arange(U1, dtype=np.uint64)
    part = ((rows * 2654435761) & 0xFFFFFFFF) >> (32 - pb)
    crowd = rows[part == part[12345]].astype(np.int32)
    assert len(crowd) > 4000
    rng = np.random.default_rng(21)
    u = rng.choice(crowd[:2000], nb * B).astype(np.int32)  # ~2,000 distinct users, ~2 occurrences each
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    hp = ops.StepHParams(adver=1, reg=0.01)
    uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
    runs = []
    for mode in ("sort", "auto"):
        ctx = ops.APRContext(U1, I1, d, B, nb, dev)
        ctx.set_plan_mode(mode)
        ctx.plan(uu, ii, jj, B)
        assert ctx.plan_kind() == ("hash" if mode == "auto" else "sort")
        tabs = _gpu_tables(P, Q, dev)
        ctx.train_planned(tabs, hp)
        lc, la = ctx.losses()
        assert ctx.step_errors() == 0
        runs.append(tabs + [lc.clone(), la.clone()])
    torch.cuda.synchronize()
    for x, y, n in zip(*runs, ("P", "Q", "accP", "accQ", "loss_clean", "loss_adv")):
        assert torch.equal(x, y), n


def test_hash_plan_range_check(ops, dev):
    """A triplet index out of range raises from the hash plan too, and the next
    clean plan works."""
    from importlib import import_module
    native = import_module("adversarial-collaborative-filtering_amd._native")
    B = 4096
    ctx = ops.APRContext(5000, 5000, 16, B, 2, dev)
    ok = torch.arange(2 * B, dtype=torch.int32, device=dev) % 5000
    bad = ok.clone()
    bad[B + 7] = 5000
    with pytest.raises(native.NativeIndexError):
        ctx.plan(ok, bad, ok, B)
    assert ctx.plan(ok, ok, ok, B) == 2 and ctx.plan_kind() == "hash"


def _sparse_stream(seed, U1, I1, B, nb, hot=64, p_hot=0.05):
    """Mostly rows that occur once per batch (fused triplets), plus a small hot
    set that recurs across consecutive batches (pending / next-batch rows)."""
    rng = np.random.default_rng(seed)
    n = nb * B

    def draw(N):
        x = rng.integers(0, N, n)
        h = rng.random(n) < p_hot
        x[h] = rng.integers(0, hot, int(h.sum()))
        return x.astype(np.int32)
    return draw(U1), draw(I1), draw(I1)


def _fused_fraction(u, i, j, B):
    frac = []
    for t in range(len(u) // B):
        s = slice(t * B, (t + 1) * B)
        cu = np.unique(u[s], return_counts=True)
        ci = np.unique(np.concatenate([i[s], j[s]]), return_counts=True)
        once_u = set(cu[0][cu[1] == 1].tolist())
        once_i = set(ci[0][ci[1] == 1].tolist())
        frac.append(np.mean([a in once_u and b in once_i and c in once_i
                             for a, b, c in zip(u[s], i[s], j[s])]))
    return float(np.mean(frac))


@pytest.mark.parametrize("d", [16, 64, 128, 512])
@pytest.mark.parametrize("adver,adv", [(0, "grad"), (1, "grad"), (1, "random")])
@pytest.mark.parametrize("mapping", ["wave", "group"])
def test_fused_triplets_bit_identical_to_slot_path(ops, dev, d, adver, adv, mapping):
    """Triplet fusion on vs off: identical bits for tables, accumulators and
    losses, over one call and over piecewise calls (in-place rows, rows pending
    from the previous batch, rows read by the next one)."""
    U1, I1, B, nb = 6000, 5000, 256, 6
    u, i, j = _sparse_stream(d + adver, U1, I1, B, nb)
    assert _fused_fraction(u, i, j, B) > 0.5
    rng = np.random.default_rng(d)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=adver, adv=adv, reg=0.01, seed=5)
    runs = []
    # "random" draws fresh noise every call (the call counter is part of its key),
    # so piecewise calls are compared only in gradient mode; a fresh context per
    # run starts every run at the same counter
    cases = ((False, [(0, nb)]), (True, [(0, nb)])) + ((True, [(0, 1), (1, 3), (4, 2)]),) * (adv == "grad")
    for fuse, pieces in cases:
        ctx = ops.APRContext(U1, I1, d, B, nb, dev)
        ctx.set_slot_mapping(mapping)
        ctx.set_fusion(fuse)  # before the plan: a triplet-centric plan updates rows in place
        ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
        tabs = _gpu_tables(P, Q, dev)
        for first, n in pieces:
            ctx.train_planned(tabs, hp, first, n, graph=first == 0)
        lc, la = ctx.losses()
        runs.append(tabs + [lc.clone(), la.clone()])
    torch.cuda.synchronize()
    names = ("P", "Q", "accP", "accQ", "loss_clean", "loss_adv")
    for other in runs[1:]:
        for x, y, n in zip(runs[0], other, names):
            if n == "loss_adv" and not adver:
                continue
            assert torch.equal(x, y), n


@pytest.mark.parametrize("adver", [0, 1])
def test_fused_large_batch_matches_oracle(ops, oracle, dev, adver, fp32_parity):
    """B = 8,192 on 400k x 300k tables (~85% fused triplets) vs the oracle."""
    U1, I1, d, B, nb = 400_000, 300_000, 64, 8192, 3
    u, i, j = _sparse_stream(40 + adver, U1, I1, B, nb, hot=256, p_hot=0.02)
    assert _fused_fraction(u, i, j, B) > 0.8
    rng = np.random.default_rng(adver)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    want, lc_w, la_w, _ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=adver))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=adver))
    lc, la = ctx.losses()
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        fp32_parity(g, w, n)
    _close(lc, lc_w, "loss_clean")
    if adver:
        _close(la, la_w, "loss_adv")


@pytest.mark.parametrize("overlap", [False, True, None])
@pytest.mark.parametrize("chunk", [1, 3, 7])
def test_plan_pipeline_equals_sequential(ops, dev, chunk, overlap):
    """PlanPipeline (next chunk planned on a side stream) == plan + train per
    chunk in sequence, bit for bit; the chunking itself is exact because every
    train_planned call ends with its flush."""
    U1, I1, d, B, nb = 300, 200, 64, 64, 10
    u, i, j = _sparse_stream(77, U1, I1, B, nb, hot=16, p_hot=0.3)
    rng = np.random.default_rng(7)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1)
    ut, it, jt = (torch.tensor(x, device=dev) for x in (u, i, j))
    a = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.plan(ut, it, jt, B)
    ctx.train_planned(a, hp, 0, nb)
    b = _gpu_tables(P, Q, dev)
    pipe = ops.PlanPipeline(U1, I1, d, B, chunk, dev, overlap=overlap)
    pipe.run(b, hp, ut, it, jt)
    pipe.run(b, hp, ut, it, jt, 2, 5)  # a second pass over a sub-range reuses the graphs
    ctx.plan(ut[2 * B: 7 * B], it[2 * B: 7 * B], jt[2 * B: 7 * B], B)
    ctx.train_planned(a, hp, 0, 5)
    torch.cuda.synchronize()
    for x, y, n in zip(a, b, ("P", "Q", "accP", "accQ")):
        assert torch.equal(x, y), n


def _overlap_stream(shape, acf, dev, B, nb, seed):
    if shape == "hot":  # rows recur inside and across batches (CSR occurrences, t-1 / t-2 sources)
        rng = np.random.default_rng(seed)
        U1, I1 = 40, 30
        u, i, j = (rng.integers(0, N, nb * B).astype(np.int32) for N in (U1, I1, I1))
        return U1, I1, u, i, j
    if shape == "sparse":  # mostly fused triplets, in-place rows, a hot set
        U1, I1 = 6000, 5000
        return (U1, I1) + _sparse_stream(seed, U1, I1, B, nb)
    ds = acf.ml1m_like()
    ep = acf.DeviceSampler(ds, B, dev, seed=seed).epoch(0)
    s = slice(0, nb * B)
    return (ds.num_users + 1, ds.num_items + 1) + tuple(x[s].cpu().numpy() for x in
                                                        (ep.user, ep.item_pos, ep.item_neg))


@pytest.mark.parametrize("d", [8, 32, 64, 128, 256, 512])
@pytest.mark.parametrize("shape", ["hot", "sparse", "ml1m"])
@pytest.mark.parametrize("fuse", [False, True])
def test_stream_bit_identical_to_two_kernels(ops, acf, dev, d, shape, fuse):
    """Streamed steps (k_stream: the whole range in one launch through tagged row
    versions; d > 256 falls back to two kernels) vs two kernels per step:
    identical bits for tables, accumulators and both losses, over one call
    (graph and eager) and over piecewise calls; no wait gave up.  (r04 also ran
    the overlapped step k_ovl here; it was removed in r05.)"""
    if shape == "ml1m" and d not in (32, 64):
        pytest.skip("ml1m shape at the headline dims only")
    B, nb = {"hot": (64, 12), "sparse": (256, 8), "ml1m": (512, 24)}[shape]
    U1, I1, u, i, j = _overlap_stream(shape, acf, dev, B, nb, seed=d + 3)
    rng = np.random.default_rng(d)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1, reg=0.01, seed=5)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_fusion(fuse)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    runs = []
    split = [(0, 1), (1, 2), (3, 4), (7, nb - 7)]
    for stream, pieces, graph in ((False, [(0, nb)], True), (False, [(0, nb)], False), (False, split, True),
                                  (True, [(0, nb)], True), (True, [(0, nb)], False), (True, split, True),
                                  (True, split, False)):
        ctx.set_stream(stream)
        tabs = _gpu_tables(P, Q, dev)
        for first, n in pieces:
            ctx.train_planned(tabs, hp, first, n, graph=graph)
        lc, la = ctx.losses()
        runs.append(tabs + [lc.clone(), la.clone()])
        assert ctx.step_errors() == 0
    torch.cuda.synchronize()
    names = ("P", "Q", "accP", "accQ", "loss_clean", "loss_adv")
    for k, other in enumerate(runs[1:]):
        for x, y, n in zip(runs[0], other, names):
            assert torch.equal(x, y), (k, n)


def test_two_kernel_timing_kinds(ops, dev):
    """time_kernels reports the launch sequence train_planned runs with streamed
    steps off: a clean and an adv launch per batch and one flush launch (and
    matches training)."""
    U1, I1, d, B, nb = 300, 200, 64, 128, 9
    u, i, j = _sparse_stream(5, U1, I1, B, nb, hot=16, p_hot=0.3)
    rng = np.random.default_rng(1)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_stream(False)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ta, tb = _gpu_tables(P, Q, dev), _gpu_tables(P, Q, dev)
    t = ctx.time_kernels(ta, hp)
    assert {k: v[1] for k, v in t.items()} == {"clean": nb, "adv": nb, "flush": 1, "stream": 0, "hot": 0}
    ctx.train_planned(tb, hp)
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)


@pytest.mark.parametrize("d", [16, 64, 256])
def test_stream_kernel_timing_kinds(ops, dev, d):
    """With streamed steps on, train_planned runs ONE k_stream launch for the
    whole plan, its write-back in the launch's tail (time_kernels reports exactly
    that), and a partial range one k_stream plus a k_stream_flush launch; the
    results equal training."""
    U1, I1, B, nb = 300, 200, 128, 9
    u, i, j = _sparse_stream(5, U1, I1, B, nb, hot=16, p_hot=0.3)
    rng = np.random.default_rng(1)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_stream(True)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ta, tb = _gpu_tables(P, Q, dev), _gpu_tables(P, Q, dev)
    t = ctx.time_kernels(ta, hp)
    assert {k: v[1] for k, v in t.items()} == {"clean": 0, "adv": 0, "flush": 0, "stream": 1, "hot": 0}
    ctx.train_planned(tb, hp)
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)
    t = ctx.time_kernels(ta, hp, 2, nb - 2)
    assert {k: v[1] for k, v in t.items()} == {"clean": 0, "adv": 0, "flush": 1, "stream": 1, "hot": 0}
    ctx.train_planned(tb, hp, 2, nb - 2)
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)
    assert ctx.step_errors() == 0


@pytest.mark.parametrize("fuse", [0, 1])
def test_stream_give_up_replays_exactly(ops, acf, dev, fuse):
    """k_stream failure safety (it needs all of its waves resident): with a spin
    limit of 0 every hand-off wait gives up at once, the gated flush writes
    nothing, and the verified call replays the chunk on the two-kernel schedule --
    the same bits as set_stream(False), no step error, the replay counted.  With
    failsafe off the give-up is reported by step_errors and the tables are left
    exactly as they were."""
    B, nb, d = 512, 24, 64
    U1, I1, u, i, j = _overlap_stream("ml1m", acf, dev, B, nb, seed=11)
    rng = np.random.default_rng(3)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1, reg=0.01, seed=5)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_fusion(fuse)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.set_stream(False)
    ref = _gpu_tables(P, Q, dev)
    ctx.train_planned(ref, hp)
    ref_l = [x.clone() for x in ctx.losses()]
    ctx.set_stream(True)
    ctx.set_spin_limit(0)
    for pieces in ([(0, nb)], [(0, 5), (5, nb - 5)]):
        before = ctx.stream_recoveries()
        got = _gpu_tables(P, Q, dev)
        for first, n in pieces:
            ctx.train_planned(got, hp, first, n)
        torch.cuda.synchronize()
        assert ctx.stream_recoveries() - before >= 1
        assert ctx.step_errors() == 0
        for x, y in zip(ref + ref_l, got + list(ctx.losses())):
            assert torch.equal(x, y)
    ctx.set_failsafe(False)
    got = _gpu_tables(P, Q, dev)
    ctx.train_planned(got, hp)
    torch.cuda.synchronize()
    assert ctx.step_errors() & 1
    for x, y in zip(_gpu_tables(P, Q, dev), got):
        assert torch.equal(x, y)
    # and a normal limit again: the streamed call goes through without a replay
    ctx.set_failsafe(True)
    ctx.set_spin_limit(1 << 16)
    before = ctx.stream_recoveries()
    got = _gpu_tables(P, Q, dev)
    ctx.train_planned(got, hp)
    torch.cuda.synchronize()
    assert ctx.step_errors() == 0 and ctx.stream_recoveries() == before
    for x, y in zip(ref, got):
        assert torch.equal(x, y)


def test_unverified_give_up_reported_and_next_call_applied(ops, acf, dev):
    """failsafe off: a streamed call that gives up is dropped and
    reported; its failure word is the launch's own (seq-tagged), so the NEXT call
    is applied normally, and the report stays until step_errors() reads it,
    switching failsafe back on included."""
    B, nb, d = 512, 12, 64
    U1, I1, u, i, j = _overlap_stream("ml1m", acf, dev, B, 2 * nb, seed=13)
    rng = np.random.default_rng(4)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1)
    first = [torch.tensor(x[:nb * B], device=dev) for x in (u, i, j)]
    second = [torch.tensor(x[nb * B:], device=dev) for x in (u, i, j)]
    # reference: the second call's batches alone, on the two-kernel schedule
    ref = _gpu_tables(P, Q, dev)
    rctx = ops.APRContext(U1, I1, d, B, nb, dev)
    rctx.set_stream(False)
    rctx.plan(*second, B)
    rctx.train_planned(ref, hp)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_failsafe(False)
    got = _gpu_tables(P, Q, dev)
    ctx.set_spin_limit(0)
    ctx.plan(*first, B)
    ctx.train_planned(got, hp)  # gives up: dropped
    ctx.set_spin_limit(1 << 16)
    ctx.plan(*second, B)
    ctx.train_planned(got, hp)  # applied
    torch.cuda.synchronize()
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
    ctx.set_failsafe(True)
    assert ctx.step_errors() & 1  # the first call's report survived the second call and the toggle
    assert ctx.step_errors() == 0 and ctx.stream_recoveries() == 0


def test_pipeline_failed_chunks_gate_and_replay(ops, acf, dev):
    """Verified calls without a host sync: with a spin limit of 0 every streamed
    chunk of a PlanPipeline gives up; the first failure gates the later chunks
    of both contexts, and the re-plan of a context (and the final settling)
    replays them in order -- the tables equal the two-kernel schedule's bits."""
    B, chunk, nb, d = 512, 4, 12, 64
    U1, I1, u, i, j = _overlap_stream("ml1m", acf, dev, B, nb, seed=17)
    rng = np.random.default_rng(5)
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    hp = ops.StepHParams(adver=1, reg=0.01)
    tu, ti, tj = (torch.tensor(x, device=dev) for x in (u, i, j))
    ref = _gpu_tables(P, Q, dev)
    rp = ops.PlanPipeline(U1, I1, d, B, chunk, dev, overlap=False)
    rp.set_stream(False)
    rp.run(ref, hp, tu, ti, tj)
    pipe = ops.PlanPipeline(U1, I1, d, B, chunk, dev, overlap=False)
    pipe.set_spin_limit(0)
    got = _gpu_tables(P, Q, dev)
    pipe.run(got, hp, tu, ti, tj)
    pipe.resolve()
    assert pipe.stream_recoveries() == nb // chunk
    assert pipe.step_errors() == 0
    for x, y in zip(ref, got):
        assert torch.equal(x, y)
    # and with a normal limit: nothing replayed, the same bits
    pipe.set_spin_limit(1 << 16)
    got = _gpu_tables(P, Q, dev)
    pipe.run(got, hp, tu, ti, tj)
    torch.cuda.synchronize()
    assert pipe.stream_recoveries() == nb // chunk and pipe.step_errors() == 0
    for x, y in zip(ref, got):
        assert torch.equal(x, y)


@pytest.mark.parametrize("case", ["one_per_batch", "identical", "identical_large", "edge_rows"])
@pytest.mark.parametrize("stream", [False, True])
def test_degenerate_batches_match_oracle(ops, oracle, dev, case, stream):
    """Edge cases of the batch shape against the oracle: one triplet per batch;
    batches of B identical triplets (one user slot and one or two item slots with
    B occurrences each; in the first batch the negative IS the positive, so the
    item's contributions cancel pair by pair); the same at B = 4,096 (hash plan,
    hot-slot pieces); only the first and last rows of both tables."""
    U1, I1, d = 37, 29, 64
    rng = np.random.default_rng(len(case))
    if case == "one_per_batch":
        B, nb = 1, 6
        u, i, j = rng.integers(0, U1, nb), rng.integers(0, I1, nb), rng.integers(0, I1, nb)
    elif case.startswith("identical"):
        B, nb = (4096, 2) if case == "identical_large" else (256, 3)
        u = np.full(nb * B, 3)
        i = np.full(nb * B, 5)
        j = np.full(nb * B, 7)
        j[:B] = 5
    else:
        B, nb = 64, 4
        u = rng.choice([0, U1 - 1], nb * B)
        i, j = rng.choice([0, I1 - 1], nb * B), rng.choice([0, I1 - 1], nb * B)
    u, i, j = (x.astype(np.int32) for x in (u, i, j))
    P = (rng.standard_normal((U1, d)) * 0.3).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.3).astype(np.float32)
    want, lc_w, la_w, _ = _oracle_run(oracle, P, Q, u, i, j, B, HParams(adver=1))
    tabs = _gpu_tables(P, Q, dev)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_stream(stream)
    ctx.plan(torch.tensor(u, device=dev), torch.tensor(i, device=dev), torch.tensor(j, device=dev), B)
    ctx.train_planned(tabs, ops.StepHParams(adver=1))
    lc, la = ctx.losses()
    torch.cuda.synchronize()
    assert ctx.step_errors() == 0
    # a row's sum over n occurrences in another order (lane-group teams, hot-slot
    # pieces): Higham's bound 2 n u, relative to the row's scale, as test_hot_slots_*
    n_terms = max(2 * np.bincount(u[:B]).max(), np.bincount(np.concatenate([i[:B], j[:B]])).max())
    rtol = max(RTOL, 2 * n_terms * 2.0 ** -24)
    for g, w, n in zip(tabs, want, ("P", "Q", "accP", "accQ")):
        atol = max(ATOL, rtol * float(np.abs(w).max()))
        np.testing.assert_allclose(g.cpu().numpy(), w, rtol=rtol, atol=atol, err_msg=n)
    np.testing.assert_allclose(lc.cpu().numpy(), lc_w, rtol=rtol, atol=ATOL)
    np.testing.assert_allclose(la.cpu().numpy(), la_w, rtol=rtol, atol=ATOL)
