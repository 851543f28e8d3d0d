"""The split APR step (distributed.ShardedAPR) over gloo on CPU:
users and items row-sharded over the ranks, triplets routed by user, the
item sums completed by their owners through all_to_all exchanges.  The local
passes are the oracle's restatement of the HIP shard passes
(oracle/shard_oracle.py); the routing, exchange plans and collectives are the
product code.  Result vs one process training the full tables (the C oracle)
at the fp32 bar (tests/conftest.py fp32_parity): the item sums are added in a
different order (per rank, then over ranks), nothing else differs."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO

U1, I1, D, B, NB, CHUNK = 53, 41, 16, 32, 6, 4


def _problem(hot=False):
    rng = np.random.default_rng(12)
    P = (rng.standard_normal((U1, D)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, D)) * 0.2).astype(np.float32)
    u = rng.integers(0, U1, NB * B).astype(np.int32)
    i = rng.integers(0, I1, NB * B).astype(np.int32)
    j = rng.integers(0, I1, NB * B).astype(np.int32)
    j[::13] = i[::13]  # the trainList quirk allows i == j
    if hot:
        i[::3] = 7  # one item in a third of every batch, on every rank
    return P, Q, u, i, j


def _worker(rank, world, port, out_dir, adver, reg, hot, exchange="all_to_all"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from apr_oracle import HParams
    from shard_oracle import OracleShardLocal
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    P, Q, u, i, j = _problem(hot)
    sh = D_.ShardedAPR(U1, I1, D, B, init_P=P, init_Q=Q, local=OracleShardLocal, item_exchange=exchange)
    assert sh.P.shape[0] == len(range(rank, U1, world))  # only this rank's rows
    assert sh.Q.shape[0] == len(range(rank, I1, world))
    sh.train(u, i, j, HParams(adver=adver, reg=reg), chunk=CHUNK)
    full = sh.full_tables()
    stats = np.array([sh.stats["triplets"], sh.stats["steps"]])
    if rank == 0:
        np.savez(os.path.join(out_dir, "sharded.npz"), *[t.numpy() for t in full])
    np.save(os.path.join(out_dir, f"stats{rank}.npy"), stats)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,adver,reg,hot,exchange", [(2, 1, 0.0, False, "all_to_all"),
                                                          (2, 0, 0.0, False, "all_to_all"),
                                                          (3, 1, 0.01, True, "all_to_all"),
                                                          (2, 1, 0.0, True, "all_to_all"),
                                                          (2, 1, 0.0, False, "allgather"),
                                                          (3, 1, 0.01, True, "allgather")])
def test_split_step_equals_single_process(tmp_path, oracle, fp32_parity, world, adver, reg, hot, exchange):
    """exchange "allgather": E1 as the all_gather of every Q shard (north_star's
    form for configs[2]) instead of the working-set all_to_all."""
    from apr_oracle import HParams
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), adver, reg, hot, exchange), nprocs=world, join=True)
    got = np.load(os.path.join(tmp_path, "sharded.npz"))
    P, Q, u, i, j = _problem(hot)
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    oracle.apr_train(P, Q, aP, aQ, u, i, j, B, HParams(adver=adver, reg=reg))
    for k, (want, n) in enumerate(zip((P, Q, aP, aQ), ("P", "Q", "accP", "accQ"))):
        fp32_parity(got[f"arr_{k}"], want, n)
    # every triplet ran exactly once, on its user's rank
    per_rank = [np.load(os.path.join(tmp_path, f"stats{r}.npy")) for r in range(world)]
    assert sum(int(s[0]) for s in per_rank) == NB * B
    for r, s in enumerate(per_rank):
        assert int(s[0]) == int(np.sum(u % world == r)) and int(s[1]) == NB


def _bad_worker(rank, world, port, out_dir, kind):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from apr_oracle import HParams
    from shard_oracle import OracleShardLocal
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    P, Q, u, i, j = _problem()
    if kind == "routed":  # each rank holds its own users' triplets; rank 1 slips in a foreign one
        sel = np.nonzero(u % world == rank)[0][: B // world * NB]
        u, i, j = u[sel].copy(), i[sel].copy(), j[sel].copy()
        if rank == 1:
            u[5] = 0  # user 0 lives on rank 0
        sh = D_.ShardedAPR(U1, I1, D, B, init_P=P, init_Q=Q, local=OracleShardLocal, local_batch=B // world)
        run = lambda: sh.train_routed(u, i, j, HParams(adver=1), chunk=CHUNK)
    else:  # the same global stream on every rank, corrupted on rank 1 only
        if rank == 1:
            {"neg": u, "item": i, "neg_item": j}[kind][7] = -3 if kind != "item" else I1
        sh = D_.ShardedAPR(U1, I1, D, B, init_P=P, init_Q=Q, local=OracleShardLocal)
        run = lambda: sh.train(u, i, j, HParams(adver=1), chunk=CHUNK)
    try:
        run()
        res = "ok"
    except (IndexError, ValueError) as e:
        res = type(e).__name__
    with open(os.path.join(out_dir, f"res{rank}.txt"), "w") as f:
        f.write(res)
    dist.barrier()  # reached by every rank: nobody is left waiting in a collective
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind,want", [("neg", "IndexError"), ("item", "IndexError"), ("neg_item", "IndexError"),
                                       ("routed", "ValueError")])
def test_bad_triplet_on_one_rank_raises_on_every_rank(tmp_path, kind, want):
    """a bad triplet on ONE rank must make EVERY rank raise the same
    error before any rank enters the next collective (no hang on the peers)."""
    world = 2
    mp.spawn(_bad_worker, args=(world, _free_port(), str(tmp_path), kind), nprocs=world, join=True)
    for r in range(world):
        with open(os.path.join(tmp_path, f"res{r}.txt")) as f:
            assert f.read() == want, f"rank {r}"


def _skew_worker(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from apr_oracle import HParams
    from shard_oracle import OracleShardLocal
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    P, Q, u, i, j = _skew_problem()
    sh = D_.ShardedAPR(SK_U1, SK_I1, D, SK_B, init_P=P, init_Q=Q, local=OracleShardLocal)
    sh.train(u, i, j, HParams(adver=1), chunk=2)
    full = sh.full_tables()
    if rank == 0:
        np.savez(os.path.join(out_dir, "skew.npz"), *[t.numpy() for t in full])
    np.save(os.path.join(out_dir, f"C{rank}.npy"), np.array([sh._C]))
    dist.barrier()
    dist.destroy_process_group()


SK_U1, SK_I1, SK_B, SK_NB = 64, 400, 256, 4


def _skew_problem():
    rng = np.random.default_rng(21)
    P = (rng.standard_normal((SK_U1, D)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((SK_I1, D)) * 0.2).astype(np.float32)
    u = rng.integers(0, SK_U1, SK_NB * SK_B).astype(np.int32)
    u[rng.random(u.size) < 0.9] &= ~1  # 90% of the triplets on rank 0's (even) users
    i = rng.integers(0, SK_I1, SK_NB * SK_B).astype(np.int32)
    j = rng.integers(0, SK_I1, SK_NB * SK_B).astype(np.int32)
    return P, Q, u, i, j


def test_split_step_skewed_ranks_share_block_size(tmp_path, oracle, fp32_parity):
    """One rank requests many more item rows per step than the other: the fixed
    exchange blocks (distributed.py "Static step layout") must still have ONE size on
    every rank, or the equal-split all_to_alls would disagree."""
    from apr_oracle import HParams
    world = 2
    mp.spawn(_skew_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    Cs = [int(np.load(os.path.join(tmp_path, f"C{r}.npy"))[0]) for r in range(world)]
    assert Cs[0] == Cs[1] and Cs[0] > 64, Cs
    got = np.load(os.path.join(tmp_path, "skew.npz"))
    P, Q, u, i, j = _skew_problem()
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    oracle.apr_train(P, Q, aP, aQ, u, i, j, SK_B, HParams(adver=1))
    for k, (want, n) in enumerate(zip((P, Q, aP, aQ), ("P", "Q", "accP", "accQ"))):
        fp32_parity(got[f"arr_{k}"], want, n)


def _lifetime_worker(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import gc
    import weakref
    from apr_oracle import HParams
    from shard_oracle import OracleShardLocal
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    P, Q, u, i, j = _problem()
    res = []
    # with-block: close() runs at its end
    with D_.ShardedAPR(U1, I1, D, B, init_P=P, init_Q=Q, local=OracleShardLocal) as sh:
        sh.train(u, i, j, HParams(adver=1), chunk=CHUNK)
        fin = sh._finalizer
    res.append(not fin.alive)
    # the local passes see the object through a weak proxy: no cycle, so dropping
    # the last reference runs the finalizer at once (no gc pass needed)
    gc.disable()
    sh = D_.ShardedAPR(U1, I1, D, B, init_P=P, init_Q=Q, local=OracleShardLocal)
    sh.train(u, i, j, HParams(adver=1), chunk=CHUNK)
    fin, ref = sh._finalizer, weakref.ref(sh)
    del sh
    res.append(not fin.alive and ref() is None)
    gc.enable()
    np.save(os.path.join(out_dir, f"life{rank}.npy"), np.array(res))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_lifetime_close_with_and_drop():
    """ShardedAPR releases its captured graphs (and anything else its finalizer
    holds) at close(), at the end of a with-block, or as soon as the last
    reference goes: the local passes hold only a weak proxy (world 2, gloo)."""
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_lifetime_worker, args=(2, _free_port(), tmp), nprocs=2, join=True)
        for r in range(2):
            assert np.load(os.path.join(tmp, f"life{r}.npy")).all()
