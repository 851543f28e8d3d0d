"""The split APR step (distributed.ShardedAPR) with the HIP shard
passes and owner kernels:

* world 1 over RCCL (nccl backend) on a pinterest-20-shaped problem
  (55,187 x 9,916, d = 64, B = 512, BASELINE configs[2]) and a Zipf large
  batch (hot items: pieces + combine in shard mode), vs the C oracle;
* world 2 on ONE GPU (two processes, gloo with host staging for the
  all_to_alls): the real two-way split of every batch, HIP kernels on both
  ranks, vs the C oracle.  8-GPU runs over RCCL/xGMI are the driver's.
"""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(seed, U1, I1, d, B, nb, zipf=None):
    rng = np.random.default_rng(seed)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    if zipf:
        i = ((rng.zipf(zipf, nb * B) - 1) % I1).astype(np.int32)
    else:
        i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    j[::29] = i[::29]
    return P, Q, u, i, j


def _want(oracle, P, Q, u, i, j, B, adver, reg=0.0):
    from apr_oracle import HParams
    P, Q = P.copy(), Q.copy()
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    oracle.apr_train(P, Q, aP, aQ, u, i, j, B, HParams(adver=adver, reg=reg))
    return P, Q, aP, aQ


@pytest.mark.parametrize("shape,adver,reg,exchange", [("pinterest", 1, 0.0, "all_to_all"),
                                                      ("pinterest", 0, 0.0, "all_to_all"),
                                                      ("pinterest", 1, 0.01, "all_to_all"),
                                                      ("zipf_large", 1, 0.0, "all_to_all"),
                                                      ("pinterest", 1, 0.0, "allgather"),
                                                      ("pinterest", 0, 0.01, "allgather")])
def test_sharded_rccl_world1_matches_oracle(ops, oracle, dev, fp32_parity, shape, adver, reg, exchange):
    """exchange "allgather": E1 as the RCCL all_gather of the Q shards (configs[2]'s form)."""
    D_ = importlib.import_module(PKG + ".distributed")
    if shape == "pinterest":
        U1, I1, d, B, nb, z = 55_188, 9_917, 64, 512, 12, None
    else:
        U1, I1, d, B, nb, z = 300_000, 200_000, 64, 32768, 2, 1.1
    P, Q, u, i, j = _problem(adver, U1, I1, d, B, nb, z)
    want = _want(oracle, P, Q, u, i, j, B, adver, reg)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, item_exchange=exchange)
        uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
        sh.train(uu, ii, jj, ops.StepHParams(adver=adver, reg=reg), chunk=5)
        got = sh.full_tables()
        assert sh.step_errors() == 0
        assert sh.stats["triplets"] == nb * B
    finally:
        dist.destroy_process_group()
    for g, w, n in zip(got, want, ("P", "Q", "accP", "accQ")):
        fp32_parity(g, w, n)


@pytest.mark.parametrize("adver,reg,routed,shape", [(1, 0.0, False, "zipf"), (0, 0.01, False, "zipf"),
                                                    (1, 0.0, True, "zipf"), (1, 0.0, False, "pinterest"),
                                                    (1, 0.0, True, "pinterest")])
def test_sharded_triplet_centric_matches_slot_path(ops, dev, adver, reg, routed, shape):
    """(r05) Shard mode on the hash plan and the triplet-centric kernels (local
    batches above 1,024 triplets with fusion on, the default: item occurrences
    are never single, item slots export their partial sums straight to the
    exchange rows, pass 1 reads the owners' deltas from theirs) against the sort
    plan and the slot kernels (fusion off): identical bits for every table, on
    Zipf batches of 32,768 with hot items, every exchange forced through a
    one-rank RCCL group, eager (train) and captured (train_routed).  (r06)
    "pinterest": configs[2]'s 512-triplet local batches, a chunk of them on one
    hash plan too (HipLocal.chunk_min 0)."""
    D_ = importlib.import_module(PKG + ".distributed")
    if shape == "zipf":
        U1, I1, d, B, nb = 300_000, 200_000, 64, 32768, 4
        P, Q, u, i, j = _problem(21 + adver, U1, I1, d, B, nb, 1.1)
    else:
        U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 8
        P, Q, u, i, j = _problem(23 + adver, U1, I1, d, B, nb)
        i[::5] = 17  # a hot item in every batch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    outs, kinds = [], []
    try:
        uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
        for fusion in (False, True):
            with D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, force_collectives=True,
                               local_batch=B if routed else None) as sh:
                for c in sh.local.ctxs:
                    c.set_fusion(fusion)
                hp = ops.StepHParams(adver=adver, reg=reg)
                (sh.train_routed if routed else sh.train)(uu, ii, jj, hp, chunk=2 if shape == "zipf" else 4)
                torch.cuda.synchronize(dev)
                assert sh.step_errors() == 0
                kinds.append(sh.local.ctx.plan_kind())  # the context the passes used (r06: the chunk plan's)
                outs.append(sh.full_tables())
    finally:
        dist.destroy_process_group()
    assert kinds == ["sort" if shape == "zipf" else "shard", "hash"], kinds
    for g, e, n in zip(outs[1], outs[0], ("P", "Q", "accP", "accQ")):
        assert torch.equal(g, e), n


@pytest.mark.parametrize("exchange,adver,reg,routed", [("all_to_all", 1, 0.0, False), ("allgather", 1, 0.0, True),
                                                       ("all_to_all", 0, 0.01, False), ("all_to_all", 1, 0.0, True)])
def test_sharded_graph_replay_bit_identical(ops, dev, exchange, adver, reg, routed):
    """The captured step graphs (one hipGraph per chunk at world 1, distributed.py
    "Static step layout") replay the eager step sequence bit for bit, on
    pinterest-20-shaped data (configs[2]), 3 chunks of 4 steps: the first is run
    eagerly and captured, the next ones replay."""
    D_ = importlib.import_module(PKG + ".distributed")
    U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 12
    P, Q, u, i, j = _problem(5 + adver, U1, I1, d, B, nb)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    outs, replays = [], []
    try:
        uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
        for graph in (False, True):
            sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, item_exchange=exchange, graph=graph,
                               local_batch=B if routed else None)
            hp = ops.StepHParams(adver=adver, reg=reg)
            (sh.train_routed if routed else sh.train)(uu, ii, jj, hp, chunk=4)
            torch.cuda.synchronize(dev)
            assert sh.step_errors() == 0
            outs.append(sh.full_tables())
            replays.append(sh.stats["graph_replays"])
    finally:
        dist.destroy_process_group()
    assert replays[0] == 0 and replays[1] >= 1, replays
    for g, e, n in zip(outs[1], outs[0], ("P", "Q", "accP", "accQ")):
        assert torch.equal(g, e), n


@pytest.mark.parametrize("exchange,routed", [("all_to_all", False), ("allgather", True)])
def test_sharded_collectives_captured_in_graph_world1(ops, dev, exchange, routed):
    """The RCCL collectives of the split step captured INSIDE the step graph
    (capture_collectives), rehearsed on one GPU: force_collectives issues every
    exchange through a one-rank nccl group (an RCCL self-exchange) instead of the
    world-1 identity.  With capture_collectives=True the constructor's capture
    check passes, a chunk is ONE graph, and eager / collectives-in-graph runs give
    identical bits (pinterest-20 shape, configs[2]); with the collectives kept out
    of graphs (capture_collectives=False, and the default since r06: ADVICE r05)
    a chunk is captured as segments cut at every collective (the plans in line
    while capturing: r04's pipelined plan straddled the cuts) and gives the same
    bits.  Both captured objects are then dropped without close(): the finalizer
    releases the graphs before the process group is destroyed -- in segment mode
    too, whose recorded collectives hold no reference to the object."""
    D_ = importlib.import_module(PKG + ".distributed")
    U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 12
    P, Q, u, i, j = _problem(9, U1, I1, d, B, nb)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    outs, segs = [], []
    try:
        uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
        for graph, cap in ((False, False), (None, None), (True, True)):
            sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, item_exchange=exchange, graph=graph,
                               local_batch=B if routed else None, force_collectives=True, capture_collectives=cap)
            on = bool(cap)  # the default (None) keeps the collectives between segments
            assert sh._cap_coll == on and sh.graph == (graph is not False)
            hp = ops.StepHParams(adver=1)
            (sh.train_routed if routed else sh.train)(uu, ii, jj, hp, chunk=4)
            torch.cuda.synchronize(dev)
            assert sh.step_errors() == 0
            outs.append(sh.full_tables())
            segs.append([len(r.segs) for r in sh._graphs.values()])
            assert (sh.stats["graph_replays"] >= 1) == (graph is not False)
            graphs = sh._graphs
            if graph is not False:
                assert graphs
                del sh  # no close(): the finalizer drops the graphs
                if graphs:  # never expected; drop them before the group goes (a hang otherwise)
                    graphs.clear()
                    pytest.fail("the captured graphs outlived the last reference to their ShardedAPR")
            else:
                sh.close()
                del sh
    finally:
        dist.destroy_process_group()
    assert segs[0] == [] and segs[1] and min(segs[1]) > 1, segs  # segments cut at the collectives
    assert segs[2] and segs[2] == [1] * len(segs[2]), segs  # one graph per chunk
    for o in outs[1:]:
        for g, e, n in zip(o, outs[0], ("P", "Q", "accP", "accQ")):
            assert torch.equal(g, e), n


@pytest.mark.parametrize("adver", [1, 0])
def test_shard_plan_small_matches_sort_plan(ops, dev, adver):
    """The one-workgroup shard plan (k_shard_plan, one batch of B <= 1,024) against
    the device-wide sort plan (plan mode 1) in shard mode: the same bits after 6
    split steps on pinterest-20-shaped data, with a hot item in every batch (hot
    lists, pieces) and i == j triplets."""
    D_ = importlib.import_module(PKG + ".distributed")
    U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 6
    P, Q, u, i, j = _problem(11 + adver, U1, I1, d, B, nb)
    i[::5] = 17
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    outs = []
    try:
        uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
        for mode in (0, 1):
            sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, graph=False)
            sh.local.chunk_min = 1 << 30  # one plan per step (r06: chunks of equal batches take one hash plan)
            for c in sh.local.ctxs:  # both step contexts (the next step is planned beside this one)
                c.set_plan_mode(mode)
            sh.train(uu, ii, jj, ops.StepHParams(adver=adver), chunk=3)
            torch.cuda.synchronize(dev)
            assert sh.step_errors() == 0
            outs.append(sh.full_tables())
    finally:
        dist.destroy_process_group()
    for a, b, n in zip(outs[0], outs[1], ("P", "Q", "accP", "accQ")):
        assert torch.equal(a, b), n


# two-rank problems: (U1, I1, d, B, nb, zipf, chunk); "pinterest" is BASELINE configs[2]'s
# shape (the reference's global batch of 512 split over the ranks)
SHAPES2 = {"zipf": (20_000, 9_000, 64, 4096, 4, 1.2, 3), "pinterest": (55_188, 9_917, 64, 512, 10, None, 4)}


def _worker(rank, world, port, out_dir, adver, exchange="all_to_all", shape="zipf"):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    ops = importlib.import_module(PKG + ".ops")
    U1, I1, d, B, nb, z, chunk = SHAPES2[shape]
    P, Q, u, i, j = _problem(7 + adver, U1, I1, d, B, nb, z)
    sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, item_exchange=exchange)
    uu, ii, jj = (torch.tensor(x, device=dev) for x in (u, i, j))
    sh.train(uu, ii, jj, ops.StepHParams(adver=adver), chunk=chunk)
    full = sh.full_tables()
    if rank == 0:
        np.savez(os.path.join(out_dir, "w2.npz"), *[t.cpu().numpy() for t in full])
    np.save(os.path.join(out_dir, f"n{rank}.npy"), np.array([sh.stats["triplets"], sh.step_errors()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("adver,exchange,shape", [(1, "all_to_all", "zipf"), (0, "all_to_all", "zipf"),
                                                  (1, "allgather", "zipf"), (1, "all_to_all", "pinterest"),
                                                  (1, "allgather", "pinterest")])
def test_sharded_two_ranks_one_gpu_matches_oracle(oracle, fp32_parity, tmp_path, adver, exchange, shape):
    """shape "pinterest": configs[2] (55,187 x 9,916, d = 64, global batch 512) split over two
    ranks, both E1 forms."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), adver, exchange, shape), nprocs=world, join=True)
    got = np.load(os.path.join(tmp_path, "w2.npz"))
    U1, I1, d, B, nb, z, _ = SHAPES2[shape]
    P, Q, u, i, j = _problem(7 + adver, U1, I1, d, B, nb, z)
    want = _want(oracle, P, Q, u, i, j, B, adver)
    for k, (w, n) in enumerate(zip(want, ("P", "Q", "accP", "accQ"))):
        fp32_parity(got[f"arr_{k}"], w, n)
    runs = [np.load(os.path.join(tmp_path, f"n{r}.npy")) for r in range(world)]
    assert sum(int(x[0]) for x in runs) == len(u) and all(int(x[1]) == 0 for x in runs)
