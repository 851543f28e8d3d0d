"""Row-sharded multi-process training (distributed.ShardedTables) with the gloo
backend on CPU, world size 2: bit-identical to one process training the full
tables.  The step function is the CPU oracle here (the HIP step on GPUs)."""
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

U1, I1, D, B, NB, CHUNK = 53, 41, 16, 32, 6, 3


def _problem():
    rng = np.random.default_rng(12)
    P = (rng.standard_normal((U1, D)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, D)) * 0.2).astype(np.float32)
    u = rng.integers(0, U1, NB * B).astype(np.int32)
    i = rng.integers(0, I1, NB * B).astype(np.int32)
    j = rng.integers(0, I1, NB * B).astype(np.int32)
    j[::13] = i[::13]
    return P, Q, u, i, j


def _oracle_step(P, Q, accP, accQ, u, i, j, batch_size, hp):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from apr_oracle import COracle
    arrs = [x.numpy() for x in (P, Q, accP, accQ)]
    COracle().apr_train(*arrs, u.numpy(), i.numpy(), j.numpy(), batch_size, hp)
    for t, a in zip((P, Q, accP, accQ), arrs):
        t.copy_(torch.from_numpy(a))


def _worker(rank, world, port, out_dir, adver):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from apr_oracle import HParams
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D_ = importlib.import_module(PKG + ".distributed")
    P, Q, u, i, j = _problem()
    sh = D_.ShardedTables(U1, I1, D, init_P=P, init_Q=Q)
    assert sh.P.shape[0] == len(range(rank, U1, world))  # only this rank's rows
    for c in range(0, NB, CHUNK):
        s = slice(c * B, (c + CHUNK) * B)
        sh.train_chunk(u[s], i[s], j[s], B, HParams(adver=adver), step_fn=_oracle_step)
    full = sh.full_tables()
    if rank == 0:
        np.savez(os.path.join(out_dir, "sharded.npz"), *[t.numpy() for t in full])
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("adver", [0, 1])
def test_sharded_equals_single_process(tmp_path, oracle, adver):
    from apr_oracle import HParams
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), adver), nprocs=world, join=True)
    got = np.load(os.path.join(tmp_path, "sharded.npz"))
    P, Q, u, i, j = _problem()
    aP, aQ = np.full_like(P, 0.1), np.full_like(Q, 0.1)
    oracle.apr_train(P, Q, aP, aQ, u, i, j, B, HParams(adver=adver))
    for k, want in enumerate((P, Q, aP, aQ)):
        np.testing.assert_array_equal(got[f"arr_{k}"], want)
