"""ShardedTables on the GPU through the nccl (RCCL) backend, world size 1 in this
process: the all-gather / write-back path runs on device tensors and the step is
the HIP kernels (distributed.hip_step).  Multi-rank behaviour is covered on CPU
with gloo (test_distributed.py); 8-GPU runs are the driver's."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import PKG

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("adver", [0, 1])
def test_sharded_rccl_equals_single_context(ops, dev, adver):
    D_ = importlib.import_module(PKG + ".distributed")
    U1, I1, d, B, nb = 500, 300, 64, 128, 6
    rng = np.random.default_rng(adver)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u = rng.integers(0, U1, nb * B).astype(np.int32)
    i = rng.integers(0, I1, nb * B).astype(np.int32)
    j = rng.integers(0, I1, nb * B).astype(np.int32)
    hp = ops.StepHParams(adver=adver)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sh = D_.ShardedTables(U1, I1, d, device=dev, init_P=P, init_Q=Q)
        for c in range(0, nb, 3):
            s = slice(c * B, (c + 3) * B)
            sh.train_chunk(u[s], i[s], j[s], B, hp)
        got = sh.full_tables()
    finally:
        dist.destroy_process_group()
    tabs = [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    ctx = ops.APRContext(U1, I1, d, B, 3, dev)
    for c in range(0, nb, 3):
        s = slice(c * B, (c + 3) * B)
        ctx.plan(torch.tensor(u[s], device=dev), torch.tensor(i[s], device=dev), torch.tensor(j[s], device=dev), B)
        ctx.train_planned(tabs, hp, graph=False)
    torch.cuda.synchronize()
    for x, y, n in zip(got, tabs, ("P", "Q", "accP", "accQ")):
        assert torch.equal(x, y), n
