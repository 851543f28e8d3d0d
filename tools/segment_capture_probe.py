"""r05: root cause of the caching-allocator assertion that removed the r03
segment capture of the split step.

The r03 path captured a chunk's steps as hipGraph SEGMENTS cut at every
collective (distributed._SegmentRecorder), the collectives running eagerly
between segment replays.  r04 added the pipelined plan (the plan of step t + 1
forked onto a side stream beside step t and joined before step t + 1) and then
met "HIPCachingAllocator ... use_count" when the segment path ran over RCCL.

This probe re-creates that path on one GPU: a world-1 nccl group with every
exchange forced through RCCL (force_collectives), collectives NOT captured, and
the segment capture re-enabled by hand (sh.graph = True after construction).
Variants, each in its own process under a time limit:

  pipe    the pipelined plan on (the r04 configuration);
  nopipe  the pipelined plan off (the r03 configuration).

Each prints what capture raised (or "ok" and whether the replays equal the
eager run bit for bit).  Usage: python tools/segment_capture_probe.py VARIANT
"""
import importlib
import os
import socket
import sys
import traceback

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "adversarial-collaborative-filtering_amd"


def main(variant: str) -> int:
    D_ = importlib.import_module(PKG + ".distributed")
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda", 0)
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 12
    rng = np.random.default_rng(9)
    P = (rng.standard_normal((U1, d)) * 0.1).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.1).astype(np.float32)
    u, i, j = (torch.tensor(rng.integers(0, n, nb * B).astype(np.int32), device=dev) for n in (U1, I1, I1))
    hp = ops.StepHParams(adver=1)
    outs = []
    rc = 0
    try:
        for seg in (False, True):
            sh = D_.ShardedAPR(U1, I1, d, B, device=dev, init_P=P, init_Q=Q, graph=seg, force_collectives=True,
                               capture_collectives=False)
            if seg:
                sh.graph = True  # the r03 segment capture, collectives between the segments
            if variant == "nopipe":
                sh._pipelined = lambda: False
            try:
                sh.train(u, i, j, hp, chunk=4)
                torch.cuda.synchronize(dev)
                outs.append(sh.full_tables())
                print(f"{variant} seg={seg}: ok, replays {sh.stats['graph_replays']}, "
                      f"segments per graph {[len(r.segs) for r in sh._graphs.values()]}", flush=True)
            except BaseException as e:  # noqa: BLE001
                print(f"{variant} seg={seg}: {type(e).__name__}: {str(e).splitlines()[0][:400]}", flush=True)
                traceback.print_exc()
                rc = 1
            sh.close()
            del sh
        if len(outs) == 2:
            same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
            print(f"{variant}: segments == eager bit for bit: {same}", flush=True)
    finally:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "pipe"))
