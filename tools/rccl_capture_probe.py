#!/usr/bin/env python
"""Does a one-rank RCCL collective survive hipGraph capture + replay here?
python3 tools/rccl_capture_probe.py {all_reduce|all_to_all|all_gather} [destroy|del|del_destroy|exit]
python3 tools/rccl_capture_probe.py sharded {exit|del_destroy|with_destroy}
(one probe per process, under an outer timeout: a hang is an answer too).

"sharded" (r05): a split step (distributed.ShardedAPR, default settings, every
exchange forced through the one-rank RCCL group) whose chunks were captured WITH
their collectives, then torn down without close(): "exit" leaves it alive at
interpreter exit (its weakref.finalize drops the graphs before the process
group's destructor), "del_destroy" drops the object and destroys the group,
"with_destroy" uses the with-block."""
import os
import socket
import sys

import torch
import torch.distributed as dist


def sharded(dev, mode):
    import importlib
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    pkg = "adversarial-collaborative-filtering_amd"
    D_ = importlib.import_module(pkg + ".distributed")
    ops = importlib.import_module(pkg + ".ops")
    U1, I1, d, B, nb = 55_188, 9_917, 64, 512, 12
    rng = np.random.default_rng(9)
    u, i, j = (torch.tensor(rng.integers(0, n, nb * B).astype(np.int32), device=dev) for n in (U1, I1, I1))

    def run(sh):
        sh.P.normal_(0, 0.01)
        sh.Q.normal_(0, 0.01)
        sh.train(u, i, j, ops.StepHParams(adver=1), chunk=4)
        torch.cuda.synchronize()
        print("sharded cap_coll", sh._cap_coll, "graphs", len(sh._graphs), "replays", sh.stats["graph_replays"],
              "step_errors", sh.step_errors(), flush=True)
    if mode == "with_destroy":
        with D_.ShardedAPR(U1, I1, d, B, device=dev, force_collectives=True) as sh:
            run(sh)
        dist.destroy_process_group()
        print("sharded destroyed", flush=True)
        return
    sh = D_.ShardedAPR(U1, I1, d, B, device=dev, force_collectives=True)
    run(sh)
    if mode == "del_destroy":
        del sh
        dist.destroy_process_group()
        print("sharded destroyed", flush=True)
        return
    print("sharded exit without close()", flush=True)


def main():
    kind = sys.argv[1]
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if kind == "sharded":
        sharded(dev, sys.argv[2] if len(sys.argv) > 2 else "exit")
        return
    x = torch.arange(64, dtype=torch.float32, device=dev)
    y = torch.empty_like(x)
    side = torch.cuda.Stream(dev)
    print(kind, "eager warm-up", flush=True)
    if kind == "all_reduce":
        dist.all_reduce(x)
    elif kind == "all_to_all":
        dist.all_to_all_single(y, x)
    else:
        dist.all_gather_into_tensor(y, x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side.wait_stream(torch.cuda.current_stream())
    print(kind, "capture", flush=True)
    with torch.cuda.stream(side):
        g.capture_begin(capture_error_mode="thread_local")
        x.mul_(1.0)
        if kind == "all_reduce":
            dist.all_reduce(x)
        elif kind == "all_to_all":
            dist.all_to_all_single(y, x)
        else:
            dist.all_gather_into_tensor(y, x)
        g.capture_end()
    print(kind, "replay", flush=True)
    x.copy_(torch.arange(64, dtype=torch.float32, device=dev) + 1)
    g.replay()
    torch.cuda.synchronize()
    print(kind, "replayed", flush=True)
    want = torch.arange(64, dtype=torch.float32, device=dev) + 1
    got = x if kind == "all_reduce" else y
    print(kind, "ok" if torch.equal(got, want) else f"WRONG {got[:4].tolist()}", flush=True)
    mode = sys.argv[2] if len(sys.argv) > 2 else "destroy"
    if mode in ("del", "del_destroy"):
        del g
        torch.cuda.synchronize()
        print(kind, "graph deleted", flush=True)
    if mode in ("destroy", "del_destroy"):
        dist.destroy_process_group()
        print(kind, "destroyed", flush=True)


if __name__ == "__main__":
    main()
