"""Can two ranks on ONE GPU form an RCCL (nccl backend) group here?  (probe)
Each rank runs an all_reduce, then a graph-captured all_reduce replayed twice.
Usage: python3 tools/rccl_two_ranks_probe.py   (spawns 2 processes on cuda:0)"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok1 = bool((x == 3.0).all())
    s = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    y = torch.full((1024,), float(rank + 1), device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        g.capture_begin(capture_error_mode="thread_local")
        dist.all_reduce(y)
        g.capture_end()
    torch.cuda.current_stream(dev).wait_stream(s)
    y.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    ok2 = bool((y == 3.0).all())
    del g
    print(f"rank {rank}: eager {ok1} captured {ok2}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    so = socket.socket(); so.bind(("127.0.0.1", 0)); port = so.getsockname()[1]; so.close()
    mp.spawn(work, args=(2, port), nprocs=2, join=True)
    sys.exit(0)
