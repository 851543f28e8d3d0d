#!/usr/bin/env python
"""Does a one-rank RCCL collective survive hipGraph capture + replay here?
python3 tools/rccl_capture_probe.py {all_reduce|all_to_all|all_gather} [--pool]
(one probe per process, under an outer timeout: a hang is an answer too)."""
import os
import socket
import sys

import torch
import torch.distributed as dist


def main():
    kind = sys.argv[1]
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
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
