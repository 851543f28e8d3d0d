"""configs[2]'s split step alone (world 1, pinterest-20-shaped, B = 512, d = 64), graph
replay vs eager, with the routing time of a chunk and the replay time apart:
   python3 tools/shard_pinterest.py [steps] [chunks]
   rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pp -o pp -- python3 tools/shard_pinterest.py"""
import importlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
acf = importlib.import_module(bench.PKG)
ops = importlib.import_module(bench.PKG + ".ops")
D_ = importlib.import_module(bench.PKG + ".distributed")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
nchunks = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # > 1: routing of chunk k + 1 beside chunk k
B, d = 512, 64
ds = acf.pinterest_like(seed=2019)
ep = acf.DeviceSampler(ds, B, dev, seed=3).epoch(0)
n = 3 * steps * B
u, i, j = (x[:n].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
hp = ops.StepHParams(adver=1)
out = {}
for graph in (True, False):
    sh = D_.ShardedAPR(ds.num_users + 1, ds.num_items + 1, d, B, device=dev, local_batch=B, graph=graph)
    g = torch.Generator(device=dev).manual_seed(5)
    sh.P.normal_(0, 0.01, generator=g)
    sh.Q.normal_(0, 0.01, generator=g)
    ck = steps // nchunks
    sh.train_routed(u[: steps * B], i[: steps * B], j[: steps * B], hp, chunk=ck)  # eager + capture (both sets)
    s = slice(steps * B, 2 * steps * B)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    c = sh._route(u[s], i[s], j[s], ck, 0)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    r0, rs0 = sh.stats["graph_replays"], sh.stats["route_s"]
    t2 = time.perf_counter()
    sh.train_routed(u[s], i[s], j[s], hp, chunk=ck)  # the bench's timed call: routing beside the steps
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    out["graph" if graph else "eager"] = {"route_ms_per_chunk": round(1e3 * (t1 - t0), 3), "chunk": ck,
                                           "call_us_per_step": round(1e6 * (t3 - t2) / steps, 2),
                                           "route_host_ms_in_call": round(1e3 * (sh.stats["route_s"] - rs0), 3),
                                           "replays_in_call": sh.stats["graph_replays"] - r0, "C": sh._C}
print(json.dumps(out))
dist.destroy_process_group()
