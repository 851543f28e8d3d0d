"""Where the split step's chunk routing (distributed.ShardedAPR._route) spends its time,
configs[4] shape at world 1 (24 steps of 65,536 routed triplets, d = 128): a torch
profiler table of the GPU kernels and host ops of one routing call.
   python3 tools/route_profile.py > gpurun_out/route_profile.txt"""
import importlib
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
acf = importlib.import_module(bench.PKG)
D_ = importlib.import_module(bench.PKG + ".distributed")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", str(29600 + os.getpid() % 1000))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
big = acf.synthetic_large(device=dev)
b, d, T = 65536, 128, 24
ep = acf.DeviceSampler(big, b, dev, seed=11, weights=np.ones(big.num_items, np.float32)).epoch(0)
u, i, j = (x[: 2 * T * b].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
sh = D_.ShardedAPR(big.num_users + 1, big.num_items + 1, d, b, device=dev, local_batch=b)
sh._route(u[: T * b], i[: T * b], j[: T * b], T)  # warm (allocations, kernels)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
sh._route(u[T * b:], i[T * b:], j[T * b:], T)
torch.cuda.synchronize(dev)
print(f"route of {T} steps: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                        torch.profiler.ProfilerActivity.CUDA]) as prof:
    sh._route(u[T * b:], i[T * b:], j[T * b:], T)
    torch.cuda.synchronize(dev)
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=60))
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=15, max_name_column_width=60))
dist.destroy_process_group()
