"""Run only the dedup plan (for rocprofv3 kernel breakdowns).
Usage (GPU): python tools/plan_only.py B nb d reps"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ops = importlib.import_module("adversarial-collaborative-filtering_amd.ops")

B, nb, d, reps = (int(x) for x in sys.argv[1:5])
U1, I1 = 10_000_001, 5_000_001
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
u = torch.randint(0, U1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
i = torch.randint(0, I1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
j = torch.randint(0, I1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
ctx = ops.APRContext(U1, I1, d, B, nb, dev)
for _ in range(reps):
    ctx.plan(u, i, j, B, check=False)
torch.cuda.synchronize()
print("ok")
