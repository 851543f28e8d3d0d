"""Timeline of the configs[4] split step at world 1 (diagnostic), as
bench.sharded_lines runs it (train_routed, one chunk of --steps, captured),
bracketed by spin_kernel markers.  Run under `rocprofv3 --kernel-trace -f csv`;
--analyze <kernel_trace.csv> prints per-kernel time per step between the last
two markers and the idle time between launches."""
import argparse
import csv
import importlib
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PKG = "adversarial-collaborative-filtering_amd"


def run(steps):
    import numpy as np
    import torch
    import torch.distributed as tdist
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    D_ = importlib.import_module(PKG + ".distributed")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29000 + os.getpid() % 1000))
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    big = acf.synthetic_large(device=dev)
    b, d = 65536, 128
    sampler = acf.DeviceSampler(big, b, dev, seed=11, weights=np.ones(big.num_items, np.float32))
    ep = sampler.epoch(0)
    n = 2 * steps * b
    u, i, j = (x[:n].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
    del ep, sampler
    g = torch.Generator(device=dev).manual_seed(5)
    sh = D_.ShardedAPR(big.num_users + 1, big.num_items + 1, d, b, device=dev, local_batch=b)
    sh.P.normal_(0, 0.01, generator=g)
    sh.Q.normal_(0, 0.01, generator=g)
    hp = ops.StepHParams(adver=1)
    s = slice(0, steps * b)
    sh.train_routed(u[s], i[s], j[s], hp, chunk=steps)
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(100000)
    s = slice(steps * b, n)
    sh.train_routed(u[s], i[s], j[s], hp, chunk=steps)
    torch.cuda._sleep(100000)
    torch.cuda.synchronize(dev)
    print(json.dumps({"step_errors": sh.step_errors(), "graph_replays": sh.stats["graph_replays"]}))
    sh.close()
    tdist.destroy_process_group()


def analyze(path, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [k for k, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"]]
    a, z = marks[-2], marks[-1]
    seg = rows[a + 1:z]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    per = defaultdict(lambda: [0, 0])
    busy_end, idle = t0, 0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        per[name][0] += e - s
        per[name][1] += 1
        if s > busy_end:
            idle += s - busy_end
        busy_end = max(busy_end, e)
    out = {"span_us_per_step": round((t1 - t0) / 1e3 / steps, 2), "idle_us_per_step": round(idle / 1e3 / steps, 2),
           "kernels_us_per_step": {k: [round(v[0] / 1e3 / steps, 2), round(v[1] / steps, 2)]
                                   for k, v in sorted(per.items(), key=lambda kv: -kv[1][0])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--analyze", type=str, default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, a.steps)
    else:
        run(a.steps)
