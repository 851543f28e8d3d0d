#!/usr/bin/env python
"""Fixed per-call cost of a short training call (the driver's `bench.py --steps 20`).

Replays bench.py's timed region for --steps batches (same data, tables, pipeline
and warm-up) with a marker kernel (torch.cuda._sleep -> `spin_kernel`) right
before and after it, so a `rocprofv3 --kernel-trace` of this script isolates the
timed region's dispatches.  Prints one JSON line: wall time of the region, host
time spent inside PlanPipeline.run (enqueue), and the per-batch rate.

Use with tools/trace_region.py:
  rocprofv3 --kernel-trace -f csv -d gpurun_out/sc -o sc -- python3 tools/short_call.py
  python3 tools/trace_region.py gpurun_out/sc/.../sc_kernel_trace.csv
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

PKG = "adversarial-collaborative-filtering_amd"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--reps", type=int, default=5, help="timed repetitions (each on fresh batches)")
    p.add_argument("--failsafe", type=int, default=1, help="verified streamed calls (1, default) or not (0)")
    p.add_argument("--same", action="store_true",
                   help="every rep repeats the same call (bench.py's timed call: PlanPipeline's fast path)")
    p.add_argument("--sched", default="", choices=["", "auto", "spin", "yield", "blocking"],
                   help="hipSetDeviceFlags schedule before the device is used (A/B of the host wait)")
    a = p.parse_args()
    if a.sched:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        flag = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}[a.sched]
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(flag))
        print(f"hipSetDeviceFlags({flag}) -> {rc}", file=sys.stderr)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    B, d = 512, 64
    ds = acf.ml1m_like(seed=2019)
    U1, I1 = ds.num_users + 1, ds.num_items + 1
    nbat = a.warmup + a.steps * (a.reps + 1)
    u, i, j = bench.make_triplets(acf, ds, B, max(nbat, 2 * a.steps + a.warmup), dev, seed=0)
    tabs = bench.init_tables(U1, I1, d, dev, seed=0)
    chunk = a.steps
    pipe = ops.PlanPipeline(U1, I1, d, B, chunk, dev, overlap=None)
    pipe.set_failsafe(bool(a.failsafe))
    hp = ops.StepHParams(lr=0.05, eps=0.5, reg=0.0, reg_adv=1.0, adver=1)
    pipe.run(tabs, hp, u, i, j, 0, max(a.warmup, 2 * chunk))
    torch.cuda.synchronize(dev)
    out = []
    for r in range(a.reps):
        first = a.warmup + (0 if a.same else r * a.steps)
        torch.cuda._sleep(1000)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pipe.run(tabs, hp, u, i, j, first, a.steps)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        torch.cuda._sleep(1000)
        torch.cuda.synchronize(dev)
        out.append({"region_us": round(1e6 * (t2 - t0), 1), "enqueue_us": round(1e6 * (t1 - t0), 1),
                    "triplets_per_s": round(a.steps * B / (t2 - t0), 1)})
    # floor of a timed region: one tiny kernel launch + synchronize
    floor = []
    for r in range(a.reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        tabs[0][0, 0].add_(0.0)
        torch.cuda.synchronize(dev)
        floor.append(round(1e6 * (time.perf_counter() - t0), 1))
    print(json.dumps({"steps": a.steps, "reps": out, "empty_region_us": floor,
                      "step_errors": pipe.step_errors()}), flush=True)


if __name__ == "__main__":
    main()
