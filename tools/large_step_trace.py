"""Timeline of a configs[4] training call (diagnostic): 10M x 5M Zipf, alias
negatives, B = 65,536, d from argv, --batches in chunks of 32 through
PlanPipeline, bracketed by spin_kernel markers.  Run under
`rocprofv3 --kernel-trace -f csv` and read the trace with --analyze."""
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


def run(d, nb, chunk):
    import numpy as np
    import torch
    acf = importlib.import_module(PKG)
    ops = importlib.import_module(PKG + ".ops")
    dev = torch.device("cuda", 0)
    ds = acf.synthetic_large(device=dev)
    U1, I1, B = ds.num_users + 1, ds.num_items + 1, 65536
    ep = acf.DeviceSampler(ds, B, dev, seed=7, weights=np.ones(ds.num_items, np.float32)).epoch(0)
    u, i, j = (x[: nb * B].contiguous() for x in (ep.user, ep.item_pos, ep.item_neg))
    del ep
    g = torch.Generator(device=dev).manual_seed(5)
    tabs = [torch.randn(U1, d, device=dev, generator=g) * 0.01, torch.randn(I1, d, device=dev, generator=g) * 0.01,
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    pipe = ops.PlanPipeline(U1, I1, d, B, chunk, dev)
    hp = ops.StepHParams(adver=1)
    pipe.run(tabs, hp, u, i, j, 0, nb)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    pipe.run(tabs, hp, u, i, j, 0, nb)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print(json.dumps({"ok": True, "step_errors": pipe.step_errors()}))


def analyze(path, nb):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [k for k, r in enumerate(rows) if "spin_kernel" in r[2]]
    reg = rows[marks[-2] + 1: marks[-1]]
    span = (max(e for _, e, _ in reg) - reg[0][0]) / 1e3
    dur = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in reg:
        key = n.split("(")[0].replace("void ", "")
        key = key if key.startswith("k_") else ("rocprim/other: " + key[:40])
        dur[key] += (e - s) / 1e3
        cnt[key] += 1
    # device-busy union of all kernels (concurrent plan kernels overlap the step)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in reg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    out = {"span_us": round(span, 1), "per_batch_us": round(span / nb, 2), "busy_union_us": round(busy / 1e3, 1),
           "kernels_us_per_batch": {k: [round(v / nb, 2), cnt[k]] for k, v in sorted(dur.items(), key=lambda x: -x[1])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--batches", type=int, default=128)
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--analyze", type=str, default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, a.batches)
    else:
        run(a.d, a.batches, a.chunk)
