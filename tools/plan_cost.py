"""Where the time of a chunk goes: dedup plan alone, training alone (hipGraph
replay of an already planned chunk), plan + train in sequence, and the
PlanPipeline.  Usage (GPU): python tools/plan_cost.py [--large]"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "adversarial-collaborative-filtering_amd"


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def case(ops, acf, name, U1, I1, d, B, nb, chunk, dev, stream=None):
    if stream is None:
        g = torch.Generator(device=dev).manual_seed(1)
        u = torch.randint(0, U1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
        i = torch.randint(0, I1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
        j = torch.randint(0, I1, (B * nb,), device=dev, generator=g, dtype=torch.int32)
    else:
        u, i, j = stream
    tabs = [torch.randn(U1, d, device=dev) * 0.01, torch.randn(I1, d, device=dev) * 0.01,
            torch.full((U1, d), 0.1, device=dev), torch.full((I1, d), 0.1, device=dev)]
    hp = ops.StepHParams(adver=1)
    ctx = ops.APRContext(U1, I1, d, B, chunk, dev)
    s = slice(0, chunk * B)
    out = {"case": name, "B": B, "d": d, "chunk": chunk}
    out["plan_us_per_batch"] = 1e6 * timeit(lambda: ctx.plan(u[s], i[s], j[s], B, check=False), 5) / chunk
    ctx.plan(u[s], i[s], j[s], B, check=False)
    out["train_us_per_batch"] = 1e6 * timeit(lambda: ctx.train_planned(tabs, hp, 0, chunk), 5) / chunk
    ctx.set_fusion(False)
    out["train_nofuse_us_per_batch"] = 1e6 * timeit(lambda: ctx.train_planned(tabs, hp, 0, chunk), 5) / chunk
    ctx.set_fusion(True)

    def seq():
        for b in range(0, nb, chunk):
            n = min(chunk, nb - b)
            ss = slice(b * B, (b + n) * B)
            ctx.plan(u[ss], i[ss], j[ss], B, check=False)
            ctx.train_planned(tabs, hp, 0, n)
    out["sequential_us_per_batch"] = 1e6 * timeit(seq, 2) / nb
    for ov in (False, True):
        pipe = ops.PlanPipeline(U1, I1, d, B, chunk, dev, overlap=ov)
        out[f"pipeline_overlap{int(ov)}_us_per_batch"] = 1e6 * timeit(lambda: pipe.run(tabs, hp, u, i, j, 0, nb), 2) / nb
        del pipe
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--ml-chunks", type=int, nargs="*", default=None)
    ap.add_argument("--large-chunks", type=int, nargs="*", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = importlib.import_module(PKG + ".ops")
    acf = importlib.import_module(PKG)
    ds = acf.ml1m_like(seed=2019)
    sampler = acf.DeviceSampler(ds, 512, dev, seed=0)
    eps = [sampler.epoch(e) for e in range(3)]
    st = [torch.cat([getattr(e, f) for e in eps]).contiguous() for f in ("user", "item_pos", "item_neg")]
    nb_ml = st[0].numel() // 512
    for chunk in (a.ml_chunks or [647, 1941]):
        case(ops, acf, "ml1m", ds.num_users + 1, ds.num_items + 1, 64, 512, 3 * 1941, chunk, dev,
             [x[: 3 * 1941 * 512] for x in st])
    if a.large:
        for d in (64, 128):
            for chunk in (a.large_chunks or [1, 2, 8]):
                case(ops, acf, "10Mx5M", 10_000_001, 5_000_001, d, 65536, max(16, 2 * chunk), chunk, dev)
    del nb_ml


if __name__ == "__main__":
    main()
