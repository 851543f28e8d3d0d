"""Streamed step vs two-kernel step on the same plan: max |diff| per tensor
(diagnostic for k_stream; the GPU tests assert bit equality)."""
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
ops = importlib.import_module("adversarial-collaborative-filtering_amd.ops")


def run(d, B, nb, U1, I1, fuse, seed=0, depth=None):
    rng = np.random.default_rng(seed)
    u, i, j = (rng.integers(0, N, nb * B).astype(np.int32) for N in (U1, I1, I1))
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    dev = torch.device("cuda:0")
    hp = ops.StepHParams(adver=1)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_fusion(fuse)
    ctx.plan(*(torch.tensor(x, device=dev) for x in (u, i, j)), B)
    out = []
    for stream in (False, True):
        ctx.set_stream(stream)
        tabs = [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                torch.full(P.shape, 0.1, device=dev), torch.full(Q.shape, 0.1, device=dev)]
        ctx.train_planned(tabs, hp, graph=False)
        lc, la = ctx.losses()
        out.append(tabs + [lc.clone(), la.clone()])
        err = ctx.step_errors()
    diffs = [float((a - b).abs().max()) for a, b in zip(*out)]
    rows = [int(((a - b).abs().amax(dim=1) > 0).sum()) if a.dim() == 2 else int(((a - b) != 0).sum())
            for a, b in zip(*out)]
    print(f"d={d} B={B} nb={nb} U1={U1} I1={I1} fuse={fuse} err={err} maxdiff={diffs} rows={rows}", flush=True)




def locate(d=64, B=256, nb=6, U1=6000, I1=5000, fuse=False, seed=0):
    """First triplet whose clean loss differs, with its rows' batch occurrences."""
    rng = np.random.default_rng(seed)
    u, i, j = (rng.integers(0, N, nb * B).astype(np.int32) for N in (U1, I1, I1))
    P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
    Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
    dev = torch.device("cuda:0")
    hp = ops.StepHParams(adver=1)
    ctx = ops.APRContext(U1, I1, d, B, nb, dev)
    ctx.set_fusion(fuse)
    ctx.plan(*(torch.tensor(x, device=dev) for x in (u, i, j)), B)
    out = []
    for stream in (False, True):
        ctx.set_stream(stream)
        tabs = [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                torch.full(P.shape, 0.1, device=dev), torch.full(Q.shape, 0.1, device=dev)]
        ctx.train_planned(tabs, hp, graph=False)
        lc, la = ctx.losses()
        out.append((lc.cpu().numpy(), la.cpu().numpy()))
    bad = np.nonzero(out[0][0] != out[1][0])[0]
    print("clean-loss mismatches:", len(bad), "first:", bad[:10])
    for e in bad[:5]:
        t = e // B
        print(f" e={e} t={t} u={u[e]} i={i[e]} j={j[e]}")
        for name, arr, r in (("u", u, u[e]), ("i", np.concatenate([i, j]), i[e]), ("j", np.concatenate([i, j]), j[e])):
            occ = np.nonzero(arr == r)[0]
            bt = sorted(set(int(x % (nb * B)) // B for x in occ))
            print(f"   {name}={r} batches {bt} count_in_t={int(((occ % (nb * B)) // B == t).sum())}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "repeat":
        # stream vs stream: is the streamed result deterministic?
        d, B, nb, U1, I1 = 64, 256, 6, 6000, 5000
        rng = np.random.default_rng(0)
        u, i, j = (rng.integers(0, N, nb * B).astype(np.int32) for N in (U1, I1, I1))
        P = (rng.standard_normal((U1, d)) * 0.2).astype(np.float32)
        Q = (rng.standard_normal((I1, d)) * 0.2).astype(np.float32)
        dev = torch.device("cuda:0")
        hp = ops.StepHParams(adver=1)
        ctx = ops.APRContext(U1, I1, d, B, nb, dev)
        ctx.set_fusion(False)
        ctx.plan(*(torch.tensor(x, device=dev) for x in (u, i, j)), B)
        res = []
        for rep in range(4):
            tabs = [torch.tensor(P, device=dev), torch.tensor(Q, device=dev),
                    torch.full(P.shape, 0.1, device=dev), torch.full(Q.shape, 0.1, device=dev)]
            ctx.train_planned(tabs, hp, graph=False)
            lc, la = ctx.losses()
            res.append(lc.cpu().numpy().copy())
            print("rep", rep, "err", ctx.step_errors(), "mismatch vs rep0", int((res[-1] != res[0]).sum()), flush=True)
    elif len(sys.argv) > 1 and sys.argv[1] == "locate":
        locate(fuse=False)
        locate(fuse=False, nb=3)
        locate(fuse=False, nb=2)
    else:
        for d in (8, 64, 256):
            for fuse in (False, True):
                run(d, 64, 4, 61, 47, fuse)
                run(d, 256, 6, 6000, 5000, fuse)
