"""Phase timing of k_nmf_inst (workgroup 0, clean pass) from the -DNMF_DIAG build
(tools/libacf_neumf_diag.so, s_memrealtime at 100 MHz).  GPU box only."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
native = importlib.import_module("adversarial-collaborative-filtering_amd._native")
lib = native.load_neumf(os.path.join(REPO, "tools", "libacf_neumf_diag.so"))
lib.acf_neumf_diag_stamps.argtypes = [ctypes.c_void_p]
nm = importlib.import_module("adversarial-collaborative-filtering_amd.neumf")
U, I, d, B = 25678, 25816, int(sys.argv[1]) if len(sys.argv) > 1 else 64, 512
st = nm.NeuMFState(U, I, d, "cuda")
st.keras_init(0)
ctx = nm.NeuMFContext(st, B)
rng = np.random.default_rng(0)
names = ["prologue", "stash", "fwd1", "fwd2", "head", "dz2", "bwd2", "bwd1", "wgrad_tiles", "bias+sync"]
for rep in range(5):
    u = rng.integers(0, U, B).astype(np.int32)
    i = rng.integers(0, I, B).astype(np.int32)
    y = (rng.random(B) < 0.5).astype(np.float32)
    ctx.grad(u, i, y, ctx.hparams(adver=1))
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 32)()
    lib.acf_neumf_diag_stamps(buf)
    t = np.array(buf[:11], dtype=np.int64)
    dt = np.diff(t) * 10 / 1000.0  # us
    print("rep", rep, " ".join(f"{n}={x:.2f}" for n, x in zip(names, dt)), f"total={dt.sum():.2f}us")
    rt = np.array(buf[16:22], dtype=np.int64)
    rd = np.diff(rt) * 10 / 1000.0
    print("    rows", " ".join(f"{n}={x:.2f}" for n, x in zip(["stage", "first", "accum", "g_store", "delta"], rd)),
          f"total={rd.sum():.2f}us", f"(starts {(rt[0] - t[-1]) * 10 / 1000.0:.2f}us after inst wg0 end)")
    wt = np.array(buf[24:28], dtype=np.int64)
    wd = np.diff(wt) * 10 / 1000.0
    print("    wgrad", " ".join(f"{n}={x:.2f}" for n, x in zip(["loads", "lds+sync", "tiles"], wd)),
          f"(starts {(wt[0] - t[0]) * 10 / 1000.0:.2f}us after inst wg0 start)")
