"""Adversarial NeuMF epoch rate only (bench.py's neumf line without the Adam roofline; GPU box)."""
import importlib
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
acf = importlib.import_module("adversarial-collaborative-filtering_amd")
if os.environ.get("ACF_NEUMF_LIB"):  # another build (A/B), without the build-hash check
    import ctypes
    nat = importlib.import_module("adversarial-collaborative-filtering_amd._native")
    lib = ctypes.CDLL(os.environ["ACF_NEUMF_LIB"])
    for fname, (res, args) in nat.NEUMF_SIGNATURES.items():
        fn = getattr(lib, fname)
        fn.restype, fn.argtypes = res, args
    nat._neumf = lib
nm = importlib.import_module("adversarial-collaborative-filtering_amd.neumf")
ds = acf.yelp_like()
train = sp.coo_matrix((np.ones(len(ds.pair_user), np.float32), (ds.pair_user, ds.pair_item)),
                      shape=(ds.num_users, ds.num_items))
B = 512
r = nm.AdversarialNeuMF(ds.num_users, ds.num_items, 64, weight=1.0, pop_percent=0.2, seed=0, device="cuda")
x, y = r.get_train_instances(train)
perm = np.random.default_rng(0).permutation(len(y))
U = torch.as_tensor(x[0][perm], dtype=torch.int32, device="cuda")
I = torch.as_tensor(x[1][perm], dtype=torch.int32, device="cuda")
Y = torch.as_tensor(y[perm], dtype=torch.float32, device="cuda")
ctx = r._context(B)
if os.environ.get("ROWS_IN_LINE") == "0":  # A/B: the k_nmf_rows path
    ctx.set_rows_in_line(False)
hp = r.hparams()
ctx.train(U[: 64 * B], I[: 64 * B], Y[: 64 * B], B, hp)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    losses = ctx.train(U, I, Y, B, hp)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("rep %d: %.0f instances/s  %.4f ms/step  loss %.5f" % (
        rep, len(y) / dt, 1e3 * dt / losses.shape[0],
        float(losses[-1, 0])), flush=True)
