"""End-to-end statistical parity run on the reference's Video dataset.

Reproduces the protocol behind out/janEval/Video_apr_d64_e0.5_l1.0_*.out:
  run_adv_ori.py --model apr --dataset Video --epochs 2000 --adv_epoch 1000
                 --verbose 20 --eval_mode all --embed_size 64
through this build's CLI (cli.main), with the Video files rebuilt from
tests/golden/video_data.npz, and compares the best-epoch HR@10 / NDCG@10 and
the trajectory with the published log (tests/golden/published_logs.json).

Usage: python tools/e2e_video.py [--epochs 2000] [--adv_epoch 1000] [--out DIR]
"""
import argparse
import importlib
import json
import os
import re
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=2000)
    ap.add_argument("--adv_epoch", type=int, default=1000)
    ap.add_argument("--verbose", type=int, default=20)
    ap.add_argument("--model", default="apr")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "e2e"))
    a = ap.parse_args()
    summary, _ = run(a.epochs, a.adv_epoch, a.verbose, a.model, a.seed, os.path.abspath(a.out))
    print(json.dumps(summary))


def trajectory(text):
    """{epoch: (HR@100, NDCG@100, |P|, |Q|)} from an .out log (utils.py:95-97 format)."""
    pat = re.compile(r"Epoch (\d+) \[.*?HR = ([\d.]+), NDCG = ([\d.]+).*?\|P\|=([\d.]+), \|Q\|=([\d.]+)")
    return {int(m.group(1)): tuple(float(m.group(k)) for k in range(2, 6)) for m in pat.finditer(text)}


def run(epochs=2000, adv_epoch=1000, verbose=20, model="apr", seed=0, out=None):
    """The published protocol through cli.main; returns (summary, log text)."""
    a = argparse.Namespace(epochs=epochs, adv_epoch=adv_epoch, verbose=verbose, model=model, seed=seed,
                           out=out)
    cwd = os.getcwd()
    cli = importlib.import_module("adversarial-collaborative-filtering_amd.cli")
    work = tempfile.mkdtemp(prefix="acf_e2e_")
    os.makedirs(os.path.join(work, "data"))
    z = np.load(os.path.join(GOLDEN, "video_data.npz"))
    with open(os.path.join(work, "data", "Video.train.rating"), "w") as f:
        f.writelines(f"{u}\t{i}\t{r}\t1\n" for u, i, r in zip(z["train_u"], z["train_i"], z["train_r"]))
    with open(os.path.join(work, "data", "Video.test.rating"), "w") as f:
        f.writelines(f"{u}\t{i}\t1\t1\n" for u, i in zip(z["test_u"], z["test_i"]))
    if a.out:
        os.makedirs(a.out, exist_ok=True)
    os.chdir(work)
    argv = ["--path", work + "/", "--opath", "e2e/", "--dataset", "Video", "--model", a.model,
            "--epochs", str(a.epochs), "--adv_epoch", str(a.adv_epoch), "--verbose", str(a.verbose),
            "--eval_mode", "all", "--embed_size", "64", "--ckpt", "0", "--seed", str(a.seed)]
    try:
        rc = cli.main(argv, "ori")
    finally:
        os.chdir(cwd)
    outs = sorted(os.listdir(os.path.join(work, "out", "e2e")))
    log = [f for f in outs if f.endswith(".out")][0]
    text = open(os.path.join(work, "out", "e2e", log)).read()
    if a.out:
        with open(os.path.join(a.out, log), "w") as f:
            f.write(text)
    best = re.search(r"Epoch (\d+) is the best epoch", text)
    k10 = re.search(r"K = 10: HR = ([\d.]+), NDCG = ([\d.]+) AUC = ([\d.]+)", text)
    runs = json.load(open(os.path.join(GOLDEN, "published_logs.json")))
    ref = runs["Video_apr_d64_e0.500000_l1.000000_2020_01_24_12_07_42.out" if a.model == "apr"
               else "Video_bpr_d64_2020_01_24_13_48_02.out"]
    summary = {"rc": rc, "log": log, "best_epoch": int(best.group(1)) if best else None,
               "hr10": float(k10.group(1)) if k10 else None, "ndcg10": float(k10.group(2)) if k10 else None,
               "ref_best_epoch": ref["best_epoch"], "ref_hr10": ref["best"][9][1], "ref_ndcg10": ref["best"][9][2]}
    if k10:
        summary["hr10_diff"] = round(summary["hr10"] - summary["ref_hr10"], 4)
        summary["ndcg10_diff"] = round(summary["ndcg10"] - summary["ref_ndcg10"], 4)
    if a.out:
        with open(os.path.join(a.out, "summary_%s.json" % a.model), "w") as f:
            json.dump(summary, f, indent=1)
    return summary, text


if __name__ == "__main__":
    main()
