"""Command-line drivers with the flag surface of ``run_adv_ori.py:17-64`` (the
script that produced the published logs) and ``run_adv.py:15-54`` (the one named
in the task), restricted to the models on the APR path (``bpr``, ``apr``).

    python run_adv_ori.py --dataset Video --model apr --epochs 2000 --adv_epoch 1000 \
        --verbose 20 --eval_mode all --embed_size 64
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from time import localtime, strftime

# (flag, type, default-for-run_adv_ori, default-for-run_adv, help)
_FLAGS = [
    ("--path", str, "", "", "Input data path."),
    ("--opath", str, "aaa/", "aaa/", "Output path."),
    ("--dataset", str, "fsq11-sort", "ml-1m", "Dataset file prefix under <path>data/, or "
                                              "ml-1m-synthetic / pinterest-20-synthetic."),
    ("--model", str, "pop", "apr", "bpr or apr."),
    ("--verbose", int, 1, 1, "Evaluate per X epochs."),
    ("--batch_size", int, 512, 512, "batch_size"),
    ("--epochs", int, 10, 2, "Number of epochs."),
    ("--adv_epoch", int, 0, 1, "Add APR in epoch X (0: pure APR; > epochs: pure BPR)."),
    ("--embed_size", int, 64, 64, "Embedding size."),
    ("--dns", int, 1, 1, "Number of negative samples per positive (dns)."),
    ("--reg", float, 0.0, 0.0, "Regularization for user and item embeddings."),
    ("--lr", float, 0.05, 0.05, "Learning rate."),
    ("--reg_adv", float, 1.0, 1.0, "Regularization for adversarial loss."),
    ("--restore", str, None, None, "Restore time_stamp for weights in Pretrain/."),
    ("--ckpt", int, 10, 1, "Save the model per X epochs."),
    ("--task", str, "", "", "Task name for launching experiments."),
    ("--adv", str, "grad", "grad", "Adversarial perturbation: grad or random."),
    ("--eps", float, 0.5, 0.5, "Epsilon for adversarial weights."),
]
_ORI_ONLY = [
    ("--eps_dense", float, 0.5, "Accepted for compatibility (SASRec only)."),
    ("--eps_conv", float, 0.5, "Accepted for compatibility (SASRec only)."),
    ("--eps_pos", float, 0.5, "Accepted for compatibility (SASRec only)."),
    ("--eval_mode", str, "sample", "Eval mode: sample or all."),
]


def parse_args(argv=None, flavor="ori"):
    p = argparse.ArgumentParser(description="Run AMF (MI355X APR path).")
    for flag, typ, d_ori, d_adv, hlp in _FLAGS:
        nargs = "?" if flag in ("--path", "--opath", "--dataset", "--task", "--adv") else None
        kw = dict(type=typ, default=d_ori if flavor == "ori" else d_adv, help=hlp)
        if nargs:
            kw["nargs"] = nargs
        p.add_argument(flag, **kw)
    if flavor == "ori":
        for flag, typ, d, hlp in _ORI_ONLY:
            p.add_argument(flag, type=typ, default=d, help=hlp)
    else:
        p.set_defaults(eval_mode="all")  # run_adv.py evaluates all items (evaluation_adv.py:440)
    # MI355X-build extras
    p.add_argument("--seed", type=int, default=0, help="Seed of init and device sampler.")
    p.add_argument("--sampler", choices=["device", "host"], default="device")
    p.add_argument("--no_graph", action="store_true", help="Launch eagerly instead of hipGraph replay.")
    return p.parse_args(argv)


def init_logging(args, time_stamp):
    """utils.py:270-277."""
    path = "Log/%s_%s/" % (strftime("%Y-%m-%d_%H", localtime()), args.task)
    os.makedirs(path, exist_ok=True)
    logging.basicConfig(filename=path + "%s_log_embed_size%d_%s" % (args.dataset, args.embed_size, time_stamp),
                        level=logging.INFO)
    logging.info(args)
    print(args)


def main(argv=None, flavor="ori"):
    from .data import get_dataset
    from .model import MF
    from .train import training, write2file

    time_stamp = strftime("%Y_%m_%d_%H_%M_%S", localtime())
    args = parse_args(argv, flavor)
    init_logging(args, time_stamp)
    dataset = get_dataset(args.dataset, args.path, seed=2019)
    out = args.path + "out/" + args.opath
    if args.model == "bpr":
        runName = "%s_%s_d%d_%s" % (args.dataset, args.model, args.embed_size, time_stamp)
        write2file(out, runName + ".out", runName)
        args.adver = 0
        m = MF(dataset.num_users, dataset.num_items, args).build_graph()
        write2file(out, runName + ".out", "Initialize MF_BPR")
        training(m, dataset, args, runName, epoch_start=0, epoch_end=args.epochs, time_stamp=time_stamp)
    elif args.model == "apr":
        runName = "%s_%s_d%d_e%f_l%f_%s" % (args.dataset, args.model, args.embed_size, args.eps,
                                             args.reg_adv, time_stamp)
        write2file(out, runName + ".out", runName)
        args.adver = 0
        m = MF(dataset.num_users, dataset.num_items, args).build_graph()
        write2file(out, runName + ".out", "Initialize BPR")
        training(m, dataset, args, runName, epoch_start=0, epoch_end=args.adv_epoch - 1,
                 time_stamp=time_stamp)
        args.adver = 1
        amf = MF(dataset.num_users, dataset.num_items, args).build_graph(device=m.device)
        write2file(out, runName + ".out", "Initialize APR")
        training(amf, dataset, args, runName, epoch_start=args.adv_epoch, epoch_end=args.epochs,
                 time_stamp=time_stamp)
    else:
        print("model %r is not on the APR path of this build (bpr, apr)" % args.model, file=sys.stderr)
        return 2
    return 0
