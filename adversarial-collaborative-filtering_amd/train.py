"""Epoch driver and logging: ``training``, ``training_batch``,
``training_loss_acc``, ``output_evaluate``, ``write2file``, ``prediction2file``
(``APR.py:206-292``, ``utils.py:18-32,81-175``).

Log lines, file names and checkpoint layout follow the reference so existing
tooling reading ``out/<opath>/<runName>.out|.hr|.ndcg`` keeps working.
Checkpoints are ``.npz`` files holding the tensors ``embedding_P`` /
``embedding_Q`` under the reference's ``Pretrain/<ds>/{MF_BPR,APR}/embed_<d>/<ts>/``
directories, with a TF-style ``checkpoint`` index file (TF checkpoint V2 cannot be
written without TensorFlow).
"""
from __future__ import annotations

import logging
import os
import re
from time import time

import numpy as np
import torch

from . import ops
from .evaluate import evaluate, init_eval_model
from .sampler import DeviceSampler, EpochTriplets, sampling, shuffle


def write2file(path, name, output):
    """utils.py:18-24."""
    print(output, flush=True)
    if not os.path.exists(path):
        os.makedirs(path)
    with open(path + name, "a") as f:
        f.write("%s\n" % output)


def prediction2file(path, name, pred):
    """utils.py:26-32."""
    if not os.path.exists(path):
        os.makedirs(path)
    with open(path + name, "w") as f:
        for item in pred:
            f.write("%f\n" % item)


# ---------------------------------------------------------------------------
def _as_epoch(model, batches) -> EpochTriplets:
    if isinstance(batches, EpochTriplets):
        return batches
    user_input, item_input_pos, _user_dns, item_dns = batches
    B = int(np.asarray(user_input[0]).shape[0])
    dev = model.device
    u = torch.as_tensor(np.concatenate([np.asarray(x).reshape(-1) for x in user_input]),
                        dtype=torch.int32).to(dev)
    i = torch.as_tensor(np.concatenate([np.asarray(x).reshape(-1) for x in item_input_pos]),
                        dtype=torch.int32).to(dev)
    j = torch.as_tensor(np.concatenate([np.asarray(x).reshape(-1) for x in item_dns]),
                        dtype=torch.int32).to(dev)
    return EpochTriplets(u, i, j, B)


def training_batch(model, sess, batches, adver=False, graph=True):
    """utils.py:106-140.  dns == 1: the epoch is planned in chunks (plan_chunk),
    each trained by the streamed step (APR) or replayed as one hipGraph
    (delta_update + optimizer_step per batch, in batch order).  The step error
    word is read once per epoch: a step that gave up waiting for a row version
    raises StepWaitError instead of leaving silently stale rows.
    dns > 1: per batch, the highest-scoring of dns negatives under the current
    weights, then the optimizer step (the reference never runs update_P/update_Q
    on this branch, so the adversarial terms see delta = 0)."""
    if model.dns == 1:
        ep = _as_epoch(model, batches)
        B, nb = ep.batch_size, ep.n_batches
        hp = model.hparams(adver=int(bool(adver)))
        pipe = model.pipeline(B, min(nb, plan_chunk(B)))
        pipe.run(model.launch_tables, hp, ep.user, ep.item_pos, ep.item_neg, graph=graph, check=True)
        errs = pipe.step_errors()  # one stream sync per epoch
        if errs:
            raise ops.StepWaitError(errs)
        return ep
    user_input, item_input_pos, user_dns_list, item_dns_list = batches
    hp = model.hparams(adver=int(bool(adver)))
    hp.zero_delta = 1
    negs = []
    for k in range(len(user_input)):
        u = ops._idx(user_dns_list[k], "user", model.device)
        cand = ops._idx(item_dns_list[k], "cand", model.device)
        uu = ops._idx(user_input[k], "user", model.device)
        sel = ops.dns_select(model.embedding_P, model.embedding_Q, u[::model.dns].contiguous(), cand,
                             model.dns)
        ctx = model.context(uu.numel(), 1)
        ctx.plan(uu, item_input_pos[k], sel, uu.numel())
        if hp.adver:
            ctx.delta_update(model.launch_tables, hp, 0)
        ctx.optimizer_step(model.launch_tables, hp, 0)
        negs.append(sel.cpu().numpy().reshape(-1, 1))
    return user_input, item_input_pos, negs


def plan_chunk(batch_size: int) -> int:
    """Batches per plan / hipGraph; the next chunk is planned during this one.
    Small batches: 512 (the chunk's inline records stay in the Infinity Cache);
    large batches: 2M triplets (the plan's fixed sort cost amortised)."""
    return 512 if batch_size < 4096 else max(1, (1 << 21) // batch_size)


def training_loss_acc(model, sess, train_batches, output_adv=0):
    """utils.py:159-175: mean per-batch summed clean loss and mean pairwise accuracy."""
    if output_adv:
        raise NotImplementedError("output_adv=1 is not used by the APR driver (APR.py:258,266)")
    if isinstance(train_batches, EpochTriplets):
        u, i, j, B = train_batches.user, train_batches.item_pos, train_batches.item_neg, train_batches.batch_size
    else:
        ep = _as_epoch(model, (train_batches[0], train_batches[1], None, train_batches[2]))
        u, i, j, B = ep.user, ep.item_pos, ep.item_neg, ep.batch_size
    nb = u.numel() // B
    if nb == 0:
        return 0.0, 0.0
    bl, bc, _, _ = ops.bpr_forward(model.embedding_P, model.embedding_Q, u, i, j, B)
    bl = bl.double().cpu().numpy()
    bc = bc.cpu().numpy().astype(np.float64)
    return float(bl.sum() / nb), float((bc / B).sum() / nb)


def output_evaluate(model, sess, dataset, train_batches, eval_feed_dicts, epoch_count, batch_time,
                    train_time, prev_acc, runName, args, output_adv=0):
    """utils.py:81-101."""
    loss_begin = time()
    train_loss, post_acc = training_loss_acc(model, sess, train_batches, output_adv)
    _ = time() - loss_begin
    eval_begin = time()
    result, raw_result = evaluate(model, sess, dataset, eval_feed_dicts, output_adv, args)
    eval_time = time() - eval_begin
    nP = float(torch.linalg.vector_norm(model.embedding_P.double()))
    nQ = float(torch.linalg.vector_norm(model.embedding_Q.double()))
    hr, ndcg, auc = np.swapaxes(result, 0, 1)[-1]
    res = ("Epoch %d [%.1fs + %.1fs]: HR = %.4f, NDCG = %.4f ACC = %.4f ACC_adv = %.4f [%.1fs], "
           "|P|=%.2f, |Q|=%.2f" % (epoch_count, batch_time, train_time, hr, ndcg, prev_acc, post_acc,
                                   eval_time, nP, nQ))
    write2file(args.path + "out/" + args.opath, runName + ".out", res)
    return post_acc, ndcg, result, raw_result


# ---------------------------------------------------------------------------
# checkpoints (APR.py:209-232, 289-292)
def ckpt_dirs(args, time_stamp):
    if args.adver:
        save = "Pretrain/%s/APR/embed_%d/%s/" % (args.dataset, args.embed_size, time_stamp)
        restore = "Pretrain/%s/MF_BPR/embed_%d/%s/" % (args.dataset, args.embed_size, time_stamp)
    else:
        save = "Pretrain/%s/MF_BPR/embed_%d/%s/" % (args.dataset, args.embed_size, time_stamp)
        restore = 0 if args.restore is None else "Pretrain/%s/MF_BPR/embed_%d/%s/" % (
            args.dataset, args.embed_size, args.restore)
    return save, restore


def save_checkpoint(model, directory, step):
    os.makedirs(directory, exist_ok=True)
    ops.settle_tables()
    name = "weights-%d" % step
    np.savez(os.path.join(directory, name + ".npz"),
             embedding_P=model.embedding_P.cpu().numpy(), embedding_Q=model.embedding_Q.cpu().numpy())
    with open(os.path.join(directory, "checkpoint"), "w") as f:
        f.write('model_checkpoint_path: "%s"\nall_model_checkpoint_paths: "%s"\n' % (name, name))
    return os.path.join(directory, name)


def latest_checkpoint(directory):
    idx = os.path.join(directory, "checkpoint")
    if not os.path.exists(idx):
        return None
    with open(idx) as f:
        m = re.search(r'model_checkpoint_path:\s*"([^"]+)"', f.read())
    if not m:
        return None
    path = os.path.join(directory, m.group(1))
    return path if os.path.exists(path + ".npz") else None


def restore_checkpoint(model, path):
    with np.load(path + ".npz", allow_pickle=False) as z:
        P, Q = z["embedding_P"], z["embedding_Q"]
    if P.shape != tuple(model.embedding_P.shape) or Q.shape != tuple(model.embedding_Q.shape):
        raise ValueError(f"checkpoint shapes {P.shape}/{Q.shape} do not match the model")
    model.load_embeddings(P, Q)


# ---------------------------------------------------------------------------
def training(model, dataset, args, runName, epoch_start, epoch_end, time_stamp, sampler=None):
    """APR.py:206-292 on the GPU path.  Differences kept deliberately small: the
    triplet stream comes from the device sampler (seeded; the reference's forked
    sampler is not reproducible), and an epoch that is not evaluated does not
    reuse a stale NDCG (the reference raises NameError there)."""
    from .model import Session
    if not model.built:
        model.build_graph()
    sess = Session(model)
    ckpt_save_path, ckpt_restore_path = ckpt_dirs(args, time_stamp)
    os.makedirs(ckpt_save_path, exist_ok=True)
    if ckpt_restore_path:
        os.makedirs(ckpt_restore_path, exist_ok=True)
    if args.restore is not None or epoch_start:
        ck = latest_checkpoint(ckpt_restore_path) if ckpt_restore_path else None
        if ck:
            restore_checkpoint(model, ck)
            print("restored")
    else:
        logging.info("Initialized from scratch")
    eval_feed_dicts = init_eval_model(dataset, args)
    use_host = getattr(args, "sampler", "device") == "host"
    samples = sampling(dataset) if use_host else None
    if sampler is None and not use_host:
        sampler = DeviceSampler(dataset, args.batch_size, model.device, seed=getattr(args, "seed", 0) or 0)
    graph = not getattr(args, "no_graph", False)
    max_ndcg = 0
    best_res = {}
    epoch_count = epoch_start
    for epoch_count in range(epoch_start, epoch_end + 1):
        batch_begin = time()
        if use_host:
            batches = _as_epoch(model, shuffle(samples, args.batch_size, dataset, model))
        else:
            batches = sampler.epoch(epoch_count)
        torch.cuda.synchronize(model.device)
        batch_time = time() - batch_begin
        _, prev_acc = training_loss_acc(model, sess, batches, output_adv=0)
        train_begin = time()
        train_batches = training_batch(model, sess, batches, args.adver, graph=graph)
        torch.cuda.synchronize(model.device)
        train_time = time() - train_begin
        if epoch_count % args.verbose == 0:
            _, ndcg, cur_res, raw_result = output_evaluate(
                model, sess, dataset, train_batches, eval_feed_dicts, epoch_count, batch_time,
                train_time, prev_acc, runName, args, output_adv=0)
            if max_ndcg < ndcg:
                max_ndcg = ndcg
                best_res["result"] = cur_res
                best_res["epoch"] = epoch_count
                prediction2file(args.path + "out/" + args.opath, runName + ".hr", raw_result[:, 0, -1])
                prediction2file(args.path + "out/" + args.opath, runName + ".ndcg", raw_result[:, 1, -1])
        if model.epochs == epoch_count and best_res:
            write2file(args.path + "out/" + args.opath, runName + ".out",
                       "Epoch %d is the best epoch" % best_res["epoch"])
            for idx, (hr_k, ndcg_k, auc_k) in enumerate(np.swapaxes(best_res["result"], 0, 1)):
                write2file(args.path + "out/" + args.opath, runName + ".out",
                           "K = %d: HR = %.4f, NDCG = %.4f AUC = %.4f" % (idx + 1, hr_k, ndcg_k, auc_k))
        if args.ckpt > 0 and epoch_count % args.ckpt == 0:
            save_checkpoint(model, ckpt_save_path, epoch_count)
    save_checkpoint(model, ckpt_save_path, epoch_count)
    return best_res
