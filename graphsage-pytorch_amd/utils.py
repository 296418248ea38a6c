"""Drop-in batch loop and embedding export of the reference's src/utils.py.

``apply_model``      utils.py:113-193 — one epoch: shuffle, per batch
                     extend_nodes (native, bit-exact), GraphSage forward/backward
                     (HIP), supervised head + NLL (fused HIP kernel), the
                     unsupervised losses (HIP), clip_grad_norm_(5) per model,
                     SGD(lr=0.7).
``get_gnn_embeddings`` utils.py:59-78 — every node's embedding in batches of
                     500 (the full-graph inference pass); with
                     sampler streams or several ranks, the native forward-only
                     pipeline sharded over ranks + one all-gather.
``evaluate``         utils.py:13-57 — validation / test micro-F1, checkpoint.
``train_classification`` utils.py:80-111 — classifier on frozen embeddings.

Same signatures, same randomness consumers in the same order: numpy's global
stream (sklearn ``shuffle``), Python's ``random`` (extend_nodes, then the
GraphSage sampler), so an epoch visits the reference's batches and samples.
"""
import math
import os
import random as _pyrandom
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import hip_ops as ops

_NUM_NEG = {"margin": 6, "normal": 100}  # utils.py:119-122


class _SupervisedNLL(torch.autograd.Function):
    """-Σ log_softmax(E·Wᵀ + b)[i, y_i] / B (models.py:25-27, utils.py:159-164)
    in one fused HIP launch pair that also yields the gradients; backward only
    scales them by the incoming gradient."""

    @staticmethod
    def forward(ctx, E, W, b, labels):
        E_ = E.detach().contiguous()
        B, D = E_.shape
        C = W.shape[0]
        dev = E_.device
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        dE = torch.empty_like(E_)
        dW = torch.empty(C, D, dtype=torch.float32, device=dev)
        db = torch.empty(C, dtype=torch.float32, device=dev)
        ws = ops.cls_nll_workspace(B, D, C, dev)
        ops.cls_nll_fwd_bwd(E_, W.detach().contiguous(), b.detach().contiguous(), labels, loss, dE, dW, db, ws)
        ctx.save_for_backward(dE, dW, db)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        dE, dW, db = ctx.saved_tensors
        return dE * g, dW * g, db * g, None


def supervised_loss(classification, embs, labels_batch):
    """The loss_sup of utils.py:159-164 through the fused head."""
    lin = classification.layer[0]
    y = torch.as_tensor(np.asarray(labels_batch), device=embs.device).to(torch.int32)
    return _SupervisedNLL.apply(embs, lin.weight, lin.bias, y)


def _trainable(models):
    return [p for m in models for p in m.parameters() if p.requires_grad]


def train_step(graphSage, classification, unsupervised_loss, optimizer, batch, labels, num_neg, learn_method,
               unsup):
    """The body of one apply_model batch (utils.py:146-191): extend, forward,
    losses, backward, clip per model, SGD.  Returns (loss, extended nodes);
    the loss stays on the device (no host sync)."""
    ext = getattr(unsupervised_loss, "extend_nodes_array", None)  # ours: the ids as an array
    nodes = (ext(batch, num_neg=num_neg) if ext is not None
             else np.asarray(list(unsupervised_loss.extend_nodes(batch, num_neg=num_neg))))
    embs = graphSage(nodes)
    parts = []
    if learn_method in ("sup", "plus_unsup"):
        parts.append(supervised_loss(classification, embs, labels[nodes]))
    if learn_method != "sup":
        parts.append(unsup(embs, nodes))
    loss = parts[0] if len(parts) == 1 else parts[0] + parts[1]
    loss.backward()
    models = [graphSage, classification]
    for m in models:
        nn.utils.clip_grad_norm_(m.parameters(), 5)
    optimizer.step()
    optimizer.zero_grad()
    for m in models:
        m.zero_grad()
    return loss.detach(), nodes


def apply_model(dataCenter, ds, graphSage, classification, unsupervised_loss, b_sz, unsup_loss, device,
                learn_method, verbose=True):
    """One training epoch, utils.py:113-193.  Returns (graphSage, classification)."""
    if unsup_loss not in _NUM_NEG:
        print("unsup_loss can be only 'margin' or 'normal'.")
        sys.exit(1)
    num_neg = _NUM_NEG[unsup_loss]
    train_nodes = getattr(dataCenter, ds + "_train")
    labels = getattr(dataCenter, ds + "_labels")
    from sklearn.utils import shuffle  # numpy's global stream, as the reference
    train_nodes = shuffle(train_nodes)

    models = [graphSage, classification]
    optimizer = torch.optim.SGD(_trainable(models), lr=0.7)
    optimizer.zero_grad()
    for m in models:
        m.zero_grad()
    unsup = {"margin": unsupervised_loss.get_loss_margin, "normal": unsupervised_loss.get_loss_sage}[unsup_loss]

    n_batches = math.ceil(len(train_nodes) / b_sz)
    seen = set()
    for index in range(n_batches):
        batch = train_nodes[index * b_sz:(index + 1) * b_sz]
        loss, nodes = train_step(graphSage, classification, unsupervised_loss, optimizer, batch, labels, num_neg,
                                 learn_method, unsup)
        seen.update(nodes.tolist())
        if verbose:
            print(f"Step [{index + 1}/{n_batches}], Loss: {loss.item():.4f}, "
                  f"Dealed Nodes [{len(seen)}/{len(train_nodes)}] ")
    return graphSage, classification


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_ids(n, b_sz, rank, world):
    """Ids of the batches this rank embeds: the reference's batches of b_sz in
    id order (utils.py:63-68), batch i on rank i % world, concatenated."""
    n_batches = math.ceil(n / b_sz)
    parts = [np.arange(i * b_sz, min(n, (i + 1) * b_sz), dtype=np.int64) for i in range(rank, n_batches, world)]
    return np.concatenate(parts) if parts else np.zeros(0, np.int64)


def _embed_ids(gnn_model, ids, b_sz, rngs):
    """This rank's embeddings through the native inference pipeline."""
    from .train import Embedder
    weights = [getattr(gnn_model, f"sage_layer{i}").weight for i in range(1, gnn_model.num_layers + 1)]
    X = gnn_model.raw_features
    X = X if X.is_contiguous() else X.contiguous()
    emb = Embedder(gnn_model.graph, X, weights, gnn_model.fanouts, gnn_model.agg_func, gnn_model.gcn)
    return emb.embed(ids, b_sz, rngs)


def get_gnn_embeddings(gnn_model, dataCenter, ds, b_sz=500, *, sampler_streams=None, group=None, seed=None):
    """Embeddings of every node, utils.py:59-78 (batches of 500, in id order).

    Default (one process, no `sampler_streams`): the reference's loop — one
    GraphSage call per batch on the global `random` stream, bit-exact.

    Native pipeline (`sampler_streams` = S, or torch.distributed initialised
    with world W > 1): batch i goes to rank i % W; each rank
    runs its batches through the forward-only runner (train.Embedder) with S
    sampler streams, then one all-gather assembles [N, H] on every rank.  At
    W = 1, S = 1 the stream is the global `random` state (same result and
    same state afterwards as the default loop), or the module's own `rng`
    when it was given one; otherwise stream (r, w) is
    seeded train.rank_seed(seed, r, w) (seed defaults to 824), each one a
    reference stream on its own."""
    n = len(getattr(dataCenter, ds + "_labels"))
    rank, world = _world(group)
    if world == 1 and not sampler_streams:
        out = []
        with torch.no_grad():
            for lo in range(0, n, b_sz):
                ids = np.arange(lo, min(n, lo + b_sz), dtype=np.int64)
                e = gnn_model(ids)
                assert len(e) == len(ids)
                out.append(e)
        embs = torch.cat(out, 0)
        assert len(embs) == n
        return embs.detach()

    from .sampler import RNG
    from .train import rank_seed
    S = int(sampler_streams or 1)
    ids = shard_ids(n, b_sz, rank, world)
    own = getattr(gnn_model, "rng", None)
    exact = world == 1 and S == 1 and own is None
    if exact:
        rngs = [RNG.from_python(_pyrandom)]
    elif world == 1 and S == 1:  # the module's own stream, as its forward would draw
        rngs = [own]
    else:
        base = 824 if seed is None else int(seed)
        rngs = [RNG(rank_seed(base, rank, w)) for w in range(S)]
    mine = _embed_ids(gnn_model, ids, b_sz, rngs)
    if exact:
        rngs[0].to_python(_pyrandom)
    if world == 1:
        return mine.detach()
    # all-gather: every rank knows every shard's ids, so pad to the largest
    H = mine.shape[1]
    lens = [len(shard_ids(n, b_sz, r, world)) for r in range(world)]
    buf = torch.zeros(max(lens), H, dtype=mine.dtype, device=mine.device)
    buf[:len(ids)].copy_(mine)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    embs = torch.empty(n, H, dtype=mine.dtype, device=mine.device)
    for r in range(world):
        rid = torch.from_numpy(shard_ids(n, b_sz, r, world)).to(mine.device)
        embs.index_copy_(0, rid, parts[r][:lens[r]])
    return embs.detach()


def evaluate(dataCenter, ds, graphSage, classification, device, max_vali_f1, name, cur_epoch):
    """Validation micro-F1, and test F1 + checkpoint when it improves
    (utils.py:13-57).  Same RNG use (GraphSage on the val nodes, then on the
    test nodes only when improved), same prints, same return value.  The
    checkpoint is torch.save([graphSage, classification]) as in the
    reference (GraphSage pickles without its native graph handle)."""
    from sklearn.metrics import f1_score
    test_nodes = getattr(dataCenter, ds + "_test")
    val_nodes = getattr(dataCenter, ds + "_val")
    labels = getattr(dataCenter, ds + "_labels")
    models = [graphSage, classification]
    params = []
    for model in models:
        for param in model.parameters():
            if param.requires_grad:
                param.requires_grad = False
                params.append(param)

    def predict(nodes):
        embs = graphSage(nodes)
        _, predicts = torch.max(classification(embs), 1)
        return predicts.cpu().numpy()

    predicts = predict(val_nodes)
    labels_val = labels[val_nodes]
    assert len(labels_val) == len(predicts)
    vali_f1 = f1_score(labels_val, predicts, average="micro")
    print("Validation F1:", vali_f1)
    if vali_f1 > max_vali_f1:
        max_vali_f1 = vali_f1
        predicts = predict(test_nodes)
        labels_test = labels[test_nodes]
        assert len(labels_test) == len(predicts)
        test_f1 = f1_score(labels_test, predicts, average="micro")
        print("Test F1:", test_f1)
        for param in params:
            param.requires_grad = True
        os.makedirs("models", exist_ok=True)
        torch.save(models, "models/model_best_{}_ep{}_{:.4f}.torch".format(name, cur_epoch, test_f1))
    for param in params:
        param.requires_grad = True
    return max_vali_f1


def train_classification(dataCenter, graphSage, classification, ds, device, max_vali_f1, name, epochs=800):
    """Classifier on frozen embeddings (utils.py:80-111): get_gnn_embeddings,
    then per epoch sklearn-shuffled batches of 50, -Σ logp[label] / n through
    the fused HIP head, clip_grad_norm_(5), SGD(lr=0.5), evaluate()."""
    from sklearn.utils import shuffle
    print("Training Classification ...")
    c_optimizer = torch.optim.SGD(classification.parameters(), lr=0.5)
    b_sz = 50
    train_nodes = getattr(dataCenter, ds + "_train")
    labels = getattr(dataCenter, ds + "_labels")
    features = get_gnn_embeddings(graphSage, dataCenter, ds)
    for epoch in range(epochs):
        train_nodes = shuffle(train_nodes)
        batches = math.ceil(len(train_nodes) / b_sz)
        for index in range(batches):
            nodes_batch = train_nodes[index * b_sz:(index + 1) * b_sz]
            loss = supervised_loss(classification, features[torch.as_tensor(nodes_batch, device=features.device)],
                                   labels[nodes_batch])
            loss.backward()
            nn.utils.clip_grad_norm_(classification.parameters(), 5)
            c_optimizer.step()
            c_optimizer.zero_grad()
        max_vali_f1 = evaluate(dataCenter, ds, graphSage, classification, device, max_vali_f1, name, epoch)
    return classification, max_vali_f1
