"""Drop-in batch loop and embedding export of the reference's src/utils.py.

``apply_model``      utils.py:113-193 — one epoch: shuffle, per batch
                     extend_nodes (native, bit-exact), GraphSage forward/backward
                     (HIP), supervised head + NLL (fused HIP kernel), the
                     unsupervised losses (HIP), clip_grad_norm_(5) per model,
                     SGD(lr=0.7).
``get_gnn_embeddings`` utils.py:57-78 — every node's embedding in batches of
                     500 (the full-graph inference pass).

Same signatures, same randomness consumers in the same order: numpy's global
stream (sklearn ``shuffle``), Python's ``random`` (extend_nodes, then the
GraphSage sampler), so an epoch visits the reference's batches and samples.
"""
import math
import sys

import numpy as np
import torch
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
    nodes = np.asarray(list(unsupervised_loss.extend_nodes(batch, num_neg=num_neg)))
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


def get_gnn_embeddings(gnn_model, dataCenter, ds, b_sz=500):
    """Embeddings of every node, utils.py:57-78 (batches of 500, in id order)."""
    n = len(getattr(dataCenter, ds + "_labels"))
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
