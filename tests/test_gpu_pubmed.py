"""BASELINE.json configs[1] at its stated size: the reference's training-loop
body (utils.py:144-191) on the Pubmed citation graph with b_sz = 512 —
extend_nodes(num_neg = 100, models.py:135-186) on 512 roots, GraphSage
(fanouts 10, 10, MEAN) over the ≈ 9.7k-node extended batch, the supervised
NLL head, backward, clip_grad_norm_(5) per model and SGD(0.7) — through the
drop-in modules (utils.train_step, the path `bench.py --config pubmed` times),
against the oracle's restatement of the same step (unsup_semantics.
extend_nodes + train_step_dense) on the same graph, features and `random`
stream.

Checked per step: the extended node list (order included) bit-exact, the loss
within 1e-4; after both steps the `random` state bit-exact and every weight
within 1e-4 (the fp32 train-step tolerance used throughout).
"""
import importlib
import os
import random

import numpy as np
import pytest
import torch

import oracle
from oracle import unsup_semantics as U

pytestmark = pytest.mark.gpu

models = importlib.import_module("graphsage-pytorch_amd.models")
unsup = importlib.import_module("graphsage-pytorch_amd.unsup")
utils = importlib.import_module("graphsage-pytorch_amd.utils")
ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")
DEV = torch.device("cuda", 0)
G = os.path.join(os.path.dirname(__file__), "golden")
SEED, FEAT, H, C, B, FAN, STEPS = 824, 500, 128, 3, 512, [10, 10], 2


def test_pubmed_b512_apply_model_steps_vs_oracle(gs):
    g = np.load(os.path.join(G, "graphs.npz"))
    src, dst, n = g["pubmed_src"].astype(np.int64), g["pubmed_dst"].astype(np.int64), int(g["pubmed_n"][0])
    graph = gs.CSRGraph.from_pairs(src, dst, n)
    X = torch.empty(n, FEAT, dtype=torch.float32, device=DEV)
    ops.fill_uniform(X, SEED)
    np.random.seed(SEED)  # dataCenter.py:100-111's split after main.py:41's seed
    perm = np.random.permutation(n)
    train_ids = perm[n // 3 + n // 6:]
    labels = (np.arange(n) % C).astype(np.int64)
    order = np.random.RandomState(SEED + 1).permutation(train_ids)
    batches = [order[i * B:(i + 1) * B] for i in range(STEPS)]

    torch.manual_seed(SEED)
    gsage = models.GraphSage(2, FEAT, H, X, graph, DEV, agg_func="MEAN", fanouts=FAN).to(DEV)
    cls = models.Classification(H, C).to(DEV)
    init = [gsage.sage_layer1.weight, gsage.sage_layer2.weight, cls.layer[0].weight, cls.layer[0].bias]
    init = [p.detach().cpu().clone() for p in init]
    ul = unsup.UnsupervisedLoss(graph, train_ids, DEV)
    opt = torch.optim.SGD([p for m in (gsage, cls) for p in m.parameters()], lr=0.7)
    random.seed(SEED)
    losses, ext = [], []
    for b in batches:
        loss, nodes = utils.train_step(gsage, cls, ul, opt, b, labels, 100, "sup", None)
        losses.append(float(loss))
        ext.append(nodes.tolist())
    torch.cuda.synchronize()
    state = random.getstate()

    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    adj = oracle.Adjacency(src, dst, n)
    st = U.UnsupState(adj, train_ids)
    W = [p.clone().requires_grad_(True) for p in init]
    Xc = X.cpu()
    random.seed(SEED)
    for i, b in enumerate(batches):
        nodes, ok = U.extend_nodes(st, b, 100)
        assert ok
        assert nodes == ext[i], i  # extend_nodes: same nodes in the same (CPython set) order
        assert len(nodes) > 5000  # the ≈ 9.7k-node extended batch of the bench's step
        ref = oracle.train_step_dense(adj, nodes, FAN, Xc, W[:2], W[2], W[3], torch.from_numpy(labels[nodes]),
                                      agg="MEAN")
        assert abs(losses[i] - ref) < 1e-4, (i, losses[i], ref)
    assert random.getstate() == state
    got = [gsage.sage_layer1.weight, gsage.sage_layer2.weight, cls.layer[0].weight, cls.layer[0].bias]
    for a, w in zip(got, W):
        torch.testing.assert_close(a.detach().cpu(), w.detach(), atol=1e-4, rtol=1e-4)
