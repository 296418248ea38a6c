"""Data-parallel arithmetic of the training path on CPU (gloo, world size 2).

What the multi-GPU runner does per step: rank r trains on
batch i*W + r (train.rank_batches) with its own sampler stream
(train.rank_seed), sums the flat gradients over ranks, scales by 1/W, then
clips per model and applies SGD (gs_trainer_update(grad_scale=1/W)).  Here the
per-rank gradients come from the CPU oracle; the check is that two gloo ranks
end with exactly the weights of one process averaging both ranks' gradients.
"""
import importlib
import os
import random
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from tests.golden.synth import uniform_features

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
train = importlib.import_module("graphsage-pytorch_amd.train")

F, H, C, B, STEPS, SEED, FAN = 32, 16, 5, 16, 2, 824, [5, 3]


def _setup():
    g = np.load(os.path.join(G, "graphs.npz"))
    n = int(g["rmat_n"][0])
    adj = oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n)
    X = torch.from_numpy(uniform_features(3, n, F))
    labels = torch.from_numpy(np.arange(n) % C).long()
    deg = np.bincount(np.concatenate([g["rmat_src"], g["rmat_dst"]]), minlength=n)
    cands = np.nonzero(deg > 0)[0]
    return adj, X, labels, cands


def _params():
    sage_w, cw, cb = train.reference_init(2, F, H, C, False, SEED)
    return [w.clone().requires_grad_(True) for w in sage_w] + [cw.clone().requires_grad_(True),
                                                              cb.clone().requires_grad_(True)]


def _grads(adj, X, labels, params, roots, rng):
    hops = oracle.sample_layers(adj, roots.tolist(), FAN, rng)
    emb = oracle.forward_dense(hops, X, params[:2], "MEAN", False)
    logp = torch.log_softmax(emb.mm(params[2].t()) + params[3], 1)
    oracle.nll_loss(logp, labels[torch.from_numpy(roots)]).backward()
    gs = [p.grad.detach().clone() for p in params]
    for p in params:
        p.grad = None
    return gs


def _update(params, grads, world):
    with torch.no_grad():
        scaled = [g / world for g in grads]
        for group in ((0, 1), (2, 3)):
            norm = torch.norm(torch.stack([torch.norm(scaled[i]) for i in group]))
            coef = min(1.0, 5.0 / (float(norm) + 1e-6))
            for i in group:
                scaled[i] = scaled[i] * coef
        for p, g in zip(params, scaled):
            p.add_(g, alpha=-0.7)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    adj, X, labels, cands = _setup()
    params = _params()
    rng = random.Random(train.rank_seed(SEED, rank))
    batches = list(train.rank_batches(cands, B, rank, world, SEED + 1000))[:STEPS]
    for roots in batches:
        grads = _grads(adj, X, labels, params, roots, rng)
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)  # sum over ranks, as gs_comm_allreduce_sum
        out, at = [], 0
        for g in grads:
            out.append(flat[at:at + g.numel()].view_as(g))
            at += g.numel()
        _update(params, out, world)
    torch.save([p.detach() for p in params], os.path.join(out_dir, f"rank{rank}.pt"))
    np.save(os.path.join(out_dir, f"batches{rank}.npy"), np.stack(batches))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_data_parallel_step_equals_averaged_gradients():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        got = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
        seen = [np.load(os.path.join(d, f"batches{r}.npy")) for r in range(world)]
    # every rank holds identical weights
    for a, b in zip(got[0], got[1]):
        assert torch.equal(a, b)
    # disjoint root batches across ranks
    assert not set(seen[0].reshape(-1).tolist()) & set(seen[1].reshape(-1).tolist())
    # single-process reference: average the ranks' gradients, same streams
    adj, X, labels, cands = _setup()
    params = _params()
    rngs = [random.Random(train.rank_seed(SEED, r)) for r in range(world)]
    per_rank = [list(train.rank_batches(cands, B, r, world, SEED + 1000))[:STEPS] for r in range(world)]
    for i in range(STEPS):
        gsum = None
        for r in range(world):
            g = _grads(adj, X, labels, params, per_rank[r][i], rngs[r])
            gsum = g if gsum is None else [a + b for a, b in zip(gsum, g)]
        _update(params, gsum, world)
    for a, b in zip(got[0], params):
        torch.testing.assert_close(a, b.detach(), atol=1e-7, rtol=1e-6)
