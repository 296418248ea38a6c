"""Parity at the headline workload's full size (BASELINE.json configs[2],
bench.py `rmat2m`): R-MAT scale 21 (2,097,152 ids), 20,000,000 pairs, 256-d
fp32 features, fanouts (25, 10), MEAN, B = 512 roots per step.

* the native runner (2 sampler streams, resolved-id gather, fused step) over
  3 steps against the oracle's training step on the same graph, batches and
  `random` streams: per-hop sampled sizes equal, loss per step and final
  weights within 1e-4 (the tolerance of the smaller-graph train-step test);
* determinism: a second runner over the same batches leaves bitwise the same
  parameters and losses;
* the forward-only inference runner (train.Embedder, get_gnn_embeddings'
  native path) equals the drop-in module's forward batch by batch.
"""
import importlib
import random

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

train = importlib.import_module("graphsage-pytorch_amd.train")
ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")
models = importlib.import_module("graphsage-pytorch_amd.models")
sampler = importlib.import_module("graphsage-pytorch_amd.sampler")
DEV = torch.device("cuda", 0)
SEED, F, H, C, B, FAN, S = 824, 256, 128, 16, 512, [25, 10], 2


@pytest.fixture(scope="module")
def wl(gs):
    src, dst = gs.rmat_pairs(21, 20_000_000, seed=SEED)
    n = 1 << 21
    graph = gs.CSRGraph.from_pairs(src, dst, n)
    X = torch.empty(n, F, dtype=torch.float32, device=DEV)
    ops.fill_uniform(X, SEED)
    labels = torch.from_numpy((np.arange(n) % C).astype(np.int32)).to(DEV)
    cands = np.nonzero(graph.degrees() > 0)[0]
    batches = list(train.rank_batches(cands, B, 0, 1, SEED + 1000))[:3]
    return dict(src=src, dst=dst, n=n, graph=graph, X=X, labels=labels, batches=batches)


def _run(wl):
    tr = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], C, fanouts=FAN, seed=SEED)
    r = train.Runner(tr, wl["graph"], wl["batches"], [train.make_rng(SEED, 0, w) for w in range(S)], FAN, depth=2)
    losses = []
    for _ in wl["batches"]:
        r.run(1)
        losses.append(float(tr.loss.item()))
    sizes = r.stats()["hop_sizes_sum"]
    r.close()
    return tr, losses, sizes


@pytest.fixture(scope="module")
def native(wl):
    return _run(wl)


def test_fullsize_runner_vs_oracle_train_steps(wl, native):
    tr, losses, sizes = native
    adj = oracle.Adjacency(wl["src"], wl["dst"], wl["n"])
    X = wl["X"].cpu()
    labels = wl["labels"].cpu().long()
    sage_w, cw, cb = train.reference_init(2, F, H, C, False, SEED)
    W = [w.clone().requires_grad_(True) for w in sage_w]
    cw, cb = cw.clone().requires_grad_(True), cb.clone().requires_grad_(True)
    rngs = [random.Random(train.rank_seed(SEED, 0, w)) for w in range(S)]
    n_dst = np.zeros(2)
    for i, roots in enumerate(wl["batches"]):
        rng = rngs[i % S]
        probe = random.Random()
        probe.setstate(rng.getstate())
        hops = oracle.sample_layers(adj, roots.tolist(), FAN, probe)
        n_dst += [len(hops[0][0]), len(hops[1][0])]
        ref = oracle.train_step_dense(adj, roots.tolist(), FAN, X, W, cw, cb, labels[torch.from_numpy(roots)],
                                      rng=rng)
        assert rng.getstate() == probe.getstate()  # the step drew exactly the probed words
        assert abs(losses[i] - ref) < 1e-4, (i, losses[i], ref)
    np.testing.assert_array_equal(sizes[:2, 0], n_dst)  # hop frontiers: B roots, then |L1|
    sd = tr.p.state_dict()
    for i in (1, 2):
        torch.testing.assert_close(sd[f"sage_layer{i}.weight"].cpu(), W[i - 1].detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(sd["layer.0.weight"].cpu(), cw.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(sd["layer.0.bias"].cpu(), cb.detach(), atol=1e-4, rtol=1e-4)


def test_fullsize_runner_is_deterministic(wl, native):
    tr, losses, sizes = native
    tr2, losses2, sizes2 = _run(wl)
    assert torch.equal(tr.p.params, tr2.p.params)
    assert losses == losses2
    np.testing.assert_array_equal(sizes, sizes2)


@pytest.mark.parametrize("merge", [1, 4])
def test_fullsize_embedder_matches_module_forward(wl, merge):
    W = [w.to(DEV) for w in train.reference_init(2, F, H, C, False, SEED)[0]]
    nodes = np.arange(0, 6 * 500 + 123, dtype=np.int64) * 331 % wl["n"]  # 6 full batches + a partial one
    # 6 full batches: merged steps of 4 + 2 batches, then the partial one
    emb = train.Embedder(wl["graph"], wl["X"], W, FAN, merge=merge).embed(nodes, 500, [sampler.RNG(7)])
    gsage = models.GraphSage(2, F, H, wl["X"], wl["graph"], DEV, fanouts=FAN, rng=sampler.RNG(7)).to(DEV)
    with torch.no_grad():
        for i in (1, 2):
            getattr(gsage, f"sage_layer{i}").weight.copy_(W[i - 1])
        for lo in range(0, len(nodes), 500):
            ref = gsage(nodes[lo:lo + 500])
            torch.testing.assert_close(emb[lo:lo + len(ref)], ref, atol=1e-6, rtol=1e-6, equal_nan=True)
