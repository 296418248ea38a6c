"""The product's data-parallel arithmetic on one GPU.

W ranks of the multi-GPU runner each compute the step's gradients on their
own disjoint root batch (train.rank_batches) with their own sampler stream
(train.rank_seed), RCCL sums the flat gradient buffers, and every rank runs
gs_trainer_update(grad_scale = 1/W): scale, clip per model, SGD.  Here one
process plays both ranks of W = 2 through the product's kernels —
NativeTrainer.forward_backward per rank, the sum the all-reduce produces, then
the native update — and the result is compared with the oracle's
single-process restatement (the reference's step on the averaged gradient,
as tests/test_dp_gloo.py runs it on CPU) at 1e-6.

Also on one GPU: the runner's bucketed all-reduce (ar_buckets = 2: upper
gradients on a comm stream under the layer-1 dW GEMM) leaves bitwise the
parameters of the single all-reduce, and a held runner (the bench's
measurement mode) samples nothing before release and equals an unheld one.
"""
import importlib
import os
import random
import time

import numpy as np
import pytest
import torch

import oracle
from tests.golden.synth import uniform_features

pytestmark = pytest.mark.gpu

train = importlib.import_module("graphsage-pytorch_amd.train")
models = importlib.import_module("graphsage-pytorch_amd.models")
DEV = torch.device("cuda", 0)
G = os.path.join(os.path.dirname(__file__), "golden")
F, H, C, B, STEPS, SEED, FAN, W = 32, 128, 5, 16, 3, 824, [5, 3], 2


def _setup(gs):
    g = np.load(os.path.join(G, "graphs.npz"))
    n = int(g["rmat_n"][0])
    graph = gs.CSRGraph.from_pairs(g["rmat_src"], g["rmat_dst"], n)
    adj = oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n)
    X = torch.from_numpy(uniform_features(3, n, F))
    labels = torch.from_numpy((np.arange(n) % C).astype(np.int32))
    cands = np.nonzero(graph.degrees() > 0)[0]
    return graph, adj, X, labels, cands


def _oracle_dp(adj, X, labels, per_rank, max_norm=5.0, sums=None, classes=C):
    """The reference's step per rank on its own batch and stream, the rank
    gradients summed (the all-reduce), then clip_grad_norm_(max_norm) per model
    and SGD on the sum / W (utils.py:184-187).  sums: the summed flat gradient
    [dW1 | dW2 | dWc | dbc] of each step is appended to it."""
    sage_w, cw, cb = train.reference_init(2, F, H, classes, False, SEED)
    params = [w.clone().requires_grad_(True) for w in sage_w] + [cw.clone().requires_grad_(True),
                                                                cb.clone().requires_grad_(True)]
    rngs = [random.Random(train.rank_seed(SEED, r)) for r in range(W)]
    for i in range(len(per_rank[0])):
        gsum = None
        for r in range(W):
            roots = per_rank[r][i]
            hops = oracle.sample_layers(adj, roots.tolist(), FAN, rngs[r])
            emb = oracle.forward_dense(hops, X, params[:2], "MEAN", False)
            logp = torch.log_softmax(emb.mm(params[2].t()) + params[3], 1)
            oracle.nll_loss(logp, labels.long()[torch.from_numpy(roots)]).backward()
            g = [p.grad.detach().clone() for p in params]
            for p in params:
                p.grad = None
            gsum = g if gsum is None else [a + b for a, b in zip(gsum, g)]
        if sums is not None:
            sums.append(torch.cat([x.reshape(-1) for x in gsum]))
        with torch.no_grad():  # utils.py:185-187 on the averaged gradient
            scaled = [x / W for x in gsum]
            for group in ((0, 1), (2, 3)):
                norm = torch.norm(torch.stack([torch.norm(scaled[j]) for j in group]))
                coef = min(1.0, max_norm / (float(norm) + 1e-6))
                for j in group:
                    scaled[j] = scaled[j] * coef
            for p, x in zip(params, scaled):
                p.add_(x, alpha=-0.7)
    return [p.detach() for p in params]


def test_two_rank_step_arithmetic_on_one_gpu(gs):
    graph, adj, X, labels, cands = _setup(gs)
    per_rank = [list(train.rank_batches(cands, B, r, W, SEED + 1000))[:STEPS] for r in range(W)]
    assert not set(np.concatenate(per_rank[0]).tolist()) & set(np.concatenate(per_rank[1]).tolist())
    tr = train.NativeTrainer(graph, X.to(DEV), labels.to(DEV), C, hidden=H, fanouts=FAN, seed=SEED)
    rngs = [train.make_rng(SEED, r) for r in range(W)]
    for i in range(STEPS):
        gsum = torch.zeros_like(tr.p.grads)
        for r in range(W):  # rank r's forward/backward on its own batch and stream
            roots = per_rank[r][i]
            ds = models.DeviceSample(gs.sample(graph, rngs[r], roots, FAN), DEV)
            tr.forward_backward(ds, torch.from_numpy(roots.astype(np.int32)).to(DEV))
            gsum += tr.p.grads  # what the in-place RCCL sum leaves on every rank (W = 2: one add)
        tr.p.grads.copy_(gsum)
        tr.update(grad_scale=1.0 / W)
    torch.cuda.synchronize()
    ref = _oracle_dp(adj, X, labels, per_rank)
    sd = tr.p.state_dict()
    got = [sd["sage_layer1.weight"], sd["sage_layer2.weight"], sd["layer.0.weight"], sd["layer.0.bias"]]
    for a, b in zip(got, ref):
        torch.testing.assert_close(a.cpu(), b, atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize("max_norm", [5.0, 1e-3])
def test_two_rank_deferred_update_on_one_gpu(gs, max_norm):
    """The N > 1 runner's update path at W = 2: two trainers
    play ranks 0 and 1 in deferred-communicator mode (gs_trainer_defer, what
    gs_runner_run enters with a communicator).  Per step each rank runs its
    forward/backward on its own batch and stream; the two gradient buffers are
    summed in place into both trainers (what the in-place RCCL sum leaves on
    every rank); then each rank's gs_trainer_update(1/2) leaves the update
    pending (group_sumsq_spec_kernel: the summed gradient's clip-norm partials
    and W1's speculative update), and the next step's layer-1 forward applies
    it with FwdSpec::scale = 1/2 (the pending-update kernel instance, checked by
    name).  Four steps, so three forwards apply a pending update; max_norm 5
    (the reference's) and 1e-3 (every step clipped: the forward's recompute
    path).  Against the oracle's W = 2 step at 1e-5: each step's summed
    gradient and the final weights; the ranks' weights bitwise equal."""
    steps, classes = 4, 16  # 16 classes: the flat buffer's groups stay float4-aligned (deferral needs it)
    graph, adj, X, _, cands = _setup(gs)
    labels = torch.from_numpy((np.arange(X.shape[0]) % classes).astype(np.int32))
    per_rank = [list(train.rank_batches(cands, B, r, W, SEED + 1000))[:steps] for r in range(W)]
    trs = [train.NativeTrainer(graph, X.to(DEV), labels.to(DEV), classes, hidden=H, fanouts=FAN, seed=SEED,
                               max_norm=max_norm) for _ in range(W)]
    assert all(t.defer(True) for t in trs)
    rngs = [train.make_rng(SEED, r) for r in range(W)]
    lib = gs._lib.lib()
    sums = []
    for i in range(steps):
        if i == steps - 1:  # name the forward variant the last step launches (timer site 1)
            for t in trs:
                gs._lib.check(lib.gs_trainer_time_kernels(t._h, 0b10, 1))
        for r in range(W):  # rank r: its own batch, stream and trainer
            roots = per_rank[r][i]
            ds = models.DeviceSample(gs.sample(graph, rngs[r], roots, FAN), DEV)
            trs[r].forward_backward(ds, torch.from_numpy(roots.astype(np.int32)).to(DEV))
        gsum = trs[0].p.grads + trs[1].p.grads
        for t in trs:
            t.p.grads.copy_(gsum)
            t.update(grad_scale=1.0 / W)  # deferred: applied by the next forward
        sums.append(gsum.cpu())
    torch.cuda.synchronize()
    for t in trs:
        name = lib.gs_trainer_kernel_name(t._h, 1).decode()
        assert "linear_fwd_wide_kernel" in name and name.split(">(")[0].endswith("true"), name
    for t in trs:
        t.defer(False)  # the last pending update
    torch.cuda.synchronize()
    ref_sums = []
    ref = _oracle_dp(adj, X, labels, per_rank, max_norm=max_norm, sums=ref_sums, classes=classes)
    for i, (a, b) in enumerate(zip(sums, ref_sums)):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5, msg=lambda m: f"step {i} summed grads: {m}")
    assert torch.equal(trs[0].p.params, trs[1].p.params)
    sd = trs[0].p.state_dict()
    got = [sd["sage_layer1.weight"], sd["sage_layer2.weight"], sd["layer.0.weight"], sd["layer.0.bias"]]
    for a, b in zip(got, ref):
        torch.testing.assert_close(a.cpu(), b, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("agg,batch", [("MEAN", 48), ("MAX", 48), ("MEAN", 200)])
def test_bucketed_allreduce_equals_single(gs, agg, batch, monkeypatch):
    """ar_buckets = 2 (upper gradients all-reduced on a comm stream under the
    layer-1 dW GEMM, then W1 — in one piece, or in the row chunks the trainer
    hands over as its chunked dW1 completes them, GS_AR_W1_CHUNKS = 2, the
    default) against one all-reduce, one rank: bitwise.  Every batch gives the
    layer-1 gradient several row slabs (4-6 at these frontiers), so the
    chunks' slab sums are exercised."""
    graph, adj, X, labels, cands = _setup(gs)
    Xd = torch.from_numpy(uniform_features(5, X.shape[0], 256)).to(DEV)
    batches = list(train.rank_batches(cands, batch, 0, 1, 9))[:5]
    out = []
    comm = train.Communicator(0, 1, DEV)
    for buckets, chunks in ((1, "1"), (2, "1"), (2, "2")):
        monkeypatch.setenv("GS_AR_W1_CHUNKS", chunks)
        tr = train.NativeTrainer(graph, Xd, labels.to(DEV), 16, fanouts=(25, 10), agg_func=agg, seed=SEED)
        r = train.Runner(tr, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10],
                         fail_empty=agg == "MAX", depth=2, comm=comm, ar_buckets=buckets)
        r.run(len(batches))
        torch.cuda.synchronize()
        out.append((tr.p.params.clone(), float(tr.loss)))
        r.close()
    comm.close()
    for p, loss in out[1:]:
        assert torch.equal(out[0][0], p)
        assert out[0][1] == loss


def test_held_runner_samples_nothing_before_release(gs):
    graph, adj, X, labels, cands = _setup(gs)
    Xd = torch.from_numpy(uniform_features(5, X.shape[0], 256)).to(DEV)
    batches = list(train.rank_batches(cands, 48, 0, 1, 9))[:6]
    res = []
    for hold in (False, True):
        tr = train.NativeTrainer(graph, Xd, labels.to(DEV), 16, fanouts=(25, 10), seed=SEED)
        r = train.Runner(tr, graph, batches, [train.make_rng(11, 0, w) for w in range(3)], [25, 10], depth=2,
                         hold=hold)
        if hold:
            time.sleep(0.2)
            assert r.progress() == (0, 0)
            with pytest.raises(ValueError):
                r.run(1)  # past the release mark: refused instead of waiting forever
            r.release(2)
            r.run(2)
            torch.cuda.synchronize()
            time.sleep(0.1)
            sampled, consumed = r.progress()
            assert consumed == 2 and sampled == 2  # nothing past the mark
            r.release(len(batches))
            r.run(len(batches) - 2)
        else:
            r.run(len(batches))
        torch.cuda.synchronize()
        res.append(tr.p.params.clone())
        r.close()
    assert torch.equal(res[0], res[1])
