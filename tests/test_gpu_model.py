"""Model-level parity on the MI355X: the drop-in GraphSage / SageLayer against
the reference's golden vectors (embeddings within 1e-5 fp32, weight gradients,
RNG stream position) and against the oracle on the benchmark's fanouts; the
native fused training step against the oracle's training step."""
import importlib
import os
import random

import numpy as np
import pytest
import torch

import oracle
from tests.golden.synth import hashed_binary_features, uniform_features

pytestmark = pytest.mark.gpu

models = importlib.import_module("graphsage-pytorch_amd.models")
train = importlib.import_module("graphsage-pytorch_amd.train")
DEV = torch.device("cuda", 0)
G = os.path.join(os.path.dirname(__file__), "golden")


def _graph(gs, name):
    g = np.load(os.path.join(G, "graphs.npz"))
    n = int(g[f"{name}_n"][0])
    return gs.CSRGraph.from_pairs(g[f"{name}_src"], g[f"{name}_dst"], n), g, n


def _features(name, n):
    if name == "cora":
        return hashed_binary_features(n, 1433)
    if name == "rmat":
        return uniform_features(77, n, 100)
    return uniform_features(11, n, 64)


FORWARDS = [("cora", "MEAN", "sage", 824), ("cora", "MAX", "sage", 824), ("cora", "MEAN", "gcn", 824),
            ("cora", "MAX", "gcn", 824), ("rmat", "MEAN", "sage", 5), ("rmat", "MAX", "sage", 5),
            ("pubmed", "MEAN", "sage", 824)]


@pytest.mark.parametrize("name,agg,mode,seed", FORWARDS)
@pytest.mark.parametrize("adj_kind", ["pairs", "adj_lists"])
def test_graphsage_matches_reference_vectors(gs, name, agg, mode, seed, adj_kind):
    R = np.load(os.path.join(G, f"forward_{name}_{agg}_{mode}.npz"))
    graph, g, n = _graph(gs, name)
    if adj_kind == "adj_lists":
        from collections import defaultdict
        adj = defaultdict(set)
        for a, b in zip(g[f"{name}_src"].tolist(), g[f"{name}_dst"].tolist()):
            adj[a].add(b)
            adj[b].add(a)
        graph = adj
    X = torch.from_numpy(_features(name, n)).to(DEV)
    torch.manual_seed(seed)  # the reference's init path reproduces the captured weights
    model = models.GraphSage(2, X.shape[1], 128, X, graph, DEV, gcn=(mode == "gcn"), agg_func=agg).to(DEV)
    for i in (1, 2):
        w = getattr(model, f"sage_layer{i}").weight
        assert torch.equal(w.detach().cpu(), torch.from_numpy(R[f"w__sage_layer{i}.weight"]))
    random.seed(seed)
    emb = model(R["roots"].tolist())
    assert list(random.getstate()[1]) == R["state"].tolist()  # same rng words consumed
    torch.testing.assert_close(emb.detach().cpu(), torch.from_numpy(R["emb"]), atol=1e-5, rtol=1e-5)
    (emb * torch.from_numpy(uniform_features(31, len(R["roots"]), 128)).to(DEV)).sum().backward()
    for i in (1, 2):
        torch.testing.assert_close(getattr(model, f"sage_layer{i}").weight.grad.cpu(),
                                   torch.from_numpy(R[f"grad__sage_layer{i}.weight"]), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
@pytest.mark.parametrize("fanouts", [[25, 10], [5, 3, 2]])
def test_graphsage_vs_oracle_bench_fanouts(gs, agg, fanouts):
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(3, n, 256))
    torch.manual_seed(1)
    model = models.GraphSage(len(fanouts), 256, 128, X.to(DEV), graph, DEV, agg_func=agg, fanouts=fanouts).to(DEV)
    roots = np.nonzero(graph.degrees())[0][::3][:100].tolist()
    random.seed(11)
    emb = model(roots)
    W = [getattr(model, f"sage_layer{i}").weight.detach().cpu().clone().requires_grad_(True)
         for i in range(1, len(fanouts) + 1)]
    random.seed(11)
    hops = oracle.sample_layers(oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n), roots, fanouts)
    ref = oracle.forward_dense(hops, X, W, agg, False)
    torch.testing.assert_close(emb.detach().cpu(), ref.detach(), atol=1e-5, rtol=1e-5)
    up = torch.from_numpy(uniform_features(9, len(roots), 128))
    (emb * up.to(DEV)).sum().backward()
    (ref * up).sum().backward()
    for i in range(1, len(fanouts) + 1):
        torch.testing.assert_close(getattr(model, f"sage_layer{i}").weight.grad.cpu(), W[i - 1].grad,
                                   atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("name,gcn,fanouts", [("pubmed", False, [10, 10]), ("cora", True, [10, 10]),
                                               ("rmat", False, [25, 10]), ("rmat", False, [5, 3, 2])])
def test_graphsage_sampler_helpers_bitwise(gs, name, gcn, fanouts):
    """sampler_helpers > 0 (the forward's sampling on a gs_team into a pinned
    pack): embeddings, weight gradients and the global `random` state after
    the forward are bitwise those of the team-less path, over two batches."""
    graph, g, n = _graph(gs, name)
    X = torch.from_numpy(_features(name, n)).to(DEV)
    out = []
    for helpers in (0, 3):
        torch.manual_seed(5)
        model = models.GraphSage(len(fanouts), X.shape[1], 128, X, graph, DEV, gcn=gcn, fanouts=fanouts,
                                 sampler_helpers=helpers).to(DEV)
        random.seed(21)
        embs, grads = [], []
        for b in range(2):
            roots = np.nonzero(graph.degrees())[0][b::5][:300].tolist()
            emb = model(roots)
            (emb * torch.from_numpy(uniform_features(8 + b, len(roots), 128)).to(DEV)).sum().backward()
            embs.append(emb.detach().cpu())
        grads = [getattr(model, f"sage_layer{i}").weight.grad.cpu() for i in range(1, len(fanouts) + 1)]
        out.append((embs, grads, random.getstate()))
    (e0, g0, s0), (e1, g1, s1) = out
    assert s0 == s1
    for a, b in zip(e0 + g0, e1 + g1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
def test_graphsage_duplicate_roots_vs_oracle(gs, agg):
    """Repeated ids in nodes_batch: every occurrence is sampled on its own
    (models.py:282) and gets its own output row (row i = nodes_batch[i])."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(4, n, 64))
    torch.manual_seed(2)
    model = models.GraphSage(2, 64, 128, X.to(DEV), graph, DEV, agg_func=agg, fanouts=[6, 4]).to(DEV)
    base = np.nonzero(graph.degrees())[0][::7][:30].tolist()
    roots = base + base[:9] + [base[2]] * 4
    random.seed(13)
    emb = model(roots)
    state = random.getstate()
    W = [getattr(model, f"sage_layer{i}").weight.detach().cpu().clone().requires_grad_(True) for i in (1, 2)]
    random.seed(13)
    hops = oracle.sample_layers(oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n), roots, [6, 4])
    assert random.getstate() == state
    ref = oracle.forward_dense(hops, X, W, agg, False)
    torch.testing.assert_close(emb.detach().cpu(), ref.detach(), atol=1e-5, rtol=1e-5)
    up = torch.from_numpy(uniform_features(6, len(roots), 128))
    (emb * up.to(DEV)).sum().backward()
    (ref * up).sum().backward()
    for i in (1, 2):
        torch.testing.assert_close(getattr(model, f"sage_layer{i}").weight.grad.cpu(), W[i - 1].grad,
                                   atol=1e-4, rtol=1e-4)


def test_graphsage_bf16_max_vs_oracle(gs):
    """configs[3] numerics: bf16 feature table, fp32 accumulate; oracle on the
    same bf16-rounded features, bf16-rounded W1 (tolerance stated: 2e-2)."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(3, n, 256)).to(torch.bfloat16)
    torch.manual_seed(1)
    model = models.GraphSage(2, 256, 128, X.to(DEV), graph, DEV, agg_func="MAX", fanouts=[25, 10]).to(DEV)
    roots = np.nonzero(graph.degrees())[0][:64].tolist()
    random.seed(2)
    emb = model(roots).detach().cpu()
    W = [getattr(model, "sage_layer1").weight.detach().cpu().to(torch.bfloat16).float(),
         getattr(model, "sage_layer2").weight.detach().cpu()]
    random.seed(2)
    hops = oracle.sample_layers(oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n), roots, [25, 10])
    ref = oracle.forward_dense(hops, X.float(), W, "MAX", False)
    torch.testing.assert_close(emb, ref, atol=2e-2, rtol=2e-2)


def test_sagelayer_api_and_aggregate_api(gs):
    graph, g, n = _graph(gs, "cora")
    X = torch.from_numpy(hashed_binary_features(n, 1433)).to(DEV)
    torch.manual_seed(824)
    model = models.GraphSage(2, 1433, 128, X, graph, DEV).to(DEV)
    nodes = list(range(0, 60, 3))
    random.seed(5)
    samp, d, uniq = model._get_unique_neighs_list(nodes)
    random.seed(5)
    ref = oracle.sample_hop(oracle.Adjacency(g["cora_src"], g["cora_dst"], n), nodes, 10)
    assert uniq == ref[2] and d == ref[1] and samp == ref[0]
    agg = model.aggregate(nodes, X, (uniq, samp, d))
    ref_s = [s - {nodes[i]} for i, s in enumerate(samp)]
    want = torch.stack([X[torch.tensor(sorted(s), device=DEV)].mean(0) for s in ref_s])
    torch.testing.assert_close(agg, want, atol=1e-6, rtol=1e-5)
    layer = model.sage_layer1
    sf = X[torch.tensor(nodes, device=DEV)].requires_grad_(True)
    af = agg.detach().requires_grad_(True)
    out = layer(sf, af)
    ref_out = torch.relu(layer.weight.mm(torch.cat([sf, af], 1).t())).t()
    torch.testing.assert_close(out, ref_out, atol=1e-5, rtol=1e-5)
    out.sum().backward()
    g1 = layer.weight.grad.clone()
    layer.weight.grad = None
    sf2, af2 = sf.detach().requires_grad_(True), af.detach().requires_grad_(True)
    torch.relu(layer.weight.mm(torch.cat([sf2, af2], 1).t())).t().sum().backward()
    torch.testing.assert_close(g1, layer.weight.grad, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(sf.grad, sf2.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(af.grad, af2.grad, atol=1e-5, rtol=1e-5)


def test_max_empty_neighbourhood_raises(gs):
    # node 0 only links to itself: after self removal MAX has nothing to reduce
    src = np.array([0, 1, 2, 3], np.int64)
    dst = np.array([0, 2, 3, 1], np.int64)
    graph = gs.CSRGraph.from_pairs(src, dst, 4)
    X = torch.randn(4, 16, device=DEV)
    model = models.GraphSage(1, 16, 16, X, graph, DEV, agg_func="MAX").to(DEV)
    with pytest.raises(IndexError):
        model([0, 1])
    mean = models.GraphSage(1, 16, 16, X, graph, DEV, agg_func="MEAN").to(DEV)
    out = mean([0, 1])
    assert torch.isnan(out[0]).all()  # relu(NaN) stays NaN, as torch's relu
    assert torch.isfinite(out[1]).all()


@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
def test_native_train_step_vs_oracle(gs, agg):
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256))
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32))
    tr = train.NativeTrainer(graph, X.to(DEV), labels.to(DEV), 16, fanouts=(25, 10), agg_func=agg, seed=824)
    sage_w, cw, cb = train.reference_init(2, 256, 128, 16, False, 824)
    W = [w.clone().requires_grad_(True) for w in sage_w]
    cw, cb = cw.clone().requires_grad_(True), cb.clone().requires_grad_(True)
    rng = gs.RNG(824)
    random.seed(824)
    adj = oracle.Adjacency(g["rmat_src"], g["rmat_dst"], n)
    for step, roots in enumerate(train.rank_batches(np.nonzero(graph.degrees())[0], 64, 0, 1, 7)):
        if step == 3:
            break
        s = gs.sample(graph, rng, roots, [25, 10])
        ds = models.DeviceSample(s, DEV)
        loss = tr.step(ds, torch.from_numpy(roots.astype(np.int32)).to(DEV))
        ref_loss = oracle.train_step_dense(adj, roots.tolist(), [25, 10], X, W, cw, cb,
                                           labels[torch.from_numpy(roots)].long(), agg=agg)
        assert abs(float(loss) - ref_loss) < 1e-4
    sd = tr.p.state_dict()
    for i in (1, 2):
        torch.testing.assert_close(sd[f"sage_layer{i}.weight"].cpu(), W[i - 1].detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(sd["layer.0.weight"].cpu(), cw.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(sd["layer.0.bias"].cpu(), cb.detach(), atol=1e-4, rtol=1e-4)


def test_prefetcher_matches_synchronous(gs):
    graph, g, n = _graph(gs, "rmat")
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 32, 0, 1, 3))[:6]
    pf = train.Prefetcher(graph, gs.RNG(3), batches, [25, 10], False, DEV)
    rng = gs.RNG(3)
    for roots in batches:
        ds, roots_dev, s = pf.next()
        s2 = gs.sample(graph, rng, roots, [25, 10])
        ds2 = models.DeviceSample(s2, DEV)
        for hop, names in ((1, ("nbr_ptr", "nbr", "self", "tptr", "tidx")), (2, ("pos_ptr", "pos", "dst_ids"))):
            for name in names:  # fields only: the pack's alignment padding is not initialised
                assert torch.equal(ds.field(hop, name), ds2.field(hop, name)), (hop, name)
        assert roots_dev.cpu().tolist() == roots.tolist()


def test_prefetcher_streams_each_bit_exact(gs):
    """S sampler streams: stream w serves batches w, w+S, ... and equals a
    synchronous sampler seeded rank_seed(seed, rank, w)."""
    graph, g, n = _graph(gs, "rmat")
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 32, 0, 1, 4))[:8]
    S = 3
    pf = train.Prefetcher(graph, None, batches, [25, 10], False, DEV,
                          rngs=[train.make_rng(5, 0, w) for w in range(S)])
    sync = [train.make_rng(5, 0, w) for w in range(S)]
    for i, roots in enumerate(batches):
        ds, roots_dev, info = pf.next()
        s2 = gs.sample(graph, sync[i % S], roots, [25, 10])
        ds2 = models.DeviceSample(s2, DEV)
        assert info.sizes(1) == s2.sizes(1) and info.sizes(2) == s2.sizes(2)
        for hop, names in ((1, ("nbr_ptr", "nbr", "self", "tptr", "tidx")), (2, ("pos_ptr", "pos", "dst_ids"))):
            for name in names:
                assert torch.equal(ds.field(hop, name), ds2.field(hop, name)), (i, hop, name)
        assert roots_dev.cpu().tolist() == roots.tolist()


@pytest.mark.parametrize("S,agg,gcn", [(1, "MEAN", False), (3, "MEAN", False), (1, "MAX", False),
                                       (3, "MAX", False), (3, "MEAN", True)])
def test_native_runner_matches_python_loop(gs, S, agg, gcn):
    """gs_runner (native sampler threads + pinned ring + side-stream pull,
    resolved-id layer-1 gather, fused step) leaves exactly the parameters of
    the Python loop over the same sampler streams, whose layer-1 gather is the
    expand-mode kernel (same accumulation order: bitwise equal)."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:7]
    a = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, gcn=gcn, seed=824)
    b = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, gcn=gcn, seed=824)
    pf = train.Prefetcher(graph, None, batches, [25, 10], gcn, DEV,
                          rngs=[train.make_rng(11, 0, w) for w in range(S)], fail_empty=agg == "MAX")
    for _ in batches:
        ds, roots_dev, _info = pf.next()
        a.step(ds, roots_dev)
    pf.close()
    runner = train.Runner(b, graph, batches, [train.make_rng(11, 0, w) for w in range(S)], [25, 10], gcn=gcn,
                          fail_empty=agg == "MAX", depth=2)
    runner.run(3)
    runner.run(len(batches) - 3)
    torch.cuda.synchronize()
    st = runner.stats()
    assert st["steps"] == len(batches)
    assert torch.equal(a.p.params, b.p.params)
    assert float(a.loss) == float(b.loss)
    with pytest.raises(IndexError):
        runner.run(1)  # past the last batch
    runner.close()


@pytest.mark.parametrize("max_norm", [5.0, 1e-3, 0.05])
@pytest.mark.parametrize("agg,dtype", [("MEAN", "f32"), ("MAX", "f32"), ("MAX", "bf16"), ("MEAN", "bf16")])
def test_runner_deferred_update_matches_python_loop(gs, agg, dtype, max_norm):
    """The runner's deferred update (each step's clip + SGD applied by the next
    step's launches: W1's update for clip coefficient 1 written by the slab
    sum and read by the next forward, recomputed there when the gradients
    were clipped; the other parameters updated in the forward's prologue; the
    last update at the end of each run call) leaves the parameters and the
    clipped gradients of the Python loop's separate update launches, bit for
    bit: the reference's max_norm (5.0: the first steps clip, the later ones
    do not), clipping at every step (1e-3), and a mix (0.05), over runs of
    1, 2 and 4 steps.  bf16 features: the forward's bf16 W1 comes from the
    slab sum / the recompute instead of a cast of the updated W1."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    if dtype == "bf16":
        X = X.to(torch.bfloat16)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:7]
    a = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, max_norm=max_norm, seed=824)
    b = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, max_norm=max_norm, seed=824)
    pf = train.Prefetcher(graph, None, batches, [25, 10], False, DEV,
                          rngs=[train.make_rng(11, 0, w) for w in range(2)], fail_empty=agg == "MAX")
    norms = []
    for _ in batches:
        ds, roots_dev, _info = pf.next()
        a.forward_backward(ds, roots_dev)
        g_off = a.p.group_off
        norms.append(float(torch.linalg.vector_norm(a.p.grads[int(g_off[0]):int(g_off[1])])))
        a.apply_update()
    pf.close()
    runner = train.Runner(b, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10],
                          fail_empty=agg == "MAX", depth=2)
    for k in (1, 2, 4):
        runner.run(k)
    torch.cuda.synchronize()
    assert torch.equal(a.p.params, b.p.params)
    assert torch.equal(a.p.grads, b.p.grads)
    assert float(a.loss) == float(b.loss)
    runner.close()
    if max_norm == 1e-3:  # every step took the recompute path
        assert all(x > max_norm for x in norms), norms


def test_runner_deferred_update_switch(gs):
    """defer_update off (a separate update launch per step) and the default
    deferred update leave the same parameters bit for bit."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:6]
    out = []
    for defer in (False, True):
        t = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), max_norm=0.05, seed=824)
        t.set_option("defer_update", defer)
        r = train.Runner(t, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10], depth=2)
        r.run(len(batches))
        torch.cuda.synchronize()
        out.append(t.p.params.clone())
        r.close()
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize("agg,bf16,gcn", [("MEAN", False, False), ("MAX", False, False), ("MEAN", True, False),
                                          ("MAX", True, False), ("MEAN", False, True)])
def test_self_rows_matches_default(gs, agg, bf16, gcn):
    """self_rows (default on: the side-stream gather also copies the layer-1
    rows' own features into the slot, [self | agg] rows of 2F, and the layer-1
    forward and dW read that block without the self-index round) feeds the
    GEMMs the same values in the same order as self_rows off (the GEMMs gather
    X[dst] themselves): loss, gradients and parameters bitwise equal (gcn: the
    slot keeps the agg half only)."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    if bf16:
        X = X.to(torch.bfloat16)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 96, 0, 1, 9))[:5]
    out = []
    for self_rows in (False, True):
        t = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, gcn=gcn, max_norm=0.05,
                                seed=824)
        t.set_option("self_rows", self_rows)
        r = train.Runner(t, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10],
                         fail_empty=agg == "MAX", gcn=gcn, depth=2)
        r.run(len(batches))
        torch.cuda.synchronize()
        out.append((t.p.params.clone(), t.p.grads.clone(), float(t.loss)))
        r.close()
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("agg,gcn,layers,name,B", [
    ("MEAN", False, 2, "rmat", 96), ("MAX", False, 2, "rmat", 96), ("MEAN", True, 2, "rmat", 96),
    ("MEAN", False, 3, "rmat", 96),
    # B >= 1024: the layer-2 weight gradient spans more than 8 row slabs, so the
    # fused launch's slab sum and the standalone split kernel both group slabs
    ("MEAN", False, 2, "pubmed", 1536), ("MAX", False, 2, "pubmed", 1536)])
def test_fused_backward_matches_unfused(gs, agg, gcn, layers, name, B):
    """The horizontally fused backward launches (kernels/bwd.hip) run the same
    per-role kernels and summation orders as the five-launch sequence (the
    slab sums in one shared grouped order, linear_dev.hpp sum_slabs_body):
    loss and every gradient bitwise equal.  The single-process update then
    clips with the norm partials those launches left (another summation order
    of the same squares): parameters within fp32 rounding."""
    graph, g, n = _graph(gs, name)
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    fan = [25, 10, 5][:layers]
    a = train.NativeTrainer(graph, X, labels, 16, num_layers=layers, fanouts=fan, agg_func=agg, gcn=gcn, seed=824)
    a.set_option("top_launch", False)  # the fused layer backward itself (the top launch: its own test)
    b = train.NativeTrainer(graph, X, labels, 16, num_layers=layers, fanouts=fan, agg_func=agg, gcn=gcn, seed=824)
    b.set_option("fused_bwd", False)
    rng = gs.RNG(21)
    done = 0
    for roots in train.rank_batches(np.nonzero(graph.degrees())[0], B, 0, 1, 13):
        if done == 3:
            break
        s = gs.sample(graph, rng, roots, fan)
        if agg == "MAX" and any(s.n_empty(j) for j in range(1, layers + 1)):
            continue  # MAX over an empty neighbourhood raises (models.py:321-325)
        ds = models.DeviceSample(s, DEV)
        r = torch.from_numpy(roots.astype(np.int32)).to(DEV)
        la = a.forward_backward(ds, r).clone()
        lb = b.forward_backward(ds, r).clone()
        torch.cuda.synchronize()
        assert torch.equal(la, lb)
        assert torch.equal(a.p.grads, b.p.grads)
        a.apply_update()
        b.apply_update()
        torch.testing.assert_close(a.p.params, b.p.params, atol=2e-6, rtol=1e-5)
        b.p.params.copy_(a.p.params)  # keep both on one trajectory
        done += 1
    assert done >= 1


@pytest.mark.parametrize("agg,name,B", [("MEAN", "pubmed", 512), ("MAX", "pubmed", 512), ("MEAN", "rmat", 97),
                                         ("MAX", "pubmed", 1536)])
def test_top_launch_matches_separate_launches(gs, agg, name, B):
    """The one-launch top layer + loss head (kernels/top.hip: layer-2
    aggregate, linear, relu, NLL head, dZ and dIn on the matrix cores) against the
    separate launches it replaces (agg_fwd, the MFMA linear, cls_rows, the
    MFMA dIn role), including a batch that leaves its last 4-row block
    partial.  The aggregate is the same code (bitwise); the GEMMs split their
    K range over waves (4x4x1 multi-block MFMAs, partial sums added in a fixed
    order) and the logits over 8 lanes, so loss, gradients and the updated
    parameters agree within fp32 rounding of the k order (rtol 1e-5)."""
    graph, g, n = _graph(gs, name)
    X = torch.from_numpy(uniform_features(7, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    fan = [25, 10]
    a = train.NativeTrainer(graph, X, labels, 16, num_layers=2, fanouts=fan, agg_func=agg, seed=824)
    b = train.NativeTrainer(graph, X, labels, 16, num_layers=2, fanouts=fan, agg_func=agg, seed=824)
    b.set_option("top_launch", False)
    rng = gs.RNG(5)
    done = 0
    for roots in train.rank_batches(np.nonzero(graph.degrees())[0], B, 0, 1, 17):
        if done == 3:
            break
        s = gs.sample(graph, rng, roots, fan)
        if agg == "MAX" and any(s.n_empty(j) for j in range(1, 3)):
            continue
        ds = models.DeviceSample(s, DEV)
        r = torch.from_numpy(roots.astype(np.int32)).to(DEV)
        la = a.forward_backward(ds, r).clone()
        lb = b.forward_backward(ds, r).clone()
        torch.cuda.synchronize()
        torch.testing.assert_close(la, lb, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(a.p.grads, b.p.grads, atol=1e-7, rtol=1e-5)
        a.apply_update()
        b.apply_update()
        torch.cuda.synchronize()
        torch.testing.assert_close(a.p.params, b.p.params, atol=1e-7, rtol=1e-5)
        b.p.params.copy_(a.p.params)  # keep both on one trajectory
        done += 1
    assert done >= 1


@pytest.mark.parametrize("classes,fan,agg,B", [(3, [25, 10], "MEAN", 97), (7, [15, 5], "MAX", 512),
                                                (19, [25, 10], "MEAN", 130), (16, [31, 16], "MEAN", 64),
                                                (5, [40, 20], "MAX", 96)])
def test_top_launch_edge_shapes(gs, classes, fan, agg, B):
    """The one-launch top layer away from the benchmark's shape, against the
    separate launches: class counts below 16 (the small-C head's masked class
    lanes), above 16 (the general head: 8-part logits, a softmax wave per row),
    neighbour lists longer than one 32-row round of the launch's list gather
    (fanout 40) and ragged last row blocks; within fp32 rounding of the k
    order like the bench shape's test."""
    graph, g, n = _graph(gs, "pubmed")
    X = torch.from_numpy(uniform_features(9, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % classes).astype(np.int32)).to(DEV)
    a = train.NativeTrainer(graph, X, labels, classes, num_layers=2, fanouts=fan, agg_func=agg, seed=824)
    b = train.NativeTrainer(graph, X, labels, classes, num_layers=2, fanouts=fan, agg_func=agg, seed=824)
    b.set_option("top_launch", False)
    rng = gs.RNG(7)
    done = 0
    for roots in train.rank_batches(np.nonzero(graph.degrees())[0], B, 0, 1, 23):
        if done == 2:
            break
        s = gs.sample(graph, rng, roots, fan)
        if agg == "MAX" and any(s.n_empty(j) for j in range(1, 3)):
            continue
        ds = models.DeviceSample(s, DEV)
        r = torch.from_numpy(roots.astype(np.int32)).to(DEV)
        la = a.forward_backward(ds, r).clone()
        lb = b.forward_backward(ds, r).clone()
        torch.cuda.synchronize()
        assert torch.isfinite(la).all()
        torch.testing.assert_close(la, lb, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(a.p.grads, b.p.grads, atol=1e-7, rtol=1e-5)
        a.apply_update()
        b.apply_update()
        torch.cuda.synchronize()
        torch.testing.assert_close(a.p.params, b.p.params, atol=1e-7, rtol=1e-5)
        b.p.params.copy_(a.p.params)
        done += 1
    assert done >= 1


@pytest.mark.parametrize("classes,fan,agg", [(7, (15, 5), "MEAN"), (3, (31, 16), "MAX"), (5, (40, 20), "MEAN")])
def test_native_runner_matches_python_loop_edge_shapes(gs, classes, fan, agg):
    """The runner (resolved-id layer-1 gather, padded top records, deferred
    update) at fanouts and class counts away from the benchmark's, against the
    Python loop on the same sampler stream: bitwise equal parameters and loss,
    including the one-round gather's largest fanout (16) and fanouts past what
    the one-round gather and the top launch's records take (20, 40)."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % classes).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:5]
    a = train.NativeTrainer(graph, X, labels, classes, fanouts=fan, agg_func=agg, seed=824)
    b = train.NativeTrainer(graph, X, labels, classes, fanouts=fan, agg_func=agg, seed=824)
    pf = train.Prefetcher(graph, None, batches, list(fan), False, DEV, rngs=[train.make_rng(11, 0, 0)],
                          fail_empty=agg == "MAX")
    for _ in batches:
        ds, roots_dev, _info = pf.next()
        a.step(ds, roots_dev)
    pf.close()
    runner = train.Runner(b, graph, batches, [train.make_rng(11, 0, 0)], list(fan), gcn=False,
                          fail_empty=agg == "MAX", depth=2)
    runner.run(len(batches))
    torch.cuda.synchronize()
    assert torch.equal(a.p.params, b.p.params)
    assert float(a.loss) == float(b.loss)
    runner.close()


@pytest.mark.parametrize("agg,B,classes", [("MEAN", 512, 16), ("MAX", 97, 16), ("MEAN", 130, 7)])
def test_top_pair_matches_one_block(gs, agg, B, classes):
    """The top launch's pair form (two blocks per 4 roots, half of W2 each,
    the partial logits exchanged inside the launch, dIn as two partials the
    layer-2 backward adds) against the one-block form: loss, gradients and
    updated parameters within fp32 rounding of the k order, ragged batches
    and MAX included (a pair whose exchange gave up would turn them NaN)."""
    graph, g, n = _graph(gs, "pubmed")
    X = torch.from_numpy(uniform_features(3, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % classes).astype(np.int32)).to(DEV)
    a = train.NativeTrainer(graph, X, labels, classes, num_layers=2, fanouts=[25, 10], agg_func=agg, seed=824)
    b = train.NativeTrainer(graph, X, labels, classes, num_layers=2, fanouts=[25, 10], agg_func=agg, seed=824)
    a.set_option("top_pair", True)
    b.set_option("top_pair", False)
    rng = gs.RNG(11)
    done = 0
    for roots in train.rank_batches(np.nonzero(graph.degrees())[0], B, 0, 1, 29):
        if done == 3:
            break
        s = gs.sample(graph, rng, roots, [25, 10])
        if agg == "MAX" and any(s.n_empty(j) for j in range(1, 3)):
            continue
        ds = models.DeviceSample(s, DEV)
        r = torch.from_numpy(roots.astype(np.int32)).to(DEV)
        la = a.forward_backward(ds, r).clone()
        lb = b.forward_backward(ds, r).clone()
        torch.cuda.synchronize()
        assert torch.isfinite(la).all() and torch.isfinite(a.p.grads).all()
        torch.testing.assert_close(la, lb, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(a.p.grads, b.p.grads, atol=1e-7, rtol=1e-5)
        a.apply_update()
        b.apply_update()
        torch.cuda.synchronize()
        torch.testing.assert_close(a.p.params, b.p.params, atol=1e-7, rtol=1e-5)
        b.p.params.copy_(a.p.params)
        done += 1
    assert done >= 1


def test_top_launch_is_deterministic(gs):
    """The top launch's split-K partial sums are added in a fixed order: two
    trainers on the same batches leave bitwise the same loss, gradients and
    parameters."""
    graph, g, n = _graph(gs, "pubmed")
    X = torch.from_numpy(uniform_features(7, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    out = []
    for _ in range(2):
        t = train.NativeTrainer(graph, X, labels, 16, num_layers=2, fanouts=[25, 10], seed=824)
        rng = gs.RNG(5)
        for roots in list(train.rank_batches(np.nonzero(graph.degrees())[0], 512, 0, 1, 17))[:2]:
            ds = models.DeviceSample(gs.sample(graph, rng, roots, [25, 10]), DEV)
            t.forward_backward(ds, torch.from_numpy(roots.astype(np.int32)).to(DEV))
            t.apply_update()
        torch.cuda.synchronize()
        out.append((t.p.params.clone(), t.p.grads.clone(), float(t.loss)))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


def test_rccl_communicator_single_rank(gs):
    """The native RCCL communicator (gs_comm_*, torch's librccl) on one rank:
    unique id, init, an in-place sum all-reduce (identity at world 1)."""
    comm = train.Communicator(0, 1, DEV)
    x = torch.randn(100003, device=DEV)
    y = x.clone()
    from importlib import import_module
    _l = import_module("graphsage-pytorch_amd._lib")
    _l.check(_l.lib().gs_comm_allreduce_sum(comm._h, y.data_ptr(), y.numel(), _l.stream_ptr(DEV)))
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    comm.close()


@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
def test_runner_distributed_path_single_rank(gs, agg):
    """The runner's data-parallel update path (RCCL all-reduce of the flat
    gradients, clip of the averaged sum via gs_trainer_update) run with a
    one-rank communicator equals the single-process path (clip from the
    reductions' norm partials) to fp32 rounding of the norm."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:6]
    a = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, seed=824)
    b = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), agg_func=agg, seed=824)
    ra = train.Runner(a, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10],
                      fail_empty=agg == "MAX", depth=2)
    comm = train.Communicator(0, 1, DEV)
    rb = train.Runner(b, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10],
                      fail_empty=agg == "MAX", depth=2, comm=comm)
    ra.run(len(batches))
    rb.run(len(batches))
    torch.cuda.synchronize()
    torch.testing.assert_close(a.p.params, b.p.params, atol=2e-6, rtol=1e-5)
    assert abs(float(a.loss) - float(b.loss)) < 1e-5
    ra.close()
    rb.close()
    comm.close()


@pytest.mark.parametrize("max_norm,dtype", [(5.0, "f32"), (1e-3, "f32"), (5.0, "bf16"), (1e-3, "bf16")])
def test_runner_deferred_update_with_allreduce(gs, max_norm, dtype):
    """With a communicator the deferred update starts after the all-reduce:
    one launch computes the norm partials of the summed gradient and W1's
    speculative update, the next forward applies the clip + SGD.  Parameters
    and clipped gradients bitwise those of defer_update off (the all-reduce
    path's separate norm + SGD launches), one rank, bucketed all-reduce."""
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    if dtype == "bf16":
        X = X.to(torch.bfloat16)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:6]
    comm = train.Communicator(0, 1, DEV)
    out = []
    for defer in (False, True):
        t = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), max_norm=max_norm, seed=824)
        t.set_option("defer_update", defer)
        r = train.Runner(t, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10], depth=2,
                         comm=comm, ar_buckets=2)
        r.run(2)
        r.run(len(batches) - 2)
        torch.cuda.synchronize()
        out.append((t.p.params.clone(), t.p.grads.clone()))
        r.close()
    comm.close()
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("every", [1, 3])
def test_kernel_timer_sites_strided(gs, every):
    """The bench's kernel-bound timers (gs_trainer_time_kernels_every): with
    every = e, one launch in e of each armed site is timed (the e-th, 2e-th,
    ... since arming); durations are positive and the site names the kernel
    variant it launched."""
    lib = gs._lib.lib()
    graph, g, n = _graph(gs, "rmat")
    X = torch.from_numpy(uniform_features(5, n, 256)).to(DEV)
    labels = torch.from_numpy((np.arange(n) % 16).astype(np.int32)).to(DEV)
    batches = list(train.rank_batches(np.nonzero(graph.degrees())[0], 48, 0, 1, 9))[:9]
    t = train.NativeTrainer(graph, X, labels, 16, fanouts=(25, 10), seed=824)
    runner = train.Runner(t, graph, batches, [train.make_rng(11, 0, w) for w in range(2)], [25, 10], depth=2)
    gs._lib.check(lib.gs_trainer_time_kernels_every(t._h, 0b1111, 9, every))
    runner.run(9)
    torch.cuda.synchronize()
    for site in range(4):
        out = np.zeros(9, np.float32)
        got = int(lib.gs_trainer_kernel_times(t._h, site, out.ctypes.data, 9))
        assert got == 9 // every, (site, got)
        assert (out[:got] > 0).all()
        assert lib.gs_trainer_kernel_name(t._h, site).decode().startswith(("void gs::", "gs::"))
        # per-workgroup stamp statistics: the stamped sites (forward GEMM, dW,
        # top launch) give span >= max workgroup >= mean workgroup > 0; the
        # event-timed gather gives -1
        st = np.zeros((9, 4), np.float32)
        assert int(lib.gs_trainer_kernel_block_stats(t._h, site, st.ctypes.data, 9)) == got
        st = st[:got]
        if site in (1, 2, 3):
            assert (st[:, 1] > 0).all() and (st[:, 2] >= st[:, 1]).all(), st
            assert (st[:, 0] + 1e-2 >= st[:, 2]).all() and (st[:, 3] >= 0).all(), st
        else:
            assert (st == -1).all(), st
    runner.close()


@pytest.mark.parametrize("name,gcn,fanouts,agg", [("cora", False, [10, 10], "MEAN"), ("pubmed", False, [10, 10], "MEAN"),
                                                  ("rmat", True, [25, 10], "MEAN"), ("rmat", False, [5, 4, 3], "MAX"),
                                                  ("pubmed", False, [10, 10], "MAX")])
def test_graphsage_device_sampler_bitwise(gs, name, gcn, fanouts, agg):
    """device_sampler=True (the forward's sampling on the GPU,
    the module-global `random` state moved to the device and back): the
    embeddings, weight gradients and `random` state after every forward are
    bitwise those of the host sampler, over three batches (one large)."""
    graph, g, n = _graph(gs, name)
    X = torch.from_numpy(_features(name, n)).to(DEV)
    out = []
    for on in (False, True):
        torch.manual_seed(5)
        model = models.GraphSage(len(fanouts), X.shape[1], 128, X, graph, DEV, gcn=gcn, fanouts=fanouts, agg_func=agg,
                                 device_sampler=on).to(DEV)
        random.seed(21)
        embs, states = [], []
        nz = np.nonzero(graph.degrees())[0]
        for b, B in enumerate([300, 17, 2000]):
            roots = nz[b::3][:B].tolist()
            emb = model(roots)
            (emb * torch.from_numpy(uniform_features(8 + b, len(roots), 128)).to(DEV)).sum().backward()
            embs.append(emb.detach().cpu())
            states.append(random.getstate())
        grads = [getattr(model, f"sage_layer{i}").weight.grad.cpu() for i in range(1, len(fanouts) + 1)]
        out.append((embs, grads, states))
    (e0, g0, s0), (e1, g1, s1) = out
    assert s0 == s1
    for a, b in zip(e0 + g0, e1 + g1):
        assert torch.equal(a, b)
