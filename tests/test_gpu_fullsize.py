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
  native path) equals the drop-in module's forward batch by batch;
* the two other benchmarked training paths on the same graph, each through
  NativeTrainer + Runner (sampler threads held until release) against the
  oracle's train step over 3 steps:
  - configs[3]: MAX over a bf16 feature table (bf16 agg_ids gather, bf16
    layer-1 MFMA GEMM, dW1 from bf16 inputs, argmax backward at layer 2);
    the oracle runs on the same bf16 values with W1 and the layer-1
    aggregate rounded to bf16 in the GEMM (oracle.forward_dense
    bf16_layer1).  bf16·bf16 products are exact in fp32 and the MAX aggregate
    is exact, so only fp32 summation order differs — plus, rarely, a bf16
    rounding of W1 that flips between two fp32 values 1 ulp apart, one bf16
    ulp (2^-8 relative) on that weight: tolerance 1e-3 on loss and weights;
  - configs[4]'s feature width F = 128 (rmat16m): MEAN through the 32-lane
    agg_ids variant (512-byte rows), tolerance 1e-4 as the fp32 test.
"""
import time
import importlib
import random

import numpy as np
import pytest
import torch

import oracle
from tests.fullsize_parity import check_embeddings_vs_oracle, check_pack_vs_oracle, check_timed_steps_vs_oracle

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


@pytest.fixture(scope="module")
def adj(wl):
    return oracle.Adjacency(wl["src"], wl["dst"], wl["n"])


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


def test_fullsize_runner_vs_oracle_train_steps(wl, adj, native):
    tr, losses, sizes = native
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


def test_fullsize_timed_step_embeddings_and_grads_vs_oracle(wl, adj):
    """configs[2] (the headline): the bench's timed training step itself —
    root embeddings and every gradient before clip + SGD, steps 1 and 2 of one
    runner call (step 2: the forward applying step 1's deferred update) —
    against oracle autograd at 1e-5 (fp32)."""
    worst = check_timed_steps_vs_oracle(train, wl, adj, wl["X"], wl["X"].cpu(), FAN, C)
    print("max |emb diff|, max |grad diff|, max |grad| per step:", worst)


def test_fullsize_timed_step_fp32_max_vs_oracle(wl, adj):
    """The headline graph with the MAX aggregator over the fp32 feature table
    (models.py:316-326: per-row element-wise max, first-index argmax in the
    backward): the bench's timed steps 1 and 2 against oracle autograd at 1e-5."""
    worst = check_timed_steps_vs_oracle(train, wl, adj, wl["X"], wl["X"].cpu(), FAN, C, agg="MAX")
    print("max |emb diff|, max |grad diff|, max |grad| per step:", worst)


def test_fullsize_timed_step_bf16_max_vs_oracle(wl, adj):
    """configs[3]: the same over a bf16 feature table with MAX; the oracle
    rounds layer 1's W1 and aggregate to bf16 as the HIP GEMM reads them.
    Step 1 at 1e-5; step 2 at the bf16 config's 1e-3 (its W1 after one SGD
    step may round to a bf16 value one ulp apart from the oracle's, module doc)."""
    Xb = torch.empty(wl["n"], F, dtype=torch.bfloat16, device=DEV)
    ops.fill_uniform(Xb, SEED)
    worst = check_timed_steps_vs_oracle(train, wl, adj, Xb, Xb.float().cpu(), FAN, C, agg="MAX", bf16=True,
                                        tols=(1e-5, 1e-3))
    print("max |emb diff|, max |grad diff|, max |grad| per step:", worst)


def test_fullsize_first_batch_indices_and_embeddings_vs_oracle(wl, adj):
    """North_star's parity bar at the headline size, per root of the first
    batch: the runner's pack (its sampler threads' gs_sample_pack_run_multi_team)
    holds exactly the oracle's sampled sets at both hops, the |L1| frontier in
    its CPython set order and the oracle's |L0| (tests/fullsize_parity.py);
    the drop-in module's forward on the same stream equals
    oracle.forward_dense within 1e-5 (fp32)."""
    roots = wl["batches"][0]
    seed = train.rank_seed(SEED, 0, 0)
    hops = check_pack_vs_oracle(wl["graph"], adj, roots, FAN, seed)
    W = [w.to(DEV) for w in train.reference_init(2, F, H, C, False, SEED)[0]]
    check_embeddings_vs_oracle(models, wl["graph"], wl["X"], wl["X"].cpu(), hops, roots, FAN, W, seed, DEV)


def test_fullsize_device_sampler_past_capacity_falls_back(wl):
    """A forward batch too large for the device sampler's windows / tables
    (16 Ki roots at fanouts 25, 10: the hop-1 union alone outgrows the
    device table) raises DeviceLimit inside GraphSage(device_sampler=True),
    which then samples on the host from the untouched stream: the same
    embeddings and `random` state as the host-sampler module."""
    roots = np.arange(16384, dtype=np.int64) * 127 % wl["n"]
    roots = roots[wl["graph"].degrees()[roots] > 0]
    W = [w.to(DEV) for w in train.reference_init(2, F, H, C, False, SEED)[0]]
    out = []
    for dev_s in (False, True):
        rng = sampler.RNG(11)
        m = models.GraphSage(2, F, H, wl["X"], wl["graph"], DEV, fanouts=FAN, rng=rng,
                             device_sampler=dev_s).to(DEV)
        with torch.no_grad():
            for i in (1, 2):
                getattr(m, f"sage_layer{i}").weight.copy_(W[i - 1])
            e_big = m(roots).cpu()
            st_big = rng.getstate()
            # the same module again with normal batches: the failed device run
            # must leave no stale union marks behind (its epoch is skipped)
            e_small = [m(roots[o:o + 512]).cpu() for o in (0, 4096)]
            out.append((e_big, st_big, e_small, rng.getstate()))
    (e0, (mt0, p0), s0, (mt0b, p0b)), (e1, (mt1, p1), s1, (mt1b, p1b)) = out
    assert torch.equal(e0, e1)
    assert p0 == p1
    np.testing.assert_array_equal(mt0, mt1)
    for a, b in zip(s0, s1):
        assert torch.equal(a, b)
    assert p0b == p1b
    np.testing.assert_array_equal(mt0b, mt1b)


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


def _oracle_steps(wl, adj, X_cpu, agg, feat, bf16, tol, tr, losses, sizes):
    labels = wl["labels"].cpu().long()
    sage_w, cw, cb = train.reference_init(2, feat, H, C, False, SEED)
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
        ref = oracle.train_step_dense(adj, roots.tolist(), FAN, X_cpu, W, cw, cb, labels[torch.from_numpy(roots)],
                                      agg=agg, rng=rng, bf16_layer1=bf16)
        assert abs(losses[i] - ref) < tol, (i, losses[i], ref)
    np.testing.assert_array_equal(sizes[:2, 0], n_dst)
    sd = tr.p.state_dict()
    for i in (1, 2):
        torch.testing.assert_close(sd[f"sage_layer{i}.weight"].cpu(), W[i - 1].detach(), atol=tol, rtol=tol)
    torch.testing.assert_close(sd["layer.0.weight"].cpu(), cw.detach(), atol=tol, rtol=tol)
    torch.testing.assert_close(sd["layer.0.bias"].cpu(), cb.detach(), atol=tol, rtol=tol)


def _held_runner(wl, X, agg):
    """NativeTrainer + Runner over the 3 batches with the sampler threads held
    until release (the bench's measurement mode): nothing is sampled before."""
    tr = train.NativeTrainer(wl["graph"], X, wl["labels"], C, fanouts=FAN, agg_func=agg, seed=SEED)
    r = train.Runner(tr, wl["graph"], wl["batches"], [train.make_rng(SEED, 0, w) for w in range(S)], FAN,
                     fail_empty=agg == "MAX", depth=2, hold=True)
    time.sleep(0.2)
    assert r.progress() == (0, 0)  # held: no batch sampled
    r.release(len(wl["batches"]))
    losses = []
    for _ in wl["batches"]:
        r.run(1)
        losses.append(float(tr.loss.item()))
    sizes = r.stats()["hop_sizes_sum"]
    assert r.progress() == (len(wl["batches"]), len(wl["batches"]))
    r.close()
    return tr, losses, sizes


def test_fullsize_bf16_max_runner_vs_oracle(wl, adj):
    """configs[3]: rmat2m, MAX, bf16 feature table (tolerance 1e-3, see the module doc)."""
    Xb = torch.empty(wl["n"], F, dtype=torch.bfloat16, device=DEV)
    ops.fill_uniform(Xb, SEED)  # RNE of the fp32 table's values
    tr, losses, sizes = _held_runner(wl, Xb, "MAX")
    Xc = Xb.float().cpu()
    del Xb
    _oracle_steps(wl, adj, Xc, "MAX", F, True, 1e-3, tr, losses, sizes)


def test_fullsize_f128_mean_runner_vs_oracle(wl, adj):
    """configs[4]'s F = 128 on the rmat2m graph: the 32-lane agg_ids gather (tolerance 1e-4)."""
    X128 = torch.empty(wl["n"], 128, dtype=torch.float32, device=DEV)
    ops.fill_uniform(X128, SEED)
    tr, losses, sizes = _held_runner(wl, X128, "MEAN")
    _oracle_steps(wl, adj, X128.cpu(), "MEAN", 128, False, 1e-4, tr, losses, sizes)


@pytest.mark.parametrize("S_", [1, 2])
def test_fullsize_device_sampler_runner_matches_host(wl, S_):
    """SURVEY §8 f-4 as a training path: Runner(sampler="device") — packs
    sampled on the GPU, no host sampler threads — over the same batches and
    streams as the host-sampler runner (held until release, as the bench
    runs): bitwise the same losses, parameters, hop sizes, and the same
    stream states afterwards (the reference's `random` consumption)."""
    out = {}
    for mode in ("host", "device"):
        tr = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], C, fanouts=FAN, seed=SEED)
        rngs = [train.make_rng(SEED, 0, w) for w in range(S_)]
        r = train.Runner(tr, wl["graph"], wl["batches"], rngs, FAN, depth=2, hold=True, sampler=mode)
        time.sleep(0.1)
        assert r.progress() == (0, 0)
        r.release(len(wl["batches"]))
        losses = []
        for _ in wl["batches"]:
            r.run(1)
            losses.append(float(tr.loss.item()))
        sizes = r.stats()["hop_sizes_sum"]
        r.close()
        out[mode] = (tr.p.params.clone(), losses, sizes, [g.getstate() for g in rngs])
    (p_h, l_h, s_h, st_h), (p_d, l_d, s_d, st_d) = out["host"], out["device"]
    assert l_h == l_d
    assert torch.equal(p_h, p_d)
    np.testing.assert_array_equal(s_h, s_d)
    for (mt_h, pos_h), (mt_d, pos_d) in zip(st_h, st_d):
        assert pos_h == pos_d
        np.testing.assert_array_equal(mt_h, mt_d)
