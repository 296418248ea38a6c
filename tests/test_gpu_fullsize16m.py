"""Parity of configs[4]'s per-GPU workload at its full size (BASELINE.json
configs[4], bench.py `rmat16m`): R-MAT scale 24 (16,777,216 ids), 160,000,000
pairs, 128-d fp32 features — a 2^31-element (8.6 GB) feature table —,
fanouts (25, 10), MEAN, B = 512 roots per step.  This is what each rank of the
8-GPU job trains on (the graph and features are replicated).

The native path (NativeTrainer + Runner, 2 sampler streams held until
release, the bench's measurement mode) over 3 steps against the oracle's train
step (oracle.train_step_dense over the lazy dict-of-sets oracle.Adjacency) on
the same graph, batches and `random` streams (models.py:241-330,
utils.py:144-191):

* per-hop frontier sizes equal, and each oracle step consumes exactly the
  words a probe of the same stream draws (RNG consumption exact);
* loss per step and final weights within 1e-4 (the tolerance of the 2M test);
* a second runner over the same batches: bitwise the same parameters and losses.

Rows of the table are addressed with int64 in every layer-1 kernel (agg_ids,
the layer-1 forward's self rows, dW1's self rows): element offsets reach
2^31 - 1 and byte offsets 8.6 G (past 2^32) in every batch here.
"""
import importlib
import random
import time

import numpy as np
import pytest
import torch

import oracle
from tests.fullsize_parity import check_embeddings_vs_oracle, check_pack_vs_oracle, check_timed_steps_vs_oracle

pytestmark = pytest.mark.gpu

train = importlib.import_module("graphsage-pytorch_amd.train")
models = importlib.import_module("graphsage-pytorch_amd.models")
ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")
DEV = torch.device("cuda", 0)
SEED, F, H, C, B, FAN, S, SCALE, PAIRS = 824, 128, 128, 16, 512, [25, 10], 2, 24, 160_000_000


class _Rows:
    """The device feature table as the oracle indexes it (X[ids] -> CPU rows),
    without copying all 8.6 GB to the host."""

    def __init__(self, X):
        self.X = X

    def __len__(self):
        return self.X.shape[0]

    def __getitem__(self, idx):
        return self.X[torch.as_tensor(idx, dtype=torch.long).to(self.X.device)].float().cpu()


@pytest.fixture(scope="module")
def wl(gs):
    t0 = time.time()
    src, dst = gs.rmat_pairs(SCALE, PAIRS, seed=SEED, n_threads=16)
    n = 1 << SCALE
    graph = gs.CSRGraph.from_pairs(src, dst, n, n_threads=16)
    X = torch.empty(n, F, dtype=torch.float32, device=DEV)
    assert X.numel() == 2 ** 31
    ops.fill_uniform(X, SEED)
    labels = torch.from_numpy((np.arange(n) % C).astype(np.int32)).to(DEV)
    cands = np.nonzero(graph.degrees() > 0)[0]
    batches = list(train.rank_batches(cands, B, 0, 1, SEED + 1000))[:3]
    assert max(int(b.max()) for b in batches) >= (1 << 24) - (1 << 20)  # ids high in the table
    print(f"[rmat16m] graph + features {time.time() - t0:.1f} s", flush=True)
    return dict(src=src, dst=dst, n=n, graph=graph, X=X, labels=labels, batches=batches)


def _run(wl):
    tr = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], C, fanouts=FAN, seed=SEED)
    r = train.Runner(tr, wl["graph"], wl["batches"], [train.make_rng(SEED, 0, w) for w in range(S)], FAN,
                     depth=2, hold=True)
    time.sleep(0.2)
    assert r.progress() == (0, 0)  # held: nothing sampled before release
    r.release(len(wl["batches"]))
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


@pytest.fixture(scope="module")
def adj(wl):
    t0 = time.time()
    a = oracle.Adjacency(wl["src"], wl["dst"], wl["n"], sort_device=DEV)
    print(f"[rmat16m] oracle adjacency index {time.time() - t0:.1f} s", flush=True)
    return a


def test_rmat16m_first_batch_indices_and_embeddings_vs_oracle(wl, adj):
    """Per root of the first batch at the 16M size: the runner's pack holds
    exactly the oracle's sampled sets at both hops, the |L1| frontier in its
    CPython set order and the oracle's |L0|; the module forward on the same
    stream equals oracle.forward_dense within 1e-5 (tests/fullsize_parity.py)."""
    roots = wl["batches"][0]
    seed = train.rank_seed(SEED, 0, 0)
    hops = check_pack_vs_oracle(wl["graph"], adj, roots, FAN, seed)
    W = [w.to(DEV) for w in train.reference_init(2, F, H, C, False, SEED)[0]]
    check_embeddings_vs_oracle(models, wl["graph"], wl["X"], _Rows(wl["X"]), hops, roots, FAN, W, seed, DEV)


def test_rmat16m_timed_step_embeddings_and_grads_vs_oracle(wl, adj):
    """configs[4]'s per-GPU step as the bench times it (F = 128): root
    embeddings and every gradient before clip + SGD over steps 1 and 2 of one
    runner call, against oracle autograd at 1e-5 (tests/fullsize_parity.py)."""
    worst = check_timed_steps_vs_oracle(train, wl, adj, wl["X"], _Rows(wl["X"]), FAN, C)
    print("max |emb diff|, max |grad diff|, max |grad| per step:", worst)


def test_rmat16m_runner_vs_oracle_train_steps(wl, native, adj):
    tr, losses, sizes = native
    X = _Rows(wl["X"])
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


def test_rmat16m_runner_is_deterministic(wl, native):
    tr, losses, sizes = native
    tr2, losses2, sizes2 = _run(wl)
    assert torch.equal(tr.p.params, tr2.p.params)
    assert losses == losses2
    np.testing.assert_array_equal(sizes, sizes2)
