"""evaluate / get_gnn_embeddings / train_classification (utils.py:13-111,
SURVEY §8 f-3) through the drop-in modules, against the reference's own
outputs on the same trained weights (tests/golden/eval_utils.npz, captured by
tests/golden/make_golden_eval.py), plus the native forward-only pipeline
(train.Embedder) and its rank sharding.

Tolerances: RNG state, F1 values and max_vali_f1 exact (the reference's
smallest top-2 logit margin on the val set is 9e-4, far above fp32 drift);
embeddings 1e-5; classifier weights after 2 epochs x 28 SGD steps 1e-4.
"""
import importlib
import inspect
import os
import random
import types

import numpy as np
import pytest
import torch

from tests import unsup_cases as C
from tests.golden.synth import uniform_features

models = importlib.import_module("graphsage-pytorch_amd.models")
utils = importlib.import_module("graphsage-pytorch_amd.utils")
sampler = importlib.import_module("graphsage-pytorch_amd.sampler")
train = importlib.import_module("graphsage-pytorch_amd.train")

G = os.path.join(os.path.dirname(__file__), "golden", "eval_utils.npz")


def _golden():
    return np.load(G)


def _setup(dev):
    A = _golden()
    n, F, H, Cn, seed = (int(x) for x in A["meta"])
    g = C.graphs()
    from collections import defaultdict
    adj = defaultdict(set)
    for a, b in zip(g["cora_src"].tolist(), g["cora_dst"].tolist()):
        adj[a].add(b)
        adj[b].add(a)
    np.random.seed(seed)
    perm = np.random.permutation(n)
    t, v = n // 3, n // 6
    test, val, tr = perm[:t], perm[t:t + v], perm[t + v:]
    labels = (np.arange(n) % Cn).astype(np.int64)
    dc = types.SimpleNamespace(g_test=test, g_val=val, g_train=tr, g_labels=labels)
    feats = torch.from_numpy(uniform_features(int(A["feat_seed"]), n, F)).to(dev)
    gsage = models.GraphSage(2, F, H, feats, adj, dev).to(dev)
    cls = models.Classification(H, Cn).to(dev)
    with torch.no_grad():
        for k, p in gsage.state_dict().items():
            p.copy_(torch.from_numpy(A[f"w__gs.{k}"]))
        for k, p in cls.state_dict().items():
            p.copy_(torch.from_numpy(A[f"w__cls.{k}"]))
    return A, dc, gsage, cls


def _state():
    return np.array(random.getstate()[1], np.int64)


# ------------------------------------------------------------------ CPU tests
def test_shard_ids_cover_every_batch_once():
    for n, b, w in [(23, 4, 2), (2708, 500, 8), (5, 500, 3), (1000, 500, 2)]:
        got = np.concatenate([utils.shard_ids(n, b, r, w) for r in range(w)])
        assert sorted(got.tolist()) == list(range(n))
        for r in range(w):  # whole reference batches, batch i on rank i % w
            ids = utils.shard_ids(n, b, r, w)
            assert all((i // b) % w == r for i in ids.tolist())


def test_evaluate_golden_is_self_consistent():
    A = _golden()
    assert float(A["eval_improved__max"]) == float(A["eval_improved__val_f1"][0])
    assert float(A["eval_kept__max"]) == 1.0
    assert int(A["eval_improved__saved"]) == 1
    assert float(A["tc__max"]) == max(A["tc__val_f1"].max(), 0.0)


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
def test_evaluate_matches_reference(tmp_path, monkeypatch):
    dev = torch.device("cuda", 0)
    A, dc, gsage, cls = _setup(dev)
    monkeypatch.chdir(tmp_path)
    random.seed(5)
    m = utils.evaluate(dc, "g", gsage, cls, dev, 0.0, "golden", 0)
    assert m == float(A["eval_improved__max"])
    np.testing.assert_array_equal(_state(), A["eval_improved__state"])
    saved = os.listdir(tmp_path / "models")
    assert len(saved) == 1 and saved[0].endswith("{:.4f}.torch".format(float(A["eval_improved__test_f1"][0])))
    assert all(p.requires_grad for p in list(gsage.parameters()) + list(cls.parameters()))
    loaded = torch.load(tmp_path / "models" / saved[0], weights_only=False)  # our own checkpoint
    torch.testing.assert_close(loaded[0].sage_layer1.weight, gsage.sage_layer1.weight)
    random.seed(5)
    with torch.no_grad():
        logits = cls(gsage(dc.g_val)).cpu().numpy()
    np.testing.assert_allclose(logits, A["eval__val_logits"], atol=1e-5, rtol=1e-5)
    random.seed(6)
    m = utils.evaluate(dc, "g", gsage, cls, dev, 1.0, "golden", 1)
    assert m == 1.0
    np.testing.assert_array_equal(_state(), A["eval_kept__state"])
    assert len(os.listdir(tmp_path / "models")) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [None, 1])
def test_get_gnn_embeddings_matches_reference(streams):
    """Default loop (module per batch) and the native forward-only runner
    with one stream: both the reference's embeddings and `random` state."""
    dev = torch.device("cuda", 0)
    A, dc, gsage, cls = _setup(dev)
    random.seed(7)
    E = utils.get_gnn_embeddings(gsage, dc, "g", sampler_streams=streams)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_state(), A["embed__state"])
    E = E.cpu().numpy()
    np.testing.assert_allclose(E[A["embed__rows"]], A["embed__emb"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(E.astype(np.float64).sum(1), A["embed__rowsum"], atol=1e-4, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("b_sz", [500, 256])
def test_embedder_streams_match_module_forward(b_sz):
    """S = 3 sampler streams, merged steps of m batches: batch i is sampled by
    stream (i // m) % 3 (the trailing partial batch too); each batch equals the
    drop-in module's forward drawing from that stream."""
    dev = torch.device("cuda", 0)
    A, dc, gsage, cls = _setup(dev)
    S = 3
    E = utils.get_gnn_embeddings(gsage, dc, "g", b_sz=b_sz, sampler_streams=S, seed=11)
    n = len(dc.g_labels)
    rngs = [sampler.RNG(train.rank_seed(11, 0, w)) for w in range(S)]
    m = inspect.signature(train.Embedder.__init__).parameters["merge"].default  # get_gnn_embeddings' merge
    assert m > 1
    with torch.no_grad():
        for i, lo in enumerate(range(0, n, b_sz)):
            gsage.rng = rngs[(i // m) % S]
            ref = gsage(np.arange(lo, min(n, lo + b_sz)))
            torch.testing.assert_close(E[lo:lo + len(ref)], ref, atol=1e-6, rtol=1e-6)
    gsage.rng = None


@pytest.mark.gpu
def test_train_classification_matches_reference(tmp_path, monkeypatch):
    dev = torch.device("cuda", 0)
    A, dc, gsage, cls = _setup(dev)
    monkeypatch.chdir(tmp_path)
    random.seed(8)
    np.random.seed(8)
    cls2, m = utils.train_classification(dc, gsage, cls, "g", dev, 0.0, "golden", epochs=2)
    assert cls2 is cls
    assert m == float(A["tc__max"])
    np.testing.assert_array_equal(_state(), A["tc__state"])
    for k, v in cls.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), A[f"tc__cls.{k}"], atol=1e-4, rtol=1e-4, err_msg=k)
