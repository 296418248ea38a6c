"""Pin the oracle (CPU restatement) against vectors captured from the reference."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import Adjacency, forward_dense, sample_layers
from tests.golden.synth import hashed_binary_features, uniform_features

G = os.path.join(os.path.dirname(__file__), "golden")


def _graphs():
    return np.load(os.path.join(G, "graphs.npz"))


def _adj(name):
    g = _graphs()
    return Adjacency(g[f"{name}_src"], g[f"{name}_dst"], int(g[f"{name}_n"][0]))


@pytest.mark.parametrize("name", ["cora", "pubmed", "rmat"])
def test_oracle_adjacency_order(name):
    g = _graphs()
    adj = _adj(name)
    ptr, col = g[f"{name}_row_ptr"], g[f"{name}_col"]
    for v in range(len(adj)):
        assert list(adj[v]) == col[ptr[v]:ptr[v + 1]].tolist()


def _sample_cases(name):
    S = np.load(os.path.join(G, f"sample_{name}.npz"))
    keys = sorted({k.split("__")[0] for k in S.files})
    return S, keys


@pytest.mark.parametrize("name", ["cora", "pubmed", "rmat"])
def test_oracle_sampling_matches_reference(name):
    S, keys = _sample_cases(name)
    adj = _adj(name)
    for key in keys:
        seed = int(key.split("_")[0][1:])
        fan = [int(x) for x in key.split("_f")[1].split("-")]
        random.seed(seed)
        hops = sample_layers(adj, S[key + "__roots"].tolist(), fan)
        for j, (_, samp, _, union) in enumerate(hops, start=1):
            assert union == S[f"{key}__h{j}_union"].tolist(), (key, j)
            ptr, items = S[f"{key}__h{j}_set_ptr"], S[f"{key}__h{j}_set_items"]
            got = [x for s in samp for x in s]
            assert got == items.tolist(), (key, j)
            assert np.array_equal(np.cumsum([0] + [len(s) for s in samp]), ptr)
        assert list(random.getstate()[1]) == S[key + "__state"].tolist()


def test_oracle_rng_kats():
    for rec in json.load(open(os.path.join(G, "rng.json"))):
        random.seed(rec["seed"])
        assert [random.getrandbits(32) for _ in range(8)] == rec["bits32"]


FORWARDS = [("cora", "MEAN", "sage"), ("cora", "MAX", "sage"), ("cora", "MEAN", "gcn"),
            ("cora", "MAX", "gcn"), ("rmat", "MEAN", "sage"), ("rmat", "MAX", "sage"),
            ("pubmed", "MEAN", "sage")]


def golden_features(name, n):
    if name == "cora":
        return hashed_binary_features(n, 1433)
    if name == "rmat":
        return uniform_features(77, n, 100)
    return uniform_features(11, n, 64)


@pytest.mark.parametrize("name,agg,mode", FORWARDS)
def test_oracle_forward_backward_matches_reference(name, agg, mode):
    R = np.load(os.path.join(G, f"forward_{name}_{agg}_{mode}.npz"))
    g = _graphs()
    n = int(g[f"{name}_n"][0])
    adj = _adj(name)
    X = torch.from_numpy(golden_features(name, n))
    W = [torch.tensor(R["w__sage_layer1.weight"], requires_grad=True),
         torch.tensor(R["w__sage_layer2.weight"], requires_grad=True)]
    random.seed({"cora": 824, "rmat": 5, "pubmed": 824}[name])
    hops = sample_layers(adj, R["roots"].tolist(), [10, 10])
    emb = forward_dense(hops, X, W, agg, mode == "gcn")
    assert list(random.getstate()[1]) == R["state"].tolist()
    torch.testing.assert_close(emb, torch.from_numpy(R["emb"]), atol=1e-5, rtol=1e-5)
    (emb * torch.from_numpy(uniform_features(31, len(R["roots"]), 128))).sum().backward()
    for i in (1, 2):
        torch.testing.assert_close(W[i - 1].grad, torch.from_numpy(R[f"grad__sage_layer{i}.weight"]),
                                   atol=1e-5, rtol=1e-5)
