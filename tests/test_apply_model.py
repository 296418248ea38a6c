"""The reference's epoch loop (utils.py:113-193) through the drop-in modules:
apply_model with extend_nodes (native), GraphSage (HIP), the fused supervised
head and the unsupervised losses (HIP), against the reference's own weights
after the same epoch (tests/golden/unsup_apply_model.npz, captured by
tests/golden/make_golden_unsup.py).

Tolerance: the sampled batches and the `random` stream are bit-exact (checked
through the final RNG state); the weights after 4-5 SGD steps at lr 0.7 are
compared at rtol 1e-3 / atol 1e-4 (fp32 summation-order drift of the GEMMs
and reductions, amplified by the steps; one-step parity is 1e-5 elsewhere).
"""
import importlib
import random
import types
from collections import defaultdict

import numpy as np
import pytest
import torch

from tests import unsup_cases as C
from tests.golden.synth import hashed_binary_features

models = importlib.import_module("graphsage-pytorch_amd.models")
unsup = importlib.import_module("graphsage-pytorch_amd.unsup")
utils = importlib.import_module("graphsage-pytorch_amd.utils")

CASES = {  # tag -> (learn_method, unsup_loss, agg)
    "cora_sup_normal": ("sup", "normal", "MEAN"),
    "cora_plus_unsup_normal": ("plus_unsup", "normal", "MEAN"),
    "cora_unsup_margin": ("unsup", "margin", "MEAN"),
    "cora_plus_unsup_margin": ("plus_unsup", "margin", "MEAN"),
    "cora_sup_normal_max": ("sup", "normal", "MAX"),
}


def _cora():
    g = C.graphs()
    src, dst, n = g["cora_src"].tolist(), g["cora_dst"].tolist(), int(g["cora_n"][0])
    adj = defaultdict(set)
    for a, b in zip(src, dst):
        adj[a].add(b)
        adj[b].add(a)
    return adj, n


def _split(n, seed):
    np.random.seed(seed)
    perm = np.random.permutation(n)
    t, v = n // 3, n // 6
    return perm[:t], perm[t:t + v], perm[t + v:]


@pytest.mark.gpu
@pytest.mark.parametrize("tag", sorted(CASES))
def test_apply_model_matches_reference(tag):
    A = C.apply_file()
    lm, ulo, agg = CASES[tag]
    n_train, b_sz, seed, n_classes = (int(x) for x in A[f"{tag}__meta"])
    adj, n = _cora()
    dev = torch.device("cuda", 0)
    test, val, train = _split(n, seed)
    train = train[:n_train]
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    feats = torch.from_numpy(hashed_binary_features(n, 1433)).to(dev)
    labels = (np.arange(n) % n_classes).astype(np.int64)
    dc = types.SimpleNamespace(g_test=test, g_val=val, g_train=train, g_labels=labels)
    gsage = models.GraphSage(2, 1433, 128, feats, adj, dev, agg_func=agg).to(dev)
    cls = models.Classification(128, n_classes).to(dev)
    ul = unsup.UnsupervisedLoss(adj, train, dev)

    def params():
        return {**{f"gs.{k}": v for k, v in gsage.state_dict().items()},
                **{f"cls.{k}": v for k, v in cls.state_dict().items()}}

    def pick(k, t):
        t = t.detach().cpu().numpy()
        sub = f"{tag}__sub__{k}"
        return t.reshape(-1)[A[sub]] if sub in A.files else t

    for k, v in params().items():  # same seeded init as the reference
        np.testing.assert_array_equal(pick(k, v), A[f"{tag}__init__{k}"])
    utils.apply_model(dc, "g", gsage, cls, ul, b_sz, ulo, dev, lm, verbose=False)
    torch.cuda.synchronize()
    assert list(random.getstate()[1]) == A[f"{tag}__state"].tolist()
    for k, v in params().items():
        np.testing.assert_allclose(pick(k, v), A[f"{tag}__final__{k}"], rtol=1e-3, atol=1e-4, err_msg=k)
        s = f"{tag}__sum__{k}"
        if s in A.files:
            tot = v.detach().double()
            np.testing.assert_allclose([tot.sum().item(), tot.abs().sum().item()], A[s][:2], rtol=1e-4)


def test_apply_model_rejects_unknown_unsup_loss():
    with pytest.raises(SystemExit):
        utils.apply_model(types.SimpleNamespace(), "g", None, None, None, 20, "bogus", "cpu", "sup",
                          verbose=False)
