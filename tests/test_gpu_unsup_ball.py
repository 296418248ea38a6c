"""extend_nodes' negatives with the 5-hop balls and the far-list picks on the
GPU (kernels/unsup_ball.hip, gs_unsup_attach_device):

* the reference-captured cases (tests/golden/unsup_extend.npz: Cora / Pubmed /
  R-MAT, num_neg 6 and 100, isolated nodes, batches whose models.py:147
  assertion fails) replayed through UnsupervisedLoss on a HIP device: unique
  list, pair lists, per-node dicts and the `random` state bit-exact;
* larger randomized batches, device path == host path (every output and the
  stream), on graphs whose far lists take all three orders (copy order,
  ascending ids, host emulator for a small fresh-set table).
"""
import importlib
import random

import numpy as np
import pytest
import torch

from tests import unsup_cases as C
from tests.test_unsup_native import _check, _graph

pytestmark = pytest.mark.gpu

U = importlib.import_module("graphsage-pytorch_amd.unsup")
gs = importlib.import_module("graphsage-pytorch_amd")


@pytest.mark.parametrize("tag", C.extend_tags())
def test_device_balls_match_reference(tag):
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case(tag)
    ul = U.UnsupervisedLoss(_graph(name), train, torch.device("cuda", 0), n_threads=4, device_balls=True)
    assert ul.device_balls
    random.seed(seed)
    for b in batches:
        if int(b["error"]):
            with pytest.raises(AssertionError):
                ul.extend_nodes(b["nodes"], num_neg=num_neg)
            uniq = ul.unique_nodes_batch
        else:
            uniq = ul.extend_nodes(b["nodes"], num_neg=num_neg)
        _check(ul, uniq, b)


def _outputs(ul, nodes, num_neg, seed):
    rng = gs.RNG(seed)
    ul.rng = rng
    try:
        uniq = ul.extend_nodes(list(nodes), num_neg=num_neg)
    except AssertionError:
        uniq = ul.unique_nodes_batch
    return (list(uniq), np.array(ul.positive_pairs, np.int64), np.array(ul.negtive_pairs, np.int64),
            [len(v) for v in ul.node_negtive_pairs.values()], rng.getstate())


@pytest.mark.parametrize("name,n_train_frac,num_neg,B", [("pubmed", 0.5, 100, 512), ("cora", 0.5, 6, 300),
                                                         ("cora", 0.1, 100, 200), ("rmat", 0.9, 20, 700)])
def test_device_balls_match_host(name, n_train_frac, num_neg, B):
    G_ = _graph(name)
    rs = np.random.RandomState(7)
    train = rs.permutation(G_.n_nodes)[:int(G_.n_nodes * n_train_frac)]
    dev = U.UnsupervisedLoss(G_, train, torch.device("cuda", 0), n_threads=4, device_balls=True)
    host = U.UnsupervisedLoss(G_, train, "cpu", n_threads=4)
    assert dev.device_balls and not host.device_balls
    for b in range(3):
        nodes = rs.choice(train, min(B, len(train)), replace=b == 1)
        got = _outputs(dev, nodes, num_neg, 100 + b)
        want = _outputs(host, nodes, num_neg, 100 + b)
        assert got[0] == want[0]
        np.testing.assert_array_equal(got[1], want[1])
        np.testing.assert_array_equal(got[2], want[2])
        assert got[3] == want[3]
        np.testing.assert_array_equal(got[4][0], want[4][0])
        assert got[4][1] == want[4][1]


@pytest.mark.parametrize("parts", ["extend", "negatives"])
def test_device_balls_empty_batch_matches_host(parts):
    """An empty node list on the device path (no launch, no division by the
    empty word count) behaves as the host path: extend_nodes([]) reaches the
    models.py:147 assertion; get_negtive_nodes([]) returns no pairs; the
    stream is untouched either way."""
    G_ = _graph("pubmed")
    train = np.arange(0, G_.n_nodes, 2)
    dev = U.UnsupervisedLoss(G_, train, torch.device("cuda", 0), n_threads=4, device_balls=True)
    host = U.UnsupervisedLoss(G_, train, "cpu", n_threads=4)
    res = []
    for ul in (dev, host):
        rng = gs.RNG(5)
        ul.rng = rng
        if parts == "extend":
            with pytest.raises(AssertionError):
                ul.extend_nodes([], num_neg=100)
            res.append((list(ul.unique_nodes_batch), rng.getstate()))
        else:
            res.append((list(ul.get_negtive_nodes([], 100)), rng.getstate()))
    assert res[0][0] == res[1][0]
    np.testing.assert_array_equal(res[0][1][0], res[1][1][0])
    assert res[0][1][1] == res[1][1][1]
    # the device half still works after an empty batch
    nodes = train[:64]
    assert _outputs(dev, nodes, 100, 9)[0] == _outputs(host, nodes, 100, 9)[0]
