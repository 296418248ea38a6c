"""UnsupervisedLoss drop-in (graphsage-pytorch_amd/unsup.py) against vectors
captured from the reference (tests/golden/make_golden_unsup.py):

* extend_nodes (models.py:135-186) — host code, bit-exact: unique list, pair
  lists, per-node dicts, and the global `random` state afterwards;
* get_loss_sage / get_loss_margin (models.py:65-132) — HIP kernels (GPU),
  loss and embedding gradient within 1e-5 of the reference's autograd.
"""
import importlib
import random

import numpy as np
import pytest
import torch

from tests import unsup_cases as C

U = importlib.import_module("graphsage-pytorch_amd.unsup")
gs = importlib.import_module("graphsage-pytorch_amd")


def _graph(name):
    g = C.graphs()
    return gs.CSRGraph.from_pairs(g[f"{name}_src"].astype(np.int64), g[f"{name}_dst"].astype(np.int64),
                                  int(g[f"{name}_n"][0]))


def _check(ul, uniq, b):
    assert uniq == b["unique"].tolist()
    assert np.array_equal(np.array(ul.positive_pairs, np.int64).reshape(-1, 2), b["pos"])
    assert np.array_equal(np.array(ul.negtive_pairs, np.int64).reshape(-1, 2), b["neg"])
    assert list(ul.node_positive_pairs) == b["pos_keys"].tolist()
    assert [len(v) for v in ul.node_positive_pairs.values()] == b["pos_cnt"].tolist()
    assert list(ul.node_negtive_pairs) == b["neg_keys"].tolist()
    assert [len(v) for v in ul.node_negtive_pairs.values()] == b["neg_cnt"].tolist()
    assert list(random.getstate()[1]) == b["state"].tolist()


def _replay(tag, threads=4):
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case(tag)
    ul = U.UnsupervisedLoss(_graph(name), train, "cpu", n_threads=threads)
    random.seed(seed)
    for b in batches:
        if int(b["error"]):
            with pytest.raises(AssertionError):
                ul.extend_nodes(b["nodes"], num_neg=num_neg)
            uniq = ul.unique_nodes_batch
        else:
            uniq = ul.extend_nodes(b["nodes"], num_neg=num_neg)
        _check(ul, uniq, b)
    return ul


@pytest.mark.parametrize("tag", C.extend_tags())
def test_extend_nodes_matches_reference(tag):
    _replay(tag)


def test_device_balls_default_rule():
    # host BFS below DEVICE_BALLS_MIN_NODES ids (Cora), device balls above (Pubmed), never on CPU
    m = U.DEVICE_BALLS_MIN_NODES
    assert not U.device_balls_default("cpu", 10 * m)
    assert not U.device_balls_default(torch.device("cuda", 0), 2708)
    assert U.device_balls_default(torch.device("cuda", 0), 19717)
    assert U.device_balls_default("cuda", m) and not U.device_balls_default("cuda", m - 1)
    assert not U.UnsupervisedLoss(_graph("cora"), np.arange(100), "cpu").device_balls


def test_extend_nodes_thread_count_invariant():
    for t in (1, 3, 8):
        _replay("cora_n100", threads=t)


def test_extend_nodes_from_dict_of_sets():
    """The drop-in path: the reference's own dict-of-sets adjacency adopted."""
    from collections import defaultdict
    g = C.graphs()
    adj = defaultdict(set)
    for a, b in zip(g["cora_src"].tolist(), g["cora_dst"].tolist()):
        adj[a].add(b)
        adj[b].add(a)
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case("cora_n6")
    ul = U.UnsupervisedLoss(adj, train, "cpu")
    random.seed(seed)
    for b in batches:
        _check(ul, ul.extend_nodes(b["nodes"], num_neg=num_neg), b)


def test_walks_and_negatives_separately():
    """get_positive_nodes then get_negtive_nodes == extend_nodes' pair lists."""
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case("cora_n6")
    ul = U.UnsupervisedLoss(_graph(name), train, "cpu")
    b = batches[0]
    random.seed(seed)
    ul.get_positive_nodes(b["nodes"])
    ul.get_negtive_nodes(b["nodes"], num_neg)
    assert np.array_equal(np.array(ul.positive_pairs).reshape(-1, 2), b["pos"])
    assert np.array_equal(np.array(ul.negtive_pairs).reshape(-1, 2), b["neg"])
    assert list(random.getstate()[1]) == b["state"].tolist()


def test_extend_errors():
    name, train, _, batches = C.extend_case("cora_n6")
    ul = U.UnsupervisedLoss(_graph(name), train, "cpu")
    with pytest.raises(IndexError):
        ul.extend_nodes(np.array([10 ** 6]), num_neg=6)
    with pytest.raises(ValueError):
        ul.extend_nodes(batches[0]["nodes"], num_neg=-1)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", C.loss_tags())
@pytest.mark.parametrize("kind", ["sage", "margin"])
def test_unsup_losses_match_reference(tag, kind):
    E = C.extend_file()
    ul = _replay(tag)
    dev = torch.device("cuda", 0)
    emb = torch.tensor(E[f"{tag}__emb"], device=dev, requires_grad=True)
    nodes = np.asarray(ul.unique_nodes_batch)
    loss = (ul.get_loss_sage if kind == "sage" else ul.get_loss_margin)(emb, nodes)
    assert loss.shape == (() if kind == "sage" else (1,))
    loss.sum().backward()
    ref = float(E[f"{tag}__{kind}_loss"])
    assert abs(float(loss.detach().reshape(-1)[0]) - ref) <= 1e-5 * max(1.0, abs(ref))
    torch.testing.assert_close(emb.grad.cpu(), torch.from_numpy(E[f"{tag}__{kind}_grad"]), atol=1e-6, rtol=1e-5)


@pytest.mark.gpu
def test_unsup_loss_deterministic_and_scaled():
    E = C.extend_file()
    tag = C.loss_tags()[0]
    ul = _replay(tag)
    dev = torch.device("cuda", 0)
    nodes = np.asarray(ul.unique_nodes_batch)
    grads = []
    for scale in (1.0, 1.0, 2.5):
        emb = torch.tensor(E[f"{tag}__emb"], device=dev, requires_grad=True)
        (ul.get_loss_sage(emb, nodes) * scale).backward()
        grads.append(emb.grad.clone())
    assert torch.equal(grads[0], grads[1])
    torch.testing.assert_close(grads[2], grads[0] * 2.5, rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_unsup_loss_zero_embedding_row():
    """A dead (all-zero) embedding row: cosine's eps clamp, like torch."""
    E = C.extend_file()
    tag = C.loss_tags()[0]
    ul = _replay(tag)
    dev = torch.device("cuda", 0)
    base = torch.tensor(E[f"{tag}__emb"])
    base[3] = 0
    nodes = np.asarray(ul.unique_nodes_batch)
    import oracle.unsup_semantics as O
    st = O.UnsupState(None, [])
    st.unique_nodes_batch = ul.unique_nodes_batch
    st.node_positive_pairs, st.node_negtive_pairs = ul.node_positive_pairs, ul.node_negtive_pairs
    for kind in ("sage", "margin"):
        ref_e = base.clone().requires_grad_(True)
        O.unsup_loss(st, ref_e, kind).backward()
        emb = base.to(dev).requires_grad_(True)
        (ul.get_loss_sage if kind == "sage" else ul.get_loss_margin)(emb, nodes).sum().backward()
        got, ref = emb.grad.cpu(), ref_e.grad
        keep = torch.ones(len(ref), dtype=torch.bool)
        keep[3] = False
        torch.testing.assert_close(got[keep], ref[keep], atol=1e-5, rtol=1e-5)
        # the dead row's gradient is a sum of terms scaled by 1/eps = 1e8 that
        # largely cancel: fp32 rounding of that sum, not a formula difference
        torch.testing.assert_close(got[3], ref[3], atol=1e-2, rtol=1e-3)
