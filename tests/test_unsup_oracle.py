"""Pin the unsupervised-path oracle (oracle/unsup_semantics.py) against vectors
captured from the reference's UnsupervisedLoss (models.py:45-186)."""
import random

import numpy as np
import pytest
import torch

from oracle import Adjacency
from oracle import unsup_semantics as U
from tests import unsup_cases as C


def _adj(name):
    g = C.graphs()
    return Adjacency(g[f"{name}_src"], g[f"{name}_dst"], int(g[f"{name}_n"][0]))


def _check_batch(st, got_unique, b):
    assert got_unique == b["unique"].tolist()
    assert np.array_equal(np.array(st.positive_pairs, np.int64).reshape(-1, 2), b["pos"])
    assert np.array_equal(np.array(st.negtive_pairs, np.int64).reshape(-1, 2), b["neg"])
    assert list(st.node_positive_pairs) == b["pos_keys"].tolist()
    assert [len(v) for v in st.node_positive_pairs.values()] == b["pos_cnt"].tolist()
    assert list(st.node_negtive_pairs) == b["neg_keys"].tolist()
    assert [len(v) for v in st.node_negtive_pairs.values()] == b["neg_cnt"].tolist()
    assert list(random.getstate()[1]) == b["state"].tolist()


@pytest.mark.parametrize("tag", [t for t in C.extend_tags() if not t.startswith("pubmed")])
def test_oracle_extend_nodes_matches_reference(tag):
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case(tag)
    st = U.UnsupState(_adj(name), train)
    random.seed(seed)
    for b in batches:
        uniq, ok = U.extend_nodes(st, b["nodes"], num_neg)
        assert ok == (not int(b["error"]))
        _check_batch(st, uniq, b)


@pytest.mark.parametrize("tag", C.loss_tags())
def test_oracle_unsup_losses_match_reference(tag):
    name, train, (b_sz, num_neg, nb, seed), batches = C.extend_case(tag)
    E = C.extend_file()
    st = U.UnsupState(_adj(name), train)
    random.seed(seed)
    for b in batches:
        U.extend_nodes(st, b["nodes"], num_neg)
    for kind in ("sage", "margin"):
        emb = torch.tensor(E[f"{tag}__emb"], requires_grad=True)
        loss = U.unsup_loss(st, emb, kind)
        loss.backward()
        assert abs(float(loss) - float(E[f"{tag}__{kind}_loss"])) <= 1e-5 * max(1.0, abs(float(loss)))
        torch.testing.assert_close(emb.grad, torch.from_numpy(E[f"{tag}__{kind}_grad"]), atol=1e-6, rtol=1e-5)
