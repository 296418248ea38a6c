"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the reference's unsupervised-loss path, written from its
behaviour (Lolash/graphSAGE-pytorch src/models.py):

* positives  (models.py:166-186): per batch node with a non-empty adjacency
  set, N_WALKS walks of WALK_LEN steps; each step is random.choice over
  list(adj[cur]) (set iteration order); a visited node other than the start
  that is a training node gives the pair (node, visited).
* negatives  (models.py:152-164): per batch node, the N_WALK_LEN-hop ball
  (frontier expansion by set union); far = set(train) - ball, and
  random.sample(far, num_neg) (its population is tuple(far), i.e. far's
  iteration order) unless num_neg >= len(far), which keeps all of far.
* extend     (models.py:135-147): list(set(flat positives) | set(flat
  negatives)); `set(target) < set(unique)` must hold.
* losses     (models.py:65-132): per node that has both positive and
  negative pairs, cosine similarities of its pairs' embedding rows;
  'sage'   : mean(-log σ(cos⁺)) - Q·mean(log σ(-cos⁻)), averaged over nodes;
  'margin' : max(0, max log σ(cos⁻) - min log σ(cos⁺) + MARGIN), averaged.
The CPython builtins `random` and `set` are used as-is: they define the
sample order.  Pinned by tests/golden/unsup_*.npz (tests/golden/make_golden_unsup.py).
"""
import random

import torch
import torch.nn.functional as F

N_WALKS, WALK_LEN, N_WALK_LEN, Q, MARGIN = 6, 1, 5, 10, 3


class UnsupState:
    """The attributes extend_nodes fills (models.py:47-56)."""

    def __init__(self, adj, train_nodes):
        self.adj = adj
        self.train = train_nodes
        self.train_set = set(int(x) for x in train_nodes)
        self.positive_pairs, self.negtive_pairs = [], []
        self.node_positive_pairs, self.node_negtive_pairs = {}, {}
        self.unique_nodes_batch = []


def _walk_pairs(st, nodes, rng):
    for v in nodes:
        v = int(v)
        if not st.adj[v]:
            continue
        mine = []
        for _ in range(N_WALKS):
            cur = v
            for _ in range(WALK_LEN):
                nxt = rng.choice(list(st.adj[cur]))
                if nxt != v and nxt in st.train_set:
                    mine.append((v, nxt))
                cur = nxt
        st.positive_pairs.extend(mine)
        st.node_positive_pairs[v] = mine


def _ball(adj, v, hops):
    seen, edge = {v}, {v}
    for _ in range(hops):
        reach = set()
        for u in edge:
            reach |= adj[int(u)]
        edge = reach - seen
        seen |= reach
    return seen


def _negative_pairs(st, nodes, num_neg, rng):
    train_set = set(st.train)  # the reference rebuilds it from the array each node
    for v in nodes:
        v = int(v)
        far = train_set - _ball(st.adj, v, N_WALK_LEN)
        picked = rng.sample(tuple(far), num_neg) if num_neg < len(far) else far
        mine = [(v, int(x)) for x in picked]
        st.negtive_pairs.extend(mine)
        st.node_negtive_pairs[v] = mine


def extend_nodes(st, nodes, num_neg=6, rng=random):
    st.positive_pairs, st.negtive_pairs = [], []
    st.node_positive_pairs, st.node_negtive_pairs = {}, {}
    _walk_pairs(st, nodes, rng)
    _negative_pairs(st, nodes, num_neg, rng)
    pos_ids = set(x for p in st.positive_pairs for x in p)
    neg_ids = set(x for p in st.negtive_pairs for x in p)
    st.unique_nodes_batch = [int(x) for x in (pos_ids | neg_ids)]
    ok = set(int(x) for x in nodes) < set(st.unique_nodes_batch)
    return st.unique_nodes_batch, ok


def _pair_cos(emb, where, pairs):
    a = emb[[where[p[0]] for p in pairs]]
    b = emb[[where[p[1]] for p in pairs]]
    return F.cosine_similarity(a, b)


def unsup_loss(st, emb, kind="sage"):
    where = {x: i for i, x in enumerate(st.unique_nodes_batch)}
    scores = []
    for v, pos in st.node_positive_pairs.items():
        neg = st.node_negtive_pairs[v]
        if not pos or not neg:
            continue
        cp, cn = _pair_cos(emb, where, pos), _pair_cos(emb, where, neg)
        if kind == "sage":
            s = -torch.log(torch.sigmoid(cp)).mean() - Q * torch.log(torch.sigmoid(-cn)).mean()
        else:
            s = torch.clamp(torch.log(torch.sigmoid(cn)).max() - torch.log(torch.sigmoid(cp)).min() + MARGIN, min=0)
        scores.append(s)
    return torch.stack(scores).mean()
