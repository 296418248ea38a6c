"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the reference algorithm, written from its behaviour:

* adjacency  : dict of Python int sets filled by add() in pair order
               (dataCenter.py:33-41, :77-86).  Built lazily per node from the
               insertion lists so large synthetic graphs need not be expanded
               into sets up front — replaying a row's adds in order yields the
               identical set object layout.
* sampling   : per frontier node, random.sample(tuple(row_set), k) when the
               row has >= k members, else the row set itself; each result is
               unioned with {node}; the next frontier is the union of those
               sets in CPython iteration order (models.py:277-289), applied
               hop by hop (models.py:246-251).  The CPython builtins `random`
               and `set` are used as-is: they *define* these semantics.
* aggregation: the dense 0/1 mask formulation — MEAN = (mask / rowsum) @ X,
               MAX = per-row max over the masked rows (models.py:291-330).
* layer      : relu(W @ cat([self, agg], 1).T).T (models.py:209-220).
* train step : log_softmax(Linear) + NLL mean, backward, clip_grad_norm_(5)
               per model, SGD(lr) (utils.py:136-191, models.py:8-27).
"""
import random

import numpy as np
import torch
import torch.nn.functional as F


class Adjacency:
    """Lazily materialised dict-of-sets adjacency (dataCenter.py:33-41)."""

    def __init__(self, src, dst, n_nodes, sort_device=None):
        """sort_device: optionally a torch device for the one stable sort of
        the insertion list by endpoint (a generic library sort; at the 16M-node
        / 160M-pair size numpy's stable sort of 320M keys takes minutes)."""
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int64)
        self.n_nodes = int(n_nodes)
        small = self.n_nodes < (1 << 31)
        kt = np.int32 if small else np.int64
        ends = np.empty(2 * len(src), kt)   # adds in order: adj[a].add(b); adj[b].add(a)
        other = np.empty(2 * len(src), kt)
        ends[0::2], other[0::2] = src, dst
        ends[1::2], other[1::2] = dst, src
        if sort_device is None:
            order = np.argsort(ends, kind="stable")
        else:
            keys = torch.from_numpy(ends).to(sort_device)
            order = torch.sort(keys, stable=True)[1].cpu().numpy()
            del keys
        self._ins = other[order]
        del order
        self._ptr = np.zeros(self.n_nodes + 1, np.int64)
        self._ptr[1:] = np.cumsum(np.bincount(ends, minlength=self.n_nodes))
        self._sets = {}

    def __getitem__(self, v):
        v = int(v)
        s = self._sets.get(v)
        if s is None:
            s = set()
            for x in self._ins[self._ptr[v]:self._ptr[v + 1]].tolist():
                s.add(x)
            self._sets[v] = s
        return s

    def __len__(self):
        return self.n_nodes


def sample_hop(adj, nodes, num_sample=10, rng=random):
    """One call of _get_unique_neighs_list: (sampled sets, {id: pos}, union list)."""
    sampled = []
    for v in nodes:
        row = adj[int(v)]
        if num_sample is not None and len(row) >= num_sample:
            chosen = set(rng.sample(tuple(row), num_sample))
        else:
            chosen = row
        sampled.append(chosen | {v})
    union = list(set.union(*sampled))
    return sampled, {x: i for i, x in enumerate(union)}, union


def sample_layers(adj, roots, fanouts, rng=random):
    """Hops from the roots; returns [(frontier, sampled_sets, index, union), ...]."""
    frontier = list(roots)
    hops = []
    for k in fanouts:
        samp, index, union = sample_hop(adj, frontier, k, rng)
        hops.append((frontier, samp, index, union))
        frontier = union
    return hops


def _dense_aggregate(dst_nodes, samp, index, union, X, agg, gcn):
    if not gcn:
        samp = [s - {dst_nodes[i]} for i, s in enumerate(samp)]
    emb = X if len(X) == len(index) else X[torch.as_tensor(union, dtype=torch.long)]
    rows = [i for i, s in enumerate(samp) for _ in s]
    cols = [index[n] for s in samp for n in s]
    mask = torch.zeros(len(samp), len(index))
    mask[rows, cols] = 1
    if agg == "MEAN":
        return (mask / mask.sum(1, keepdim=True)).mm(emb)
    if agg == "MAX":
        out = []
        for r in (mask == 1):
            sel = emb[r.nonzero().squeeze(1)]
            out.append(sel.max(0)[0].view(1, -1))
        return torch.cat(out, 0)
    raise ValueError(agg)


def _bf16_value(t):
    """t rounded to bf16 (round-to-nearest-even) in value only: the gradient
    passes straight through to t (the fp32 master copy a bf16 GEMM reads)."""
    return t + (t.detach().to(torch.bfloat16).float() - t.detach())


def forward_dense(hops, X, weights, agg="MEAN", gcn=False, bf16_layer1=False):
    """Bottom-up forward over sample_layers() output (models.py:255-267).

    bf16_layer1 (BASELINE configs[3], not a reference mode): X holds
    bf16-representable values; layer 1's aggregate and weight enter its GEMM
    rounded to bf16 (fp32 accumulate), as the HIP path computes with a bf16
    feature table — the reference algorithm on bf16 inputs."""
    L = len(hops)
    h = X
    for layer in range(1, L + 1):
        frontier, samp, index, union = hops[L - layer]
        a = _dense_aggregate(frontier, samp, index, union, h, agg, gcn)
        w = weights[layer - 1]
        if bf16_layer1 and layer == 1:
            a, w = _bf16_value(a), _bf16_value(w)
        if layer == 1:
            self_rows = h[torch.as_tensor(list(frontier), dtype=torch.long)]
        else:
            # _nodes_map (models.py:271-275): rows of the previous hidden state
            self_rows = h[torch.as_tensor([index[x] for x in frontier], dtype=torch.long)]
        combined = a if gcn else torch.cat([self_rows, a], 1)
        h = F.relu(w.mm(combined.t())).t()
    return h


def nll_loss(logp, labels):
    return -torch.sum(logp[range(logp.size(0)), labels], 0) / logp.size(0)


def train_step_dense(adj, roots, fanouts, X, weights, cls_w, cls_b, labels, agg="MEAN", gcn=False,
                     lr=0.7, max_norm=5.0, rng=random, bf16_layer1=False, capture=None):
    """One supervised step of utils.py:144-191 (without extend_nodes).
    capture (a dict, optional): receives the step's root embeddings ("emb")
    and its flat gradient [W1 | ... | WL | cls_w | cls_b] before the clip
    ("grads"), the layout of the native trainer's flat buffer."""
    hops = sample_layers(adj, roots, fanouts, rng)
    emb = forward_dense(hops, X, weights, agg, gcn, bf16_layer1)
    logp = torch.log_softmax(emb.mm(cls_w.t()) + cls_b, 1)
    loss = nll_loss(logp, labels)
    loss.backward()
    if capture is not None:
        capture["emb"] = emb.detach().clone()
        capture["grads"] = torch.cat([p.grad.detach().reshape(-1) for p in list(weights) + [cls_w, cls_b]])
    with torch.no_grad():
        for group in (list(weights), [cls_w, cls_b]):
            torch.nn.utils.clip_grad_norm_(group, max_norm)
        for p in list(weights) + [cls_w, cls_b]:
            p.add_(p.grad, alpha=-lr)
            p.grad = None
    return float(loss.detach())
