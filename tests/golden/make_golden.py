"""Capture golden vectors from the reference (Lolash/graphSAGE-pytorch).

Run ONLY in the build container, where the reference is mounted read-only at
/root/reference; the GPU box never sees it.  Outputs are small data files in
tests/golden/ (inputs + expected outputs); no reference source is copied.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is captured:
  rng.json       CPython `random` known answers: getrandbits, random.sample on
                 sequences of many sizes (list-pool and selected-set branches,
                 the n == k randbelow(1) quirk), random.choice.
  pyset.json     list(set.union(*[set(l) ...])) known answers.
  graphs.npz     Cora / Pubmed citation pairs (ids by first appearance in the
                 cites files, which is all the reference ships) + a tiny R-MAT
                 pair list, and each graph's adjacency as the reference holds
                 it (dataCenter.py:33-41 add order) in iteration order.
  sample_*.npz   GraphSage._get_unique_neighs_list (models.py:277-289) hop by
                 hop as GraphSage.forward calls it (models.py:246-251).
  forward_*.npz  GraphSage forward outputs and weight gradients
                 (models.py:241-330) for seeded weights and hashed features.
"""
import hashlib
import json
import os
import random
import sys
import warnings
from collections import defaultdict

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore", category=DeprecationWarning)
from src.models import GraphSage  # noqa: E402  (the reference itself)

sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
from tests.golden.synth import hashed_binary_features, uniform_features, tiny_rmat_pairs  # noqa: E402


def state_digest(r=random):
    st = r.getstate()
    return hashlib.sha256(json.dumps(list(st[1])).encode()).hexdigest()


def rng_kats():
    out = []
    for seed in [824, 0, 1, 7, 2 ** 40 + 5, -3, 123456789]:
        random.seed(seed)
        rec = {"seed": seed, "bits32": [random.getrandbits(32) for _ in range(8)]}
        rec["bits_k"] = [[k, random.getrandbits(k)] for k in (1, 5, 17, 31, 32)]
        samples = []
        for n, k in [(100, 5), (10, 10), (11, 10), (85, 10), (86, 10), (300, 10), (25, 25),
                     (277, 25), (278, 25), (70853, 25), (1, 1), (5, 0), (40, 3), (200, 100),
                     (1600, 100), (1600, 6)]:
            samples.append({"n": n, "k": k, "out": random.sample(range(n), k)})
        rec["samples"] = samples
        rec["choice"] = [[n, random.choice(range(n))] for n in (1, 2, 3, 17, 1000, 99991)]
        rec["randbelow"] = [[n, random._inst._randbelow(n)] for n in (1, 2, 3, 1000, 2 ** 31 - 1)]
        rec["state_after"] = [int(x) for x in random.getstate()[1]]
        out.append(rec)
    with open(os.path.join(OUT, "rng.json"), "w") as f:
        json.dump(out, f)


def pyset_kats():
    rng = np.random.RandomState(5)
    cases = []
    for t in range(120):
        nl = int(rng.randint(1, 40))
        hi = int(rng.choice([30, 1000, 70000, 2 ** 31 - 1]))
        lists = [[int(x) for x in rng.randint(0, hi, size=int(rng.randint(0, 30)))] for _ in range(nl)]
        lists[0] = lists[0] or [int(rng.randint(0, hi))]
        u = list(set.union(*[set(l) for l in lists]))
        cases.append({"lists": lists, "union": u})
    big = [int(x) for x in rng.randint(0, 10 ** 7, size=60000)]
    cases.append({"lists": [big[:30000], big[30000:]], "union": list(set.union(set(big[:30000]), set(big[30000:])))})
    with open(os.path.join(OUT, "pyset.json"), "w") as f:
        json.dump(cases, f)


def cora_pairs():
    ids, src, dst = {}, [], []
    with open(os.path.join(REF, "cora", "cora.cites")) as f:
        for line in f:
            a, b = line.strip().split()
            for x in (a, b):
                if x not in ids:
                    ids[x] = len(ids)
            src.append(ids[a])
            dst.append(ids[b])
    return np.array(src, np.int64), np.array(dst, np.int64), len(ids)


def pubmed_pairs():
    ids, src, dst = {}, [], []
    with open(os.path.join(REF, "pubmed-data", "Pubmed-Diabetes.DIRECTED.cites.tab")) as f:
        f.readline()
        f.readline()
        for line in f:
            info = line.strip().split("\t")
            a, b = info[1].split(":")[1], info[-1].split(":")[1]
            for x in (a, b):
                if x not in ids:
                    ids[x] = len(ids)
            src.append(ids[a])
            dst.append(ids[b])
    return np.array(src, np.int64), np.array(dst, np.int64), len(ids)


def ref_adjacency(src, dst):
    adj = defaultdict(set)
    for a, b in zip(src.tolist(), dst.tolist()):
        adj[a].add(b)
        adj[b].add(a)
    return adj


def adj_csr(adj, n):
    ptr = [0]
    col = []
    for v in range(n):
        col.extend(list(adj[v]))
        ptr.append(len(col))
    return np.array(ptr, np.int64), np.array(col, np.int32)


def capture_sampling(name, adj, n, seeds, batch_sizes, fanouts_list, gcn_list):
    """Hop-by-hop frontier lists / sampled sets, the reference's own calls."""
    gs = GraphSage(len(fanouts_list[0]), 8, 8, torch.zeros(n, 8), adj, "cpu")
    recs = {}
    for seed in seeds:
        perm = np.random.RandomState(seed).permutation(n)
        for B in batch_sizes:
            for fanouts in fanouts_list:
                roots = [int(x) for x in perm[:B]]
                random.seed(seed)
                frontier = list(roots)
                key = f"s{seed}_b{B}_f{'-'.join(map(str, fanouts))}"
                recs[key + "__roots"] = np.array(roots, np.int64)
                for j, k in enumerate(fanouts):
                    samp, d, uniq = gs._get_unique_neighs_list(frontier, num_sample=k)
                    assert all(d[x] == i for i, x in enumerate(uniq))
                    ptr = np.cumsum([0] + [len(s) for s in samp]).astype(np.int64)
                    items = np.array([x for s in samp for x in s], np.int64)
                    recs[f"{key}__h{j + 1}_set_ptr"] = ptr
                    recs[f"{key}__h{j + 1}_set_items"] = items
                    recs[f"{key}__h{j + 1}_union"] = np.array(uniq, np.int64)
                    frontier = uniq
                recs[key + "__state"] = np.array(random.getstate()[1], np.int64)
    np.savez_compressed(os.path.join(OUT, f"sample_{name}.npz"), **recs)


def capture_forward(name, adj, feats, n, seed, B, agg, gcn, num_layers=2):
    torch.manual_seed(seed)
    gs = GraphSage(num_layers, feats.shape[1], 128, feats, adj, "cpu", gcn=gcn, agg_func=agg)
    w = {k: v.detach().clone() for k, v in gs.state_dict().items()}
    roots = [int(x) for x in np.random.RandomState(seed + 1).permutation(n)[:B]]
    random.seed(seed)
    emb = gs(roots)
    g = torch.from_numpy(uniform_features(31, B, 128))  # fixed upstream gradient
    (emb * g).sum().backward()
    rec = {"roots": np.array(roots, np.int64), "emb": emb.detach().numpy(),
           "state": np.array(random.getstate()[1], np.int64)}
    for k, v in w.items():
        rec[f"w__{k}"] = v.numpy()
    for pname, p in gs.named_parameters():
        rec[f"grad__{pname}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, f"forward_{name}_{agg}_{'gcn' if gcn else 'sage'}.npz"), **rec)


def main():
    torch.set_num_threads(8)
    rng_kats()
    pyset_kats()
    cs, cd, cn = cora_pairs()
    ps, pd, pn = pubmed_pairs()
    rs, rd, rn = tiny_rmat_pairs()
    graphs = {}
    for nm, (s, d, n) in {"cora": (cs, cd, cn), "pubmed": (ps, pd, pn), "rmat": (rs, rd, rn)}.items():
        adj = ref_adjacency(s, d)
        ptr, col = adj_csr(adj, n)
        graphs.update({f"{nm}_src": s.astype(np.int32), f"{nm}_dst": d.astype(np.int32),
                       f"{nm}_n": np.array([n]), f"{nm}_row_ptr": ptr, f"{nm}_col": col})
    np.savez_compressed(os.path.join(OUT, "graphs.npz"), **graphs)

    cora = ref_adjacency(cs, cd)
    pub = ref_adjacency(ps, pd)
    rmat = ref_adjacency(rs, rd)
    capture_sampling("cora", cora, cn, [824, 1, 7], [20, 512, cn], [(10, 10)], [False])
    capture_sampling("pubmed", pub, pn, [824], [512], [(10, 10)], [False])
    capture_sampling("rmat", rmat, rn, [824, 3], [64, 256], [(25, 10), (10, 10), (5, 3, 2)], [False])

    cf = torch.from_numpy(hashed_binary_features(cn, 1433))
    for agg in ("MEAN", "MAX"):
        for gcn in (False, True):
            capture_forward("cora", cora, cf, cn, 824, 20, agg, gcn)
    rf = torch.from_numpy(uniform_features(77, rn, 100))
    for agg in ("MEAN", "MAX"):
        capture_forward("rmat", rmat, rf, rn, 5, 48, agg, False)
    pf = torch.from_numpy(uniform_features(11, pn, 64))
    capture_forward("pubmed", pub, pf, pn, 824, 64, "MEAN", False)
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
