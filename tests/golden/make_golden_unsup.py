"""Capture golden vectors for the reference's unsupervised-loss path and its
batch loop (Lolash/graphSAGE-pytorch):

  UnsupervisedLoss.extend_nodes      models.py:135-147 (random walks :166-186,
                                     5-hop negatives :152-164)
  get_loss_sage / get_loss_margin    models.py:65-132
  apply_model (sup / plus_unsup / unsup, 'normal' / 'margin')  utils.py:113-193

Run ONLY in the build container (the reference is mounted read-only at
/root/reference; the GPU box never sees it).  Writes small data files under
tests/golden/ (inputs + expected outputs); no reference source is copied.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_unsup.py
"""
import os
import random
import sys
import types
import warnings
from collections import defaultdict

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore", category=DeprecationWarning)
from src.models import Classification, GraphSage, UnsupervisedLoss  # noqa: E402  (the reference)
from src.utils import apply_model  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
from tests.golden.synth import hashed_binary_features, tiny_rmat_pairs, uniform_features  # noqa: E402
from tests.golden.make_golden import cora_pairs, pubmed_pairs  # noqa: E402


def adjacency(src, dst):
    adj = defaultdict(set)
    for a, b in zip(src.tolist(), dst.tolist()):
        adj[a].add(b)
        adj[b].add(a)
    return adj


def split(n, seed=824):
    """dataCenter.py:100-111 after np.random.seed(seed) (main.py:41)."""
    np.random.seed(seed)
    perm = np.random.permutation(n)
    t, v = n // 3, n // 6
    return perm[:t], perm[t:t + v], perm[t + v:]


def pairs_arr(pairs):
    return np.array(pairs, np.int64).reshape(-1, 2)


def capture_extend(rec, tag, adj, n, train, b_sz, num_neg, n_batches, seed):
    random.seed(seed)
    ul = UnsupervisedLoss(adj, train, "cpu")
    order = np.random.RandomState(seed + 9).permutation(train)
    rec[f"{tag}__train"] = np.asarray(train, np.int64)
    rec[f"{tag}__meta"] = np.array([b_sz, num_neg, n_batches, seed], np.int64)
    for b in range(n_batches):
        nodes = order[b * b_sz:(b + 1) * b_sz]
        k = f"{tag}__b{b}"
        try:
            uniq = ul.extend_nodes(nodes, num_neg=num_neg)
            rec[k + "_error"] = np.array(0)
        except AssertionError:  # models.py:147 `set(target) < set(unique)` can fail
            uniq = ul.unique_nodes_batch
            rec[k + "_error"] = np.array(1)
        rec[k + "_nodes"] = np.asarray(nodes, np.int64)
        rec[k + "_unique"] = np.array([int(x) for x in uniq], np.int64)
        rec[k + "_pos"] = pairs_arr(ul.positive_pairs)
        rec[k + "_neg"] = pairs_arr(ul.negtive_pairs)
        rec[k + "_pos_keys"] = np.array([int(x) for x in ul.node_positive_pairs], np.int64)
        rec[k + "_pos_cnt"] = np.array([len(v) for v in ul.node_positive_pairs.values()], np.int64)
        rec[k + "_neg_keys"] = np.array([int(x) for x in ul.node_negtive_pairs], np.int64)
        rec[k + "_neg_cnt"] = np.array([len(v) for v in ul.node_negtive_pairs.values()], np.int64)
        rec[k + "_state"] = np.array(random.getstate()[1], np.int64)
    return ul


def capture_losses(rec, tag, ul, D=128):
    uniq = ul.unique_nodes_batch
    nodes = np.asarray(list(uniq))
    base = torch.from_numpy(uniform_features(41, len(uniq), D))
    for name in ("sage", "margin"):
        E = base.clone().requires_grad_(True)
        fn = ul.get_loss_sage if name == "sage" else ul.get_loss_margin
        loss = fn(E, nodes)
        loss.sum().backward()
        rec[f"{tag}__{name}_loss"] = np.array(float(loss.detach().reshape(-1)[0]), np.float64)
        rec[f"{tag}__{name}_grad"] = E.grad.numpy()
    rec[f"{tag}__emb"] = base.numpy()


def capture_apply_model(rec, tag, src, dst, n, feats, n_classes, n_train, b_sz, learn_method, unsup_loss,
                        agg="MEAN", gcn=False, seed=824):
    adj = adjacency(src, dst)
    test, val, train = split(n, seed)
    train = train[:n_train]
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    labels = (np.arange(n) % n_classes).astype(np.int64)
    dc = types.SimpleNamespace(g_test=test, g_val=val, g_train=train, g_labels=labels)
    gsage = GraphSage(2, feats.shape[1], 128, feats, adj, "cpu", gcn=gcn, agg_func=agg)
    cls = Classification(128, n_classes)
    init = {**{f"gs.{k}": v.detach().clone() for k, v in gsage.state_dict().items()},
            **{f"cls.{k}": v.detach().clone() for k, v in cls.state_dict().items()}}
    ul = UnsupervisedLoss(adj, train, "cpu")
    apply_model(dc, "g", gsage, cls, ul, b_sz, unsup_loss, "cpu", learn_method)
    rec[f"{tag}__meta"] = np.array([n_train, b_sz, seed, n_classes], np.int64)
    final = {**{f"gs.{k}": v.detach() for k, v in gsage.state_dict().items()},
             **{f"cls.{k}": v.detach() for k, v in cls.state_dict().items()}}
    pick = np.random.RandomState(99)
    for k in init:
        a, b = init[k].numpy(), final[k].numpy()
        if a.size > 65536:  # sage_layer1 [128, 2F]: a fixed random subset + checksums (fixture size)
            idx = np.sort(pick.choice(a.size, 16384, replace=False))
            rec[f"{tag}__sub__{k}"] = idx
            a, b = a.reshape(-1)[idx], b.reshape(-1)[idx]
            rec[f"{tag}__sum__{k}"] = np.array([final[k].double().sum().item(), final[k].double().abs().sum().item(),
                                                init[k].double().sum().item()])
        rec[f"{tag}__init__{k}"] = a
        rec[f"{tag}__final__{k}"] = b
    rec[f"{tag}__state"] = np.array(random.getstate()[1], np.int64)


def main():
    torch.set_num_threads(8)
    cs, cd, cn = cora_pairs()
    ps, pd, pn = pubmed_pairs()
    rs, rd, rn = tiny_rmat_pairs()

    rec = {}
    cora = adjacency(cs, cd)
    _, _, ctrain = split(cn)
    capture_extend(rec, "cora_n100", cora, cn, ctrain, 20, 100, 3, 824)
    ul = capture_extend(rec, "cora_n6", cora, cn, ctrain, 20, 6, 3, 7)
    capture_losses(rec, "cora_n6", ul)
    ul = capture_extend(rec, "cora_n100_b64", cora, cn, ctrain, 64, 100, 1, 1)
    capture_losses(rec, "cora_n100_b64", ul)
    rmat = adjacency(rs, rd)
    _, _, rtrain = split(rn)
    capture_extend(rec, "rmat_n6", rmat, rn, rtrain, 32, 6, 3, 824)
    capture_extend(rec, "rmat_n100", rmat, rn, rtrain, 32, 100, 2, 3)
    pub = adjacency(ps, pd)
    _, _, ptrain = split(pn)
    capture_extend(rec, "pubmed_n100", pub, pn, ptrain, 512, 100, 1, 824)
    capture_extend(rec, "pubmed_n6", pub, pn, ptrain, 64, 6, 2, 5)
    np.savez_compressed(os.path.join(OUT, "unsup_extend.npz"), **rec)

    rec = {}
    cf = torch.from_numpy(hashed_binary_features(cn, 1433))
    for lm, ulo in [("sup", "normal"), ("plus_unsup", "normal"), ("unsup", "margin"), ("plus_unsup", "margin")]:
        capture_apply_model(rec, f"cora_{lm}_{ulo}", cs, cd, cn, cf, 7, cn, 300, lm, ulo)
    capture_apply_model(rec, "cora_sup_normal_max", cs, cd, cn, cf, 7, 400, 100, "sup", "normal", agg="MAX")
    np.savez_compressed(os.path.join(OUT, "unsup_apply_model.npz"), **rec)
    print("golden vectors written to", OUT)


if __name__ == "__main__":
    main()
