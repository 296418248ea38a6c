"""Shared readers for tests/golden/unsup_*.npz (captured from the reference by
tests/golden/make_golden_unsup.py)."""
import os

import numpy as np

G = os.path.join(os.path.dirname(__file__), "golden")
GRAPH_OF = {"cora": "cora", "rmat": "rmat", "pubmed": "pubmed"}


def extend_file():
    return np.load(os.path.join(G, "unsup_extend.npz"))


def apply_file():
    return np.load(os.path.join(G, "unsup_apply_model.npz"))


def graphs():
    return np.load(os.path.join(G, "graphs.npz"))


def extend_tags():
    E = extend_file()
    return sorted({k.split("__")[0] for k in E.files})


def extend_case(tag):
    """(graph name, train, meta(b_sz, num_neg, n_batches, seed), [batch dicts])."""
    E = extend_file()
    b_sz, num_neg, n_batches, seed = (int(x) for x in E[f"{tag}__meta"])
    batches = []
    for b in range(n_batches):
        k = f"{tag}__b{b}"
        batches.append({f: E[f"{k}_{f}"] for f in ("nodes", "unique", "pos", "neg", "pos_keys", "pos_cnt",
                                                  "neg_keys", "neg_cnt", "state", "error")})
    return tag.split("_")[0], E[f"{tag}__train"], (b_sz, num_neg, n_batches, seed), batches


def loss_tags():
    E = extend_file()
    return sorted({k.split("__")[0] for k in E.files if k.endswith("__sage_loss")})


def apply_tags():
    A = apply_file()
    return sorted({k.split("__")[0] for k in A.files})
