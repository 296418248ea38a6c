"""Capture golden vectors for the reference's evaluation / inference helpers
(Lolash/graphSAGE-pytorch src/utils.py):

  evaluate              utils.py:13-57   (val F1, test F1 when improved, RNG use)
  get_gnn_embeddings    utils.py:59-78   (every node, batches of 500, id order)
  train_classification  utils.py:80-111  (classifier SGD on frozen embeddings,
                                          evaluate() after every epoch)

Inputs: the Cora citation graph (pairs from tests/golden/graphs.npz, which
make_golden.py took from the reference's cites file), 64-d hashed U(-1,1)
features, labels id % 7, the dataCenter.py:100-111 split under seed 824.  The
models are the reference's own GraphSage / Classification after one
apply_model epoch (utils.py:113-193); their weights are stored as inputs, so
the test loads them instead of retraining.

Run ONLY in the build container (the reference is mounted read-only at
/root/reference; the GPU box never sees it):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_eval.py
"""
import contextlib
import io
import os
import random
import sys
import tempfile
import types
import warnings

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
sys.path.insert(0, REF)
warnings.filterwarnings("ignore", category=DeprecationWarning)
from src.models import Classification, GraphSage, UnsupervisedLoss  # noqa: E402  (the reference)
from src.utils import apply_model, evaluate, get_gnn_embeddings, train_classification  # noqa: E402

sys.path.insert(0, ROOT)
from tests.golden.make_golden_unsup import adjacency, split  # noqa: E402
from tests.golden.synth import uniform_features  # noqa: E402

F, H, C, SEED = 64, 128, 7, 824


def printed_f1(text, what):
    return [float(l.split(":")[1]) for l in text.splitlines() if l.startswith(what)]


def main():
    torch.set_num_threads(8)
    g = np.load(os.path.join(OUT, "graphs.npz"))
    src, dst, n = g["cora_src"], g["cora_dst"], int(g["cora_n"][0])
    adj = adjacency(src, dst)
    test, val, train = split(n, SEED)
    labels = (np.arange(n) % C).astype(np.int64)
    dc = types.SimpleNamespace(g_test=test, g_val=val, g_train=train, g_labels=labels)
    feats = torch.from_numpy(uniform_features(11, n, F))

    random.seed(SEED)
    np.random.seed(SEED)
    torch.manual_seed(SEED)
    gsage = GraphSage(2, F, H, feats, adj, "cpu", agg_func="MEAN")
    cls = Classification(H, C)
    ul = UnsupervisedLoss(adj, train, "cpu")
    with contextlib.redirect_stdout(io.StringIO()):
        apply_model(dc, "g", gsage, cls, ul, 300, "normal", "cpu", "sup")

    rec = {"meta": np.array([n, F, H, C, SEED], np.int64), "feat_seed": np.array(11)}
    for k, v in gsage.state_dict().items():
        rec[f"w__gs.{k}"] = v.numpy().copy()
    for k, v in cls.state_dict().items():
        rec[f"w__cls.{k}"] = v.numpy().copy()

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        os.makedirs("models")
        try:
            # evaluate: improved (max_vali_f1 = 0) then not improved (= 1.0)
            random.seed(5)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                m = evaluate(dc, "g", gsage, cls, "cpu", 0.0, "golden", 0)
            rec["eval_improved__max"] = np.array(m)
            rec["eval_improved__val_f1"] = np.array(printed_f1(buf.getvalue(), "Validation F1"))
            rec["eval_improved__test_f1"] = np.array(printed_f1(buf.getvalue(), "Test F1"))
            rec["eval_improved__state"] = np.array(random.getstate()[1], np.int64)
            rec["eval_improved__saved"] = np.array(len(os.listdir("models")))
            random.seed(5)
            with torch.no_grad():
                rec["eval__val_logits"] = cls(gsage(val)).numpy()
            random.seed(6)
            with contextlib.redirect_stdout(io.StringIO()):
                m = evaluate(dc, "g", gsage, cls, "cpu", 1.0, "golden", 1)
            rec["eval_kept__max"] = np.array(m)
            rec["eval_kept__state"] = np.array(random.getstate()[1], np.int64)

            # get_gnn_embeddings: every node, batches of 500
            random.seed(7)
            with contextlib.redirect_stdout(io.StringIO()):
                E = get_gnn_embeddings(gsage, dc, "g").numpy()
            rows = np.arange(0, n, 9)
            rec["embed__rows"] = rows
            rec["embed__emb"] = E[rows]
            rec["embed__rowsum"] = E.astype(np.float64).sum(1)
            rec["embed__state"] = np.array(random.getstate()[1], np.int64)

            # train_classification: 2 epochs on the frozen embeddings
            random.seed(8)
            np.random.seed(8)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                cls2, m = train_classification(dc, gsage, cls, "g", "cpu", 0.0, "golden", epochs=2)
            rec["tc__max"] = np.array(m)
            rec["tc__val_f1"] = np.array(printed_f1(buf.getvalue(), "Validation F1"))
            rec["tc__state"] = np.array(random.getstate()[1], np.int64)
            for k, v in cls2.state_dict().items():
                rec[f"tc__cls.{k}"] = v.numpy().copy()
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(OUT, "eval_utils.npz"), **rec)
    print("golden vectors written to", os.path.join(OUT, "eval_utils.npz"))


if __name__ == "__main__":
    main()
