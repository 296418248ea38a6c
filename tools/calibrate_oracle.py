"""Calibrate the CPU baseline (the oracle port, bench.py cpu_baseline) against
the reference itself on identical rmat2m inputs in THIS container (SURVEY
§8(d)(ii)).  Study/measurement tool: imports the reference read-only from
/root/reference (PYTHONDONTWRITEBYTECODE=1); never shipped, never run on the GPU
box (the reference does not travel).

Inputs (bench.py rmat2m): R-MAT scale 21, 20M pairs, seed 824, hashed U(-1,1)
256-d features (gs_uniform_host = the device fill's values), labels id % 16,
batches train.rank_batches(seed + 1000), fanouts (25, 10), MEAN, B = 512.
Both run the apply_model body without extend_nodes (utils.py:144-191):
forward, log_softmax NLL, backward, clip_grad_norm_(5) per model, SGD 0.7,
from the same torch.manual_seed(824) init and the same random.seed(824)
stream.  The losses must agree (a full-size parity check of the oracle
against the reference) and the per-step times give the port/reference ratio.

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_oracle.py [steps] [threads]
"""
import importlib
import json
import os
import platform
import random
import sys
import time
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
gs = importlib.import_module("graphsage-pytorch_amd")
train = importlib.import_module("graphsage-pytorch_amd.train")
import oracle  # noqa: E402

SEED, F, H, C, B, FAN = 824, 256, 128, 16, 512, (25, 10)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sys.path.insert(0, "/root/reference")
    from src.models import Classification, GraphSage  # the reference, read-only

    t0 = time.perf_counter()
    src, dst = gs.rmat_pairs(21, 20_000_000, seed=SEED)
    n = 1 << 21
    X = torch.from_numpy(gs.uniform_host(SEED, 0, F, n)) if hasattr(gs, "uniform_host") else None
    if X is None:
        buf = np.empty((n, F), np.float32)
        gs._lib.check(gs._lib.lib().gs_uniform_host(SEED, 0, F, n, buf.ctypes.data))
        X = torch.from_numpy(buf)
    labels = torch.from_numpy(np.arange(n) % C).long()
    deg = np.bincount(np.concatenate([src, dst]), minlength=n)
    cands = np.nonzero(deg > 0)[0]
    batches = list(train.rank_batches(cands, B, 0, 1, SEED + 1000))[:steps]
    t_in = time.perf_counter() - t0

    t0 = time.perf_counter()
    adj = defaultdict(set)  # dataCenter.py:33-41, pairs in generation order
    for a, b in zip(src.tolist(), dst.tolist()):
        adj[a].add(b)
        adj[b].add(a)
    t_adj = time.perf_counter() - t0

    torch.manual_seed(SEED)
    ref = GraphSage(2, F, H, X, adj, torch.device("cpu"))
    cls = Classification(H, C)
    hop = [0]
    orig = ref._get_unique_neighs_list

    def fanout_hops(nodes, num_sample=10):  # the bench's fanouts, hop 1 = the roots
        k = FAN[hop[0] % len(FAN)]
        hop[0] += 1
        return orig(nodes, num_sample=k)
    ref._get_unique_neighs_list = fanout_hops
    init = [p.detach().clone() for p in (ref.sage_layer1.weight, ref.sage_layer2.weight, cls.layer[0].weight,
                                         cls.layer[0].bias)]
    opt = torch.optim.SGD(list(ref.parameters()) + list(cls.parameters()), lr=0.7)
    random.seed(SEED)
    ref_t, ref_loss = [], []
    for roots in batches:
        t = time.perf_counter()
        hop[0] = 0
        emb = ref(roots.tolist())
        logp = cls(emb)
        loss = -torch.sum(logp[range(logp.size(0)), labels[torch.from_numpy(roots)]], 0) / len(roots)
        loss.backward()
        for m in (ref, cls):
            torch.nn.utils.clip_grad_norm_(m.parameters(), 5)
        opt.step()
        opt.zero_grad()
        ref_t.append(time.perf_counter() - t)
        ref_loss.append(float(loss))
    ref_state = random.getstate()

    t0 = time.perf_counter()
    oadj = oracle.Adjacency(src, dst, n)
    t_oadj = time.perf_counter() - t0
    W = [p.clone().requires_grad_(True) for p in init]
    random.seed(SEED)
    port_t, port_loss = [], []
    for roots in batches:
        t = time.perf_counter()
        port_loss.append(oracle.train_step_dense(oadj, roots.tolist(), list(FAN), X, W[:2], W[2], W[3],
                                                 labels[torch.from_numpy(roots)]))
        port_t.append(time.perf_counter() - t)
    assert random.getstate() == ref_state, "the oracle drew a different random stream"
    dl = max(abs(a - b) for a, b in zip(ref_loss, port_loss))
    dw = max(float((a.detach() - b.detach()).abs().max()) for a, b in
             zip(W, (ref.sage_layer1.weight, ref.sage_layer2.weight, cls.layer[0].weight, cls.layer[0].bias)))
    med = lambda v: float(np.median(v[1:] if len(v) > 1 else v))  # noqa: E731
    out = {
        "what": "oracle port (bench.py cpu_baseline) vs the reference itself, identical rmat2m inputs, same host",
        "host": {"cpu": cpu_model(), "visible_cpus": os.cpu_count(), "torch_threads": threads},
        "workload": f"rmat2m: R-MAT scale 21, 20M pairs, F {F}, fanouts {FAN}, MEAN, B {B}, {steps} steps "
                    "(first untimed), apply_model body without extend_nodes",
        "reference_ms_per_step": round(med(ref_t) * 1e3, 1),
        "port_ms_per_step": round(med(port_t) * 1e3, 1),
        "reference_roots_per_s": round(B / med(ref_t), 1),
        "port_roots_per_s": round(B / med(port_t), 1),
        "port_over_reference": round(med(ref_t) / med(port_t), 3),
        "max_loss_diff": dl, "max_weight_diff": dw, "random_state_equal": True,
        "setup_s": {"inputs": round(t_in, 1), "reference_adj_lists": round(t_adj, 1), "port_adjacency": round(t_oadj, 1)},
        "losses": [round(x, 6) for x in ref_loss],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
