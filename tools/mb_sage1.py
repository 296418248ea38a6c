"""Microbenchmark of layer 1 on one rmat2m batch: fused gs_sage1_fwd (H=128
and H=16, i.e. nearly no GEMM) vs gs_agg_fwd + gs_sage_linear_fwd.  Run under
rocprofv3 --kernel-trace --stats for per-kernel durations (tools/prof_mb.sh
with MB=tools/mb_sage1.py).  GPU only; not a test."""
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
gs = importlib.import_module("graphsage-pytorch_amd")
ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")
models = importlib.import_module("graphsage-pytorch_amd.models")
train = importlib.import_module("graphsage-pytorch_amd.train")


def main():
    dev = torch.device("cuda:0")
    src, dst = gs.rmat_pairs(21, 20_000_000, seed=824, n_threads=16)
    g = gs.CSRGraph.from_pairs(src, dst, 1 << 21, n_threads=16)
    X = torch.empty(1 << 21, 256, device=dev)
    ops.fill_uniform(X, 824)
    roots = next(iter(train.rank_batches(np.nonzero(g.degrees())[0], 512, 0, 1, 1824)))
    s = gs.sample(g, gs.RNG(824), roots, [25, 10])
    ds = models.DeviceSample(s, dev)
    _, col = g.device_csr(dev)
    ptr_, ent, dsts = ds.field(2, "pos_ptr"), ds.field(2, "pos"), ds.field(2, "dst_ids")
    n = s.sizes(2)[0]
    for H in (128, 16):
        W = torch.randn(H, 512, device=dev) * 0.05
        a = torch.empty(n, 256, device=dev)
        h = torch.empty(n, H, device=dev)
        for _ in range(30):
            ops.sage1_fwd("MEAN", X, ptr_, ent, col, dsts, W, a, h)
            torch.cuda._sleep(20000)
        for _ in range(30):
            ops.agg_fwd("MEAN", X, ptr_, ent, a, row_ptr=None, col=col, dst_ids=dsts)
            ops.sage_linear_fwd(a, W, h, Xs=X, sidx=dsts)
            torch.cuda._sleep(20000)
    torch.cuda.synchronize()
    print("n_dst", n, "n_pos", s.sizes(2)[1])


if __name__ == "__main__":
    main()
