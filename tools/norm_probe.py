"""Per-step gradient norms of the bench workload: how often clip_grad_norm_
(max_norm 5, utils.py:186) actually scales the gradients.  Runs the bench's
runner one step at a time and reads the clipped gradients it leaves behind
(per group: the sage weights, the classifier); a group norm at max_norm means
the step was clipped.  Developer tool:
  python3 tools/norm_probe.py [config=rmat2m] [steps=300]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

gs = bench.gs
train = bench.train


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "rmat2m"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    cfg = bench.CONFIGS[name]
    device = torch.device("cuda", 0)
    wl = bench.build_workload(cfg, device, 824, 1)
    trainer = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], cfg["classes"], num_layers=2, hidden=128,
                                  fanouts=cfg["fanouts"], agg_func=cfg["agg"], seed=824)
    batches = list(train.rank_batches(wl["candidates"], cfg["batch"], 0, 1, 824 + 1000))[:steps]
    runner = train.Runner(trainer, wl["graph"], batches, [train.make_rng(824, 0, w) for w in range(4)],
                          cfg["fanouts"], gcn=False, fail_empty=cfg["agg"] == "MAX")
    g_off = trainer.p.group_off
    norms = []
    for s in range(len(batches)):
        runner.run(1)
        torch.cuda.synchronize()
        g = trainer.p.grads
        norms.append([float(torch.linalg.vector_norm(g[int(g_off[i]):int(g_off[i + 1])]).item()) for i in range(2)])
        if s % 25 == 0:
            print(f"step {s}: post-clip group norms {norms[-1][0]:.4f} {norms[-1][1]:.4f}", flush=True)
    runner.close()
    n = np.array(norms)
    clipped = (n >= 5.0 * (1 - 1e-5)).any(axis=1)
    print(f"{name}: {len(n)} steps, clipped in {int(clipped.sum())} ({clipped.mean():.1%}); "
          f"group-0 norm median {np.median(n[:, 0]):.4f} max {n[:, 0].max():.4f}; "
          f"group-1 median {np.median(n[:, 1]):.4f} max {n[:, 1].max():.4f}")


if __name__ == "__main__":
    main()
