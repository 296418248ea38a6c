"""Per-workgroup timing of one trainer timer site at the bench workload: a
runner step loop with the site stamped (sites 1-4: the kernel stores each
workgroup's s_memrealtime start and end), then the last launches' stamps in
block ranges.  Developer tool:
    python tools/lab/site_stamps.py SITE [steps] [config] [split,...]
SITE 2: the layer-1 dW launch (dw1_top_kernel: dW1 blocks first), 4: the slab
pair (layer-2 blocks first).  `split` lists block indices where a new range
starts (default: every 40 blocks)."""
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
bench = importlib.import_module("bench")
gs = importlib.import_module("graphsage-pytorch_amd")
train = importlib.import_module("graphsage-pytorch_amd.train")


def main():
    site = int(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    name = sys.argv[3] if len(sys.argv) > 3 else "rmat2m"
    cuts = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else None
    cfg = dict(bench.CONFIGS[name])
    dev = torch.device("cuda", 0)
    wl = bench.build_workload(cfg, dev, 824, 1)
    t = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], cfg["classes"], num_layers=2, hidden=128,
                            fanouts=cfg["fanouts"], agg_func=cfg["agg"], seed=824)
    batches = list(train.rank_batches(wl["candidates"], cfg["batch"], 0, 1, 824))[:steps]
    r = train.Runner(t, wl["graph"], batches, [train.make_rng(824, 0, w) for w in range(7)], cfg["fanouts"],
                     gcn=False, helpers=1)
    lib = gs._lib.lib()
    r.run(steps - 10)
    torch.cuda.synchronize()
    gs._lib.check(lib.gs_trainer_time_kernels(t._h, 1 << site, 10))
    r.run(10)
    torch.cuda.synchronize()
    print(f"site {site} kernel:", lib.gs_trainer_kernel_name(t._h, site).decode()[:90])
    S = np.zeros(1024, np.uint64)
    E = np.zeros(1024, np.uint64)
    for launch in range(7, 10):
        got = int(lib.gs_trainer_kernel_stamps(t._h, site, launch, S.ctypes.data, E.ctypes.data))
        if got <= 0:
            print("no stamps", got)
            return
        have = np.nonzero(S)[0]
        t0 = S[have].min()
        s = (S.astype(np.float64) - float(t0)) * 1e-2
        e = (E.astype(np.float64) - float(t0)) * 1e-2
        print(f"launch {launch}: blocks stamped {len(have)}, span {e[have].max():.2f} us")
        edges = sorted(set([0] + (cuts or list(range(40, int(have.max()) + 1, 40))) + [int(have.max()) + 1]))
        for lo, hi in zip(edges[:-1], edges[1:]):
            bl = have[(have >= lo) & (have < hi)]
            if not len(bl):
                continue
            d = e[bl] - s[bl]
            print(f"  blocks {lo}..{hi - 1}: start {s[bl].min():.2f}..{s[bl].max():.2f}  end {e[bl].min():.2f}.."
                  f"{e[bl].max():.2f}  dur med {np.median(d):.2f} max {d.max():.2f}")
    r.close()


if __name__ == "__main__":
    main()
