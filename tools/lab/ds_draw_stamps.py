"""Phase stamps of one hop-2 draw_masked workgroup at the headline size
(rmat2m, B=512, fanouts 25,10): load, mask build, walks (gs_dsampler_debug 56..61)."""
import sys, importlib
sys.path.insert(0, '.')
import numpy as np, torch
gs = importlib.import_module("graphsage-pytorch_amd")
train = importlib.import_module("graphsage-pytorch_amd.train")
L = importlib.import_module("graphsage-pytorch_amd._lib")
src, dst = gs.rmat_pairs(21, 20_000_000, seed=824, n_threads=16)
G = gs.CSRGraph.from_pairs(src, dst, 1 << 21, n_threads=16)
cand = np.nonzero(G.degrees() > 0)[0]
batches = list(train.rank_batches(cand, 512, 0, 1, 1824))
ds = gs.DeviceSampler(G, np.array([25, 10], np.int32), 512)
ds.set_rng(gs.RNG(824))
pack = torch.zeros(ds.pack_bound(512), dtype=torch.int32, device="cuda")
for b in range(6):
    ds.run(batches[b], pack)
    d = np.zeros(64, np.int64)
    L.check(L.lib().gs_dsampler_debug(ds._h, d.ctypes.data, 64))
    us = lambda a, b_: (d[b_] - d[a]) / 100.0
    x, y = int(d[60]), int(d[61])
    print(f"batch {b}: load {us(56, 57):.1f} us, masks {us(57, 58):.1f} us, walks {us(58, 59):.1f} us; "
          f"nodes {x & 0xffff}, entries {(x >> 16) & 0xffff}, blocks {x >> 32}, work items {y & 0xffff}, "
          f"W {(y >> 16) & 0xffff}, draws {y >> 32}", flush=True)
