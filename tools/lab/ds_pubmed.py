"""Device sampler at the Pubmed apply_model shape (≈9.7k roots, fanouts 10,10):
wall time per batch and the big union's phase stamps (gs_dsampler_debug)."""
import sys, importlib, time
sys.path.insert(0, '.')
import numpy as np, torch
gs = importlib.import_module("graphsage-pytorch_amd")
L = importlib.import_module("graphsage-pytorch_amd._lib")
g = np.load("tests/golden/graphs.npz")
src, dst, n = g["pubmed_src"].astype(np.int64), g["pubmed_dst"].astype(np.int64), int(g["pubmed_n"][0])
G = gs.CSRGraph.from_pairs(src, dst, n)
rs = np.random.RandomState(5)
ds = gs.DeviceSampler(G, np.array([10, 10], np.int32), 10000)
ds.set_rng(gs.RNG(824))
pack = torch.zeros(ds.pack_bound(10000), dtype=torch.int32, device="cuda")
for b in range(8):
    roots = torch.as_tensor(rs.choice(n, 9705, replace=False).astype(np.int32), device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    ds.run(roots, pack)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3
    d = np.zeros(64, np.int64)
    L.check(L.lib().gs_dsampler_debug(ds._h, d.ctypes.data, 64))
    us = lambda a, b_: (d[b_] - d[a]) / 100.0
    nst = int(d[3])
    line = f"batch {b}: {wall:.3f} ms; ublock fresh {us(0,1):.1f} sched {us(1,5):.1f}; ubig launch gap {us(5,2):.1f}; {nst} stages:"
    for s in range(min(nst, 12)):
        t0, t1, t2, x = d[8 + 4 * s], d[9 + 4 * s], d[10 + 4 * s], d[11 + 4 * s]
        line += f" [prep {(t1 - t0) / 100.0:.1f} settle {(t2 - t1) / 100.0:.1f} k{x >> 32} m{x & 0xffffffff}]"
    line += f" frontier {(d[4] - d[10 + 4 * (min(nst, 12) - 1)]) / 100.0:.1f} us"
    print(line, flush=True)
