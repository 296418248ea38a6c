"""Device sampler phase stamps (gs_dsampler_debug) at the headline size:
the frontier union's phases and per-stage settle rounds, a few batches."""
import sys, importlib, ctypes
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
    nst = int(d[3])
    line = f"batch {b}: scans+compact {us(0,1):.1f} us, schedule {us(1,2):.1f} us, stages {nst}:"
    prev = d[2]
    for s in range(min(nst, 12)):
        t0, t1, t2, x = d[8 + 4 * s], d[9 + 4 * s], d[10 + 4 * s], d[11 + 4 * s]
        line += (f" [prep {(t0 - prev) / 100.0:.1f} r1 {(t1 - t0) / 100.0:.1f} rest {(t2 - t1) / 100.0:.1f}us "
                 f"r{x >> 48} k{(x >> 32) & 0xffff} m{x & 0xffffffff}]")
        prev = t2
    line += f" frontier {(d[4] - prev) / 100.0:.1f} us; total {us(0, 4):.1f} us"
    print(line, flush=True)
    print(f"  tables last block (hop 2): load+nodes+build {(d[46]-d[40])/100:.1f} us, walk {(d[41]-d[46])/100:.1f} us; "
          f"bw {d[42]} nsr {d[43]} C {d[44]} nvalid {d[45]}; slow pool {d[48]} slow set {d[49]}", flush=True)
