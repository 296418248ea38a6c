"""Debug helper: device vs host one-hop pack, print mismatching roots."""
import sys, importlib
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from test_gpu_dsampler import mixed_graph, host_pack, gs
import importlib
M = importlib.import_module("graphsage-pytorch_amd.mt19937") if False else None
graph = mixed_graph()
deg = graph.degrees()
for fan in ([25], [10], [3]):
    fan = np.array(fan, np.int32)
    rng_h = gs.RNG(824)
    ds = gs.sampler.DeviceSampler(graph, fan, 512)
    ds.set_rng(rng_h)
    rs = np.random.RandomState(1)
    roots = rs.choice(np.arange(graph.n_nodes), 512, replace=True).astype(np.int64)
    ref, sizes, offs, used = host_pack(graph, rng_h, roots, fan)
    pack, dsz, doff, dused = ds.run(roots)
    got = pack[:used].cpu().numpy()
    bad = np.nonzero(got != ref)[0]
    print("fan", fan, "mismatches", len(bad))
    pp = ref[offs[0, 0]:offs[0, 0] + len(roots) + 1]
    pos0 = offs[0, 1]
    rp = graph.row_ptr()
    for i in bad[:10]:
        if i >= pos0 and i < pos0 + pp[-1]:
            e = i - pos0
            r = np.searchsorted(pp, e, side='right') - 1
            v = roots[r]
            print(f"  root {r} v {v} deg {deg[v]} slot {e - pp[r]}: got pos {got[i]-rp[v]} want {ref[i]-rp[v]}",
                  "row got", got[pos0+pp[r]:pos0+pp[r+1]] - rp[v], "want", ref[pos0+pp[r]:pos0+pp[r+1]] - rp[v])
        else:
            print("  idx", i, got[i], ref[i])
