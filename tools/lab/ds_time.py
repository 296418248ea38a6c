"""Device sampler at the headline size (rmat2m, B=512, fanouts 25,10):
parity with the host sampler on the first batches, then the per-batch
latency (one batch at a time) and the throughput (back to back)."""
import sys, time, importlib
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from test_gpu_dsampler import host_pack, assert_packs_equal
gs = importlib.import_module("graphsage-pytorch_amd")
train = importlib.import_module("graphsage-pytorch_amd.train")
t0 = time.time()
src, dst = gs.rmat_pairs(21, 20_000_000, seed=824, n_threads=16)
G = gs.CSRGraph.from_pairs(src, dst, 1 << 21, n_threads=16)
print("graph", time.time() - t0, flush=True)
cand = np.nonzero(G.degrees() > 0)[0]
batches = list(train.rank_batches(cand, 512, 0, 1, 1824))
fan = np.array([25, 10], np.int32)
rng = gs.RNG(824)
ds = gs.DeviceSampler(G, fan, 512)
ds.set_rng(rng)
pack = torch.zeros(ds.pack_bound(512), dtype=torch.int32, device="cuda")
for b in range(3):
    ref, sizes, offs, used = host_pack(G, rng, batches[b], fan)
    p, dsz, doff, dused = ds.run(batches[b], pack)
    assert dused == used
    assert_packs_equal(p[:used].cpu().numpy(), ref, sizes, offs, 512, f"batch {b}")
    print("batch", b, "equal; sizes", sizes.tolist(), flush=True)
roots = [torch.from_numpy(b.astype(np.int32)).cuda() for b in batches[3:103]]
torch.cuda.synchronize()
lat = []
for r in roots[:30]:
    t = time.perf_counter()
    ds.run(r, pack)
    lat.append(time.perf_counter() - t)
print("latency per batch (run + result sync) ms: median %.3f min %.3f" % (np.median(lat) * 1e3, np.min(lat) * 1e3))
st = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
L = importlib.import_module("graphsage-pytorch_amd._lib")
e0.record()
for r in roots[30:]:
    L.check(L.lib().gs_dsampler_run(ds._h, r.data_ptr(), 512, pack.data_ptr(), pack.numel(), L.stream_ptr()))
e1.record()
torch.cuda.synchronize()
print("back-to-back device ms per batch: %.3f" % (e0.elapsed_time(e1) / len(roots[30:])))
mt_d, pos_d = ds.get_rng()
