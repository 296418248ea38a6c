"""cProfile of bench.py's Pubmed apply_model step (host time by function):
the bench's own workload and step, 10 warmup + 30 profiled steps."""
import cProfile, importlib, pstats, random, sys, time
sys.path.insert(0, '.')
import numpy as np, torch
bench = importlib.import_module("bench")
models = importlib.import_module("graphsage-pytorch_amd.models")
unsup = importlib.import_module("graphsage-pytorch_amd.unsup")
utils = importlib.import_module("graphsage-pytorch_amd.utils")
cfg = dict(bench.CONFIGS["pubmed"])
dev = torch.device("cuda", 0)
wl = bench.pubmed_workload(cfg, dev, 824)
torch.manual_seed(824)
g = models.GraphSage(2, cfg["feat"], 128, wl["X"], wl["graph"], dev, agg_func=cfg["agg"],
                     fanouts=list(cfg["fanouts"]), sampler_helpers=7).to(dev)
cls = models.Classification(128, cfg["classes"]).to(dev)
ul = unsup.UnsupervisedLoss(wl["graph"], wl["train"], dev, n_threads=16)
opt = torch.optim.SGD([p for m in (g, cls) for p in m.parameters()], lr=0.7)
order = np.random.RandomState(825).permutation(wl["train"])
nb = len(order) // cfg["batch"]
batches = [order[(i % nb) * cfg["batch"]:(i % nb + 1) * cfg["batch"]] for i in range(40)]
random.seed(824)
step = lambda b: utils.train_step(g, cls, ul, opt, b, wl["labels"], 100, "sup", None)  # noqa: E731
for b in batches[:10]:
    step(b)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for b in batches[10:]:
    step(b)
torch.cuda.synchronize()
pr.disable()
print("ms/step", (time.perf_counter() - t0) / 30 * 1e3)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumtime").print_stats(40)
