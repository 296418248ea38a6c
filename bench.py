"""Headline benchmark: GraphSAGE supervised training throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config rmat2m]
    torchrun --nproc-per-node N bench.py --gpus N ...     (data parallel, RCCL)

A step = one pass of the hot path over one batch of B roots per GPU: sample
both hops (bit-exact host sampler, prefetched on a thread) -> one H2D copy ->
layer-1 gather-aggregate + MFMA SageLayer -> layer 2 -> classifier + NLL ->
full backward -> RCCL all-reduce of the flat gradient -> clip + SGD.
Throughput = roots processed by all ranks / max-over-ranks wall time of the
timed steps (weak scaling: B roots per GPU per step).

Prints ONE JSON line on rank 0.  `roofline` prices the dominant kernel (the
largest average in the committed rocprofv3 summary of the config: the layer-1
forward GEMM at fp32, the dW GEMM at bf16) from its algorithmic flops or bytes
against the peak of the MFMA it issues (the bf16 dW widens its operands to
fp32: fp32 peak, the bf16 peak and fraction beside it) and its launch duration
inside the timed region: the kernel's own span
(per-workgroup s_memrealtime stamps, min start .. max end) for the forward
and top launches, kernel-bound HIP events for the gather and dW;
`cpu_baseline` times the oracle (the CPU restatement of the reference's
algorithm) on a bounded sample of the same workload on this host.
"""
import argparse
import csv
import glob
import json
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import importlib  # noqa: E402

gs = importlib.import_module("graphsage-pytorch_amd")
from importlib import import_module  # noqa: E402

train = import_module("graphsage-pytorch_amd.train")
ops = import_module("graphsage-pytorch_amd.hip_ops")
models = import_module("graphsage-pytorch_amd.models")

CONFIGS = {
    # BASELINE.json configs[2]: the headline metric's workload
    "rmat2m": dict(scale=21, pairs=20_000_000, feat=256, fanouts=(25, 10), agg="MEAN", dtype="fp32",
                   batch=512, classes=16),
    # configs[3]
    "rmat2m-max-bf16": dict(scale=21, pairs=20_000_000, feat=256, fanouts=(25, 10), agg="MAX",
                            dtype="bf16", batch=512, classes=16),
    # configs[1]: the reference's own loop (apply_model, utils.py:113-193) on the Pubmed citation
    # graph (pairs from the reference's cites file, tests/golden/graphs.npz): every step
    # extend_nodes(512 roots, num_neg=100) -> GraphSage forward over the extended batch
    # (fanouts 10,10) -> supervised NLL -> backward -> clip -> SGD, through the drop-in modules
    "pubmed": dict(graph="pubmed", feat=500, fanouts=(10, 10), agg="MEAN", dtype="fp32", batch=512, classes=3,
                   loop="apply_model"),
    # configs[0]: the reference's CPU-runnable case (Cora, b_sz 20, supervised) through the same
    # apply_model loop as pubmed (cites-file graph from tests/golden/graphs.npz)
    "cora": dict(graph="cora", feat=1433, fanouts=(10, 10), agg="MEAN", dtype="fp32", batch=20, classes=7,
                 loop="apply_model"),
    # configs[4] (per-GPU share of the 8-GPU job)
    "rmat16m": dict(scale=24, pairs=160_000_000, feat=128, fanouts=(25, 10), agg="MEAN", dtype="fp32",
                    batch=512, classes=16),
    # get_gnn_embeddings (utils.py:59-78) over the rmat2m graph — batches of 500 node ids
    # in id order, batch i on rank i % W, forward-only runner, one all-gather of the [N, 128] result
    "rmat2m-embed": dict(scale=21, pairs=20_000_000, feat=256, fanouts=(25, 10), agg="MEAN", dtype="fp32",
                         batch=500, classes=16, loop="embed"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# the trainer's kernel timer sites (gs_trainer_time_kernels)
SITES = (0, 1, 2, 3)
SITE_NAMES = {0: "gather", 1: "fwd", 2: "dw", 3: "top"}
SITE_ROLES = {0: "layer-1 gather-aggregate (models.py:291-330 at layer 1)",
              1: "layer-1 SageLayer forward GEMM relu([X[self] | agg]·W1ᵀ) (models.py:216-219)",
              2: "layer-1 weight-gradient GEMM dW1 = dZ1ᵀ·[X[self] | agg] row slabs (autograd of models.py:219)",
              3: "top layer + loss head in one launch: layer-2 aggregate, linear + relu, log_softmax/NLL, dZ2, "
                 "dIn2 = dZ2·W2 (models.py:291-330, :216-219, :8-27; utils.py:159-164)"}
MFMA_PEAK_TFS = {"fp32": 157.3, "bf16": 2500.0}  # MI355X_MICROARCH.md: dense F32 / BF16 matrix peaks (spec)


def host_cores():
    """CPUs this process may use: affinity, capped by a cgroup-v2 CPU quota
    (the GPU boxes grant 16 CPUs per GPU while showing every core)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def host_threads():
    return max(1, min(16, host_cores()))


def build_workload(cfg, device, seed=824, world=1):
    """R-MAT pairs -> host CSR (CPython-set row order), hashed features, labels.
    With several ranks the CSR is built once per node: local rank
    0 generates the pairs, builds it and writes its image to /dev/shm; the
    other ranks map that image read-only (no pairs, no build, no copy)."""
    t0 = time.perf_counter()
    n = 1 << cfg["scale"]
    src = dst = None

    def build():
        nonlocal src, dst
        src, dst = gs.rmat_pairs(cfg["scale"], cfg["pairs"], seed=seed, n_threads=host_threads())
        return gs.CSRGraph.from_pairs(src, dst, n, n_threads=host_threads())

    shm = None
    if world > 1:
        shm = f"/dev/shm/gs_csr_s{cfg['scale']}_p{cfg['pairs']}_{seed}_{os.environ.get('MASTER_PORT', '0')}.bin"
        graph = gs.CSRGraph.shared(build, shm, int(os.environ.get("LOCAL_RANK", "0")), dist.barrier)
        dist.barrier()  # every rank has mapped the image: the file can go (the mappings stay)
        if int(os.environ.get("LOCAL_RANK", "0")) == 0 and os.path.exists(shm):
            os.unlink(shm)
        if src is not None:
            del src, dst  # the cpu_baseline leg (the only pair-list user) runs at world 1
            src = dst = None
    else:
        graph = build()
    t_graph = time.perf_counter() - t0
    dt = torch.bfloat16 if cfg["dtype"] == "bf16" else torch.float32
    X = torch.empty(n, cfg["feat"], dtype=dt, device=device)
    ops.fill_uniform(X, seed)
    labels = torch.from_numpy((np.arange(n, dtype=np.int64) % cfg["classes"]).astype(np.int32)).to(device)
    deg = graph.degrees()
    candidates = np.nonzero(deg > 0)[0]
    return dict(src=src, dst=dst, n=n, graph=graph, X=X, labels=labels, candidates=candidates,
                t_graph=t_graph, deg=deg, shm=shm, csr_shared=shm is not None)


def block_stats_us(trainer, n, site):
    """Per stamped launch of `site`: span, mean / max workgroup duration and
    the spread of workgroup starts (us), medians over the launches; None for
    an event-timed site."""
    if not hasattr(gs._lib.lib(), "gs_trainer_kernel_block_stats"):  # an older library (A/B runs)
        return None
    out = np.zeros((max(n, 1), 4), np.float32)
    got = int(gs._lib.lib().gs_trainer_kernel_block_stats(trainer._h, site, out.ctypes.data, n))
    out = out[:max(got, 0)]
    out = out[out[:, 0] >= 0]
    if not len(out):
        return None
    med = np.median(out, axis=0)
    return {"span": round(float(med[0]), 2), "workgroup_mean": round(float(med[1]), 2),
            "workgroup_max": round(float(med[2]), 2), "start_spread": round(float(med[3]), 2),
            "launches": int(len(out))}


def kernel_times_ms(trainer, n, site=0):
    """Kernel-bound HIP-event durations recorded by the native step on its
    launch stream (gs_trainer_time_agg arms them): site 0 the layer-1
    gather-aggregate, 1 the layer-1 SageLayer GEMM, 2 its weight-gradient GEMM."""
    out = np.zeros(max(n, 1), np.float32)
    got = int(gs._lib.lib().gs_trainer_kernel_times(trainer._h, site, out.ctypes.data, n))
    if got < 0:
        raise RuntimeError("event timing failed")
    return out[:got]


def agg1_times_ms(trainer, n):
    return kernel_times_ms(trainer, n, 0)


def cgroup_throttle():
    """Cumulative CPU-quota throttling of this cgroup (us), or None."""
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            if line.startswith("throttled_usec"):
                return int(line.split()[1])
    except OSError:
        pass
    return None


def agg1_bytes(n_dst, n_pos, F, elem):
    """Algorithmic HBM bytes of one layer-1 K-agg launch:
    neighbour feature rows once per sampled edge + sampled positions and CSR
    column entries (4 B each) + one output row per destination + per-destination
    metadata (dst id 4 B, row_ptr 8 B, pos_ptr 4 B)."""
    return n_pos * (F * elem + 8) + n_dst * (F * elem + 16)


def top_bytes(B, n_nbr, H, C):
    """Algorithmic HBM bytes of one fused top launch (kernels/top.hip): the
    roots' neighbour and self rows of h1, their neighbour lists, W2 and the
    classifier, and the rows it writes (agg, E, dZ: H each; dIn: 2H)."""
    return (n_nbr + B) * H * 4 + n_nbr * 4 + H * 2 * H * 4 + C * (H + 1) * 4 + B * 5 * H * 4


def agg1_ids_bytes(n_dst, n_pos, F, elem, k, self_rows=True):
    """Algorithmic HBM bytes of one launch of the runner's layer-1 gather over
    resolved ids (agg_ids_kernel): one feature row per sampled edge, the
    destination's k padded neighbour ids (4 B each), one output row; with the
    self rows in the slot (the trainer's default) also the destination's own
    row read and written beside it."""
    return n_pos * F * elem + n_dst * (k * 4 + F * elem) + (2 * n_dst * F * elem if self_rows else 0)


def replay_frontiers(graph, batches, n_streams, fanouts, seed, rank, upto):
    """Per batch i < upto: (B, |L1|, |L0|) — the roots and both hops' unique
    frontiers, the reference's `nodes_batch_layers` (models.py:246-251).  The
    runner never materialises the last hop's union (the layer-1 gather needs
    only the sampled positions), so its size comes from replaying the same
    streams afterwards: stream w drew batches w, w+S, ... in order from
    make_rng(seed, rank, w), and the same draws on a copy give the identical
    hops (bit-exact sampler), here with the last union materialised."""
    rngs = [train.make_rng(seed, rank, w) for w in range(n_streams)]
    out = np.zeros((upto, 3), np.int64)
    for i in range(upto):
        smp = gs.sampler.sample(graph, rngs[i % n_streams], batches[i], list(fanouts), full=True)
        L = smp.n_hops
        out[i, 0] = len(batches[i])
        out[i, 1] = smp.sizes(1)[2]  # hop 1's union: |L1|
        out[i, 2] = smp.sizes(L)[2]  # the last hop's union: |L0|
    return out


def port_calibration():
    """The oracle port's speed relative to the reference itself on identical
    rmat2m inputs, measured in the build container (tools/calibrate_oracle.py;
    the reference never travels to the GPU box)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "r02_oracle_calibration_rmat2m.json")))
        return {"port_over_reference": d["port_over_reference"], "reference_ms_per_step": d["reference_ms_per_step"],
                "port_ms_per_step": d["port_ms_per_step"], "host": d["host"], "losses_equal": d["max_loss_diff"] == 0.0,
                "source": "profiles/r02_oracle_calibration_rmat2m.json"}
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(wl, cfg, seconds_budget=25.0, seed=824):
    """Oracle train step (CPU restatement of the reference) on this host."""
    import random as pyrandom
    import oracle
    threads = host_threads()
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    adj = oracle.Adjacency(wl["src"], wl["dst"], wl["n"])
    t_adj = time.perf_counter() - t0
    sage_w, cls_w, cls_b = train.reference_init(2, cfg["feat"], 128, cfg["classes"], False, seed)
    W = [w.clone().requires_grad_(True) for w in sage_w]
    cw, cb = cls_w.clone().requires_grad_(True), cls_b.clone().requires_grad_(True)
    X = wl["X"].float().cpu()  # same feature table, fetched once (not timed)
    labels_all = wl["labels"].cpu().long()
    batches = train.rank_batches(wl["candidates"], cfg["batch"], 0, 1, seed + 1000)
    pyrandom.seed(seed)
    times = []
    t_start = time.perf_counter()
    for i, roots in enumerate(batches):
        t = time.perf_counter()
        oracle.train_step_dense(adj, roots.tolist(), list(cfg["fanouts"]), X, W, cw, cb,
                                labels_all[torch.from_numpy(roots)], agg=cfg["agg"])
        times.append(time.perf_counter() - t)
        if time.perf_counter() - t_start > seconds_budget and len(times) >= 3:
            break
    med = float(np.median(times[1:] if len(times) > 1 else times))
    cal = port_calibration() if cfg.get("scale") == 21 and cfg["agg"] == "MEAN" and cfg["dtype"] == "fp32" else None
    out = {"value": cfg["batch"] / med, "unit": "root nodes/s", "cores": threads, "kind": "port",
           "sample": f"{len(times)} oracle train steps of B={cfg['batch']} roots (first untimed), "
                     f"median {med * 1e3:.1f} ms/step; lazy dict-of-sets adjacency (built "
                     f"per touched node), dense-mask mean, torch CPU {threads} threads; "
                     f"pair-list indexing {t_adj:.1f} s excluded"}
    if cal:
        out["calibration"] = cal
        out["reference_estimate"] = round(out["value"] / cal["port_over_reference"], 1)
    return out


# rocprofv3 --kernel-trace --stats summaries of the bench command, per config
# and batch (tools/gpu_pass.sh; earlier rounds: the pass scripts in git history): the profiler's own per-launch average for
# the kernel beside the live event-timed one
# (newest round first: the first file present is used)
ROCPROF_TOL = 0.15  # live vs committed rocprofv3 average: `rocprof_agrees` within this fraction
ROCPROF_STATS = {("rmat2m", 512): ["profiles/r06_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r05_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04f_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04e_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04d_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04c_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04b_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r04_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r03c_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r03b_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r03_kernel_stats_rmat2m_steps300.csv",
                                   "profiles/r02_kernel_stats_rmat2m_steps300.csv"],
                 ("rmat2m-max-bf16", 512): ["profiles/r06_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r05_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04f_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04e_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04d_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04c_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04b_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r04_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r03c_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r03b_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r03_kernel_stats_rmat2m_max_bf16_steps300.csv",
                                            "profiles/r02_kernel_stats_rmat2m_max_bf16_steps300.csv"],
                 ("rmat16m", 512): ["profiles/r06_kernel_stats_rmat16m_steps300.csv",
                                    "profiles/r03c_kernel_stats_rmat16m_steps300.csv",
                                    "profiles/r03_kernel_stats_rmat16m_steps300.csv",
                                    "profiles/r02_kernel_stats_rmat16m_steps300.csv"]}


def rocprof_stats_file(config_name, batch):
    for rel in ROCPROF_STATS.get((config_name, int(batch)), []):
        if os.path.exists(os.path.join(ROOT, rel)):
            return rel
    return None


def kernel_key(name):
    """A kernel's name without its parameter list, and without the
    deferred-update flag of the layer-1 forward (linear_fwd_wide_kernel's fifth
    template argument: the instance with the previous step's update pending and
    the one without, at a run's first step, are one kernel here)."""
    key = name.split("(")[0].strip()
    m = re.match(r"^(.*linear_fwd_wide_kernel<[^,<>]+, \d+, (?:true|false), (?:true|false)), (?:true|false)>$", key)
    return m.group(1) + ">" if m else key


def load_rocprof_avg(config_name, batch, kernel):
    rel = rocprof_stats_file(config_name, batch)
    if not rel:
        return None
    key = kernel_key(kernel)
    best = None
    with open(os.path.join(ROOT, rel)) as f:
        for row in csv.DictReader(f):  # the matching instance with the most calls
            if kernel_key(row.get("Name", "")) == key and (best is None or int(row["Calls"]) > int(best["Calls"])):
                best = row
    if best is None:
        return None
    return {"avg_us": round(float(best["AverageNs"]) / 1e3, 2), "min_us": round(float(best["MinNs"]) / 1e3, 2),
            "source": rel}


def load_traffic(config_name, batch, kernel):
    """Per-launch HBM bytes of `kernel` (its launched name) from the newest
    committed rocprofv3 --pmc summary (profiles/*pmc*.json, tools/pmc_summary.py)
    recorded for this config and this batch size, else None."""
    key = kernel_key(kernel)
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config") != config_name or int(d.get("batch", -1)) != int(batch):
            continue
        k = _most_dispatched(d, lambda n: kernel_key(n) == key)
        if k and "hbm_bytes" in k:
            best = {"hbm_bytes": k["hbm_bytes"], "dispatches": k.get("dispatches"),
                    "source": os.path.relpath(p, ROOT)}
    return best


def _most_dispatched(summary, match):
    """The matching kernel instance of a PMC summary with the most dispatches
    (the in-step one: e.g. the layer-1 forward's pending-update instance runs
    every step but a run's first)."""
    cands = [v for n, v in summary.get("kernels", {}).items() if match(n)]
    return max(cands, key=lambda v: v.get("dispatches", 0)) if cands else None


def load_mfma_busy(config_name, kernel):
    """MFMA utilisation of `kernel` (SQ_VALU_MFMA_BUSY_CYCLES over the SIMDs'
    cycles, per dispatch) from the newest committed rocprofv3 --pmc summary of
    this config (profiles/*pmc_mfma_<config>.json, tools/pmc_mfma_summary.py),
    else None."""
    def bare(n):  # the PMC summaries name kernels with or without the return type
        k = kernel_key(n)
        return k[5:] if k.startswith("void ") else k
    key = bare(kernel)
    best = None
    pat = os.path.join(ROOT, "profiles", f"*pmc_mfma_{config_name.replace('-', '_')}.json")
    for p in sorted(glob.glob(pat)):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        k = _most_dispatched(d, lambda n: bare(n) == key)
        if k and "mfma_util" in k:
            best = {"mfma_util": k["mfma_util"], "dispatches": k.get("dispatches"),
                    "source": os.path.relpath(p, ROOT)}
    return best


def pubmed_workload(cfg, device, seed=824):
    """A citation graph from the reference's cites file (cfg["graph"]: pubmed or cora)."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "graphs.npz"))
    name = cfg.get("graph", "pubmed")
    src, dst, n = g[f"{name}_src"].astype(np.int64), g[f"{name}_dst"].astype(np.int64), int(g[f"{name}_n"][0])
    graph = gs.CSRGraph.from_pairs(src, dst, n)
    X = torch.empty(n, cfg["feat"], dtype=torch.float32, device=device)
    ops.fill_uniform(X, seed)
    np.random.seed(seed)  # dataCenter.py:100-111 split after main.py:41's seed
    perm = np.random.permutation(n)
    train = perm[n // 3 + n // 6:]
    labels = (np.arange(n) % cfg["classes"]).astype(np.int64)
    return dict(src=src, dst=dst, n=n, graph=graph, X=X, train=train, labels=labels)


def cpu_baseline_loop(wl, cfg, batches, seconds_budget=25.0, seed=824):
    """The oracle's restatement of one apply_model step (extend_nodes with
    Python sets + dense-mask forward/backward + clip + SGD) on this host."""
    import random as pyrandom
    import oracle
    from oracle import unsup_semantics as U
    threads = host_threads()
    torch.set_num_threads(threads)
    adj = oracle.Adjacency(wl["src"], wl["dst"], wl["n"])
    st = U.UnsupState(adj, wl["train"])
    sage_w, cls_w, cls_b = train.reference_init(2, cfg["feat"], 128, cfg["classes"], False, seed)
    W = [w.clone().requires_grad_(True) for w in sage_w]
    cw, cb = cls_w.clone().requires_grad_(True), cls_b.clone().requires_grad_(True)
    X = wl["X"].float().cpu()
    labels = torch.from_numpy(wl["labels"])
    pyrandom.seed(seed)
    times = []
    t_start = time.perf_counter()
    for roots in batches:
        t = time.perf_counter()
        nodes, _ = U.extend_nodes(st, roots, 100)
        oracle.train_step_dense(adj, nodes, list(cfg["fanouts"]), X, W, cw, cb,
                                labels[torch.as_tensor(nodes)], agg=cfg["agg"])
        times.append(time.perf_counter() - t)
        if time.perf_counter() - t_start > seconds_budget and len(times) >= 3:
            break
    med = float(np.median(times[1:] if len(times) > 1 else times))
    return {"value": cfg["batch"] / med, "unit": "root nodes/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle apply_model steps of B={cfg['batch']} roots (first untimed), median "
                      f"{med * 1e3:.1f} ms/step: extend_nodes (Python sets, num_neg 100) + dense-mask forward/"
                      f"backward on the extended batch, torch CPU {threads} threads"}


def run_apply_model_loop(args, cfg):
    """configs[1] (pubmed) and configs[0] (cora): timed steps of the reference's
    training loop body through the drop-in modules (UnsupervisedLoss /
    GraphSage / fused head, utils.train_step)."""
    import random as pyrandom
    unsup = import_module("graphsage-pytorch_amd.unsup")
    utils = import_module("graphsage-pytorch_amd.utils")
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    wl = pubmed_workload(cfg, device, args.seed)
    torch.manual_seed(args.seed)
    # the forward's sampling with helper threads (same draws, same pack; the
    # host is otherwise idle while the step's single stream samples)
    helpers = args.helpers_cli if args.helpers_cli is not None else min(7, host_threads() - 1)
    dev_samp = args.sampler == "device"
    gsage = models.GraphSage(2, cfg["feat"], 128, wl["X"], wl["graph"], device, agg_func=cfg["agg"],
                             fanouts=list(cfg["fanouts"]), sampler_helpers=0 if dev_samp else helpers,
                             device_sampler=dev_samp).to(device)
    cls = models.Classification(128, cfg["classes"]).to(device)
    ul = unsup.UnsupervisedLoss(wl["graph"], wl["train"], device, n_threads=host_threads())
    params = [p for m in (gsage, cls) for p in m.parameters()]
    opt = torch.optim.SGD(params, lr=0.7)
    order = np.random.RandomState(args.seed + 1).permutation(wl["train"])
    nb = len(order) // cfg["batch"]
    batches = [order[(i % nb) * cfg["batch"]:(i % nb + 1) * cfg["batch"]] for i in range(args.warmup + args.steps)]
    pyrandom.seed(args.seed)
    step = lambda b: utils.train_step(gsage, cls, ul, opt, b, wl["labels"], 100, "sup", None)  # noqa: E731
    for b in batches[:args.warmup]:
        step(b)
    torch.cuda.synchronize()
    ext = 0
    t0 = time.perf_counter()
    for b in batches[args.warmup:]:
        loss, nodes = step(b)
        ext += len(nodes)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline_loop(wl, cfg, batches, args.cpu_budget, args.seed)
    out = {
        "metric": "sampled nodes/sec (2-layer, fanout 25,10) at 1/2/4/8 MI355X",
        "value": round(cfg["batch"] * args.steps / elapsed, 1), "unit": "root nodes/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": cfg["dtype"],
        "data": f"{cfg['graph'].capitalize()} citation graph (reference cites file), synthetic U(-1,1) "
                f"{cfg['feat']}-d features, labels id%{cfg['classes']}",
        "config": {"workload": f"{args.config}: apply_model step (extend_nodes num_neg 100 + GraphSage fanouts "
                               f"{tuple(cfg['fanouts'])} {cfg['agg']} over the extended batch + sup NLL + backward + "
                               f"clip + SGD), B={cfg['batch']} roots",
                   "global_batch": cfg["batch"], "parallelism": "dp1",
                   "epoch_s": round(len(wl["train"]) // cfg["batch"] * elapsed / args.steps, 4),
                   "extended_nodes_per_step": round(ext / args.steps, 1), "final_loss": round(float(loss), 5),
                   "forward_sampler": "device" if dev_samp else "host",
                   "forward_sampler_helpers": 0 if dev_samp else helpers,
                   "extend_balls": "device" if ul.device_balls else "host"},
        "roofline": None,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)


def cpu_baseline_embed(wl, cfg, seconds_budget=25.0, seed=824):
    """The oracle's forward (sampling + dense-mask layers) over batches of
    embedded node ids, as get_gnn_embeddings runs it, on this host."""
    import random as pyrandom
    import oracle
    threads = host_threads()
    torch.set_num_threads(threads)
    adj = oracle.Adjacency(wl["src"], wl["dst"], wl["n"])
    W = train.reference_init(2, cfg["feat"], 128, cfg["classes"], False, seed)[0]
    X = wl["X"].float().cpu()
    pyrandom.seed(seed)
    times, B = [], cfg["batch"]
    t_start = time.perf_counter()
    with torch.no_grad():
        for i in range(wl["n"] // B):
            t = time.perf_counter()
            hops = oracle.sample_layers(adj, list(range(i * B, (i + 1) * B)), list(cfg["fanouts"]))
            oracle.forward_dense(hops, X, W, cfg["agg"], False)
            times.append(time.perf_counter() - t)
            if time.perf_counter() - t_start > seconds_budget and len(times) >= 3:
                break
    med = float(np.median(times[1:] if len(times) > 1 else times))
    return {"value": B / med, "unit": "embedded nodes/s", "cores": threads, "kind": "port",
            "sample": f"{len(times)} oracle forward batches of {B} ids in id order (first untimed), median "
                      f"{med * 1e3:.1f} ms/batch; torch CPU {threads} threads"}


def run_embed(args, cfg):
    """full-graph inference throughput (utils.get_gnn_embeddings'
    native path): this rank's batches through train.Embedder, then the
    all-gather of [N, 128].  Times the first --steps batches per rank (all of
    them with --full-graph)."""
    utils = import_module("graphsage-pytorch_amd.utils")
    rank, world = train.init_distributed()
    device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(device)
    wl = build_workload(cfg, device, args.seed, world)
    n, B = wl["n"], cfg["batch"]
    n_used = n if args.full_graph else min(n, args.steps * world * B)
    weights = [w.to(device) for w in train.reference_init(2, cfg["feat"], 128, cfg["classes"], False, args.seed)[0]]
    # inference is sampler-throughput bound: by default more streams without
    # helpers (≈ 30 % more batches per second than streams + helpers,
    # profiles/r02_ab_sampler_layouts.txt; the latency a helper saves buys nothing here)
    helpers = args.helpers_cli if args.helpers_cli is not None else 0
    if args.streams_cli is None:
        args.sampler_streams = (max(1, min(12, args.per_gpu - 3)) if not helpers
                                else max(1, min(8, (args.per_gpu - 2) // (1 + helpers))))
    args.sampler_helpers = helpers
    emb = train.Embedder(wl["graph"], wl["X"], weights, cfg["fanouts"], cfg["agg"], merge=args.embed_merge,
                         helpers=helpers)
    mine = utils.shard_ids(n_used, B, rank, world)
    warm = utils.shard_ids(min(n, args.warmup * world * B), B, rank, world)
    if len(warm):
        emb.embed(warm, B, [train.make_rng(args.seed + 1, rank, w) for w in range(args.sampler_streams)])
    rngs = [train.make_rng(args.seed, rank, w) for w in range(args.sampler_streams)]
    n_units = -(-(len(mine) // B) // emb.merge)  # merged steps of emb.merge batches
    n_timed = min(n_units, 200)  # event-bound launches cost host time: time the first 200 gathers
    gs._lib.check(gs._lib.lib().gs_trainer_time_agg(emb.trainer._h, n_timed))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    E = emb.embed(mine, B, rngs)
    if world > 1:  # the assembly get_gnn_embeddings does
        lens = [len(utils.shard_ids(n_used, B, r, world)) for r in range(world)]
        buf = torch.zeros(max(lens), E.shape[1], device=device)
        buf[:len(mine)].copy_(E)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    st = emb.last_stats
    n_b = len(mine) // B
    agg_ms = float(np.mean(agg1_times_ms(emb.trainer, n_timed))) if n_timed else float("nan")
    if rank == 0:
        L = len(cfg["fanouts"])
        sizes = st["hop_sizes_sum"] / max(1, st["steps"])
        agg_bytes = agg1_ids_bytes(sizes[L - 1, 0], sizes[L - 1, 1], cfg["feat"], 4, cfg["fanouts"][-1])
        achieved = float(agg_bytes) / (agg_ms * 1e-3) / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline_embed(wl, cfg, args.cpu_budget, args.seed)
        out = {
            "metric": "embedded nodes/sec (get_gnn_embeddings, 2-layer, fanout 25,10)",
            "value": round(n_used / elapsed, 1), "unit": "embedded nodes/s", "n_gpus": world,
            "steps": n_b, "warmup": len(warm) // B, "ms_per_step": round(elapsed / max(1, n_b) * 1e3, 4),
            "higher_is_better": True, "scaling": "strong" if args.full_graph else "weak", "vs_baseline": None,
            "dtype": cfg["dtype"], "data": "synthetic (R-MAT graph, hashed U(-1,1) features), reference-init weights",
            "config": {"workload": f"rmat2m-embed: {n_used} of {n} node ids in batches of {B} (id order), "
                                   f"fanout {tuple(cfg['fanouts'])}, MEAN, forward only + all-gather",
                       "global_batch": B * world, "parallelism": f"dp{world}",
                       "sampler_streams_per_gpu": args.sampler_streams,
                       "sampler_helpers_per_stream": args.sampler_helpers,
                       "sampler_depth_per_stream": args.sampler_depth, "batches_per_launch": emb.merge,
                       "host_sampler_ms_per_batch": round(1e3 * st["sample_s"] / max(1, n_b), 3),
                       "host_ms_per_batch": {k: round(1e3 * st[k + "_s"] / max(1, n_b), 4)
                                             for k in ("wait", "wait_sample", "wait_ring", "wait_gather", "issue")},
                       "lookahead_misses": st["lookahead_misses"]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "agg_ids_kernel (layer-1 gather-mean over resolved neighbour ids)",
                         "avg_launch_us": round(agg_ms * 1e3, 2), "algo_bytes_per_launch": int(agg_bytes)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def reference_stream_window(trainer, wl, cfg, args, batches):
    """The reference's own sampling trajectory, driver-timed: ONE sampler
    stream seeded exactly as random.seed(seed) (stream 0 of rank 0,
    models.py:281-282, main.py:40) — every batch's draws are the reference's
    words in order, bit for bit — with helper threads building its sets and
    lists (the same draws).  Steps run back to back after a short warmup; the
    single stream is sequential on its `random` state, so this window is
    sampler-bound by construction and reports the sampler's per-batch time."""
    helpers = max(1, min(7, args.per_gpu - 2))
    K, W = args.ref_stream_steps, 5
    rb = batches[:W + K]
    runner = train.Runner(trainer, wl["graph"], rb, [train.make_rng(args.seed, 0, 0)], cfg["fanouts"], gcn=False,
                          fail_empty=cfg["agg"] == "MAX", helpers=helpers, warm=not args.no_warm,
                          sampler=args.sampler)
    runner.run(W)
    torch.cuda.synchronize()
    runner.stats(reset=True)
    t0 = time.perf_counter()
    runner.run(K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = runner.stats()
    runner.close()
    n = max(1, st["steps"])
    return {"value": round(cfg["batch"] * K / el, 1), "unit": "root nodes/s", "steps": K, "warmup": W,
            "ms_per_step": round(el / K * 1e3, 4),
            "stream": f"random.seed({args.seed}) (stream 0 of rank 0: the reference's single global stream)",
            "sampler": {"streams": 1, "helpers": helpers, "ms_per_batch": round(1e3 * st["sample_s"] / n, 4)},
            "lookahead_misses": st["lookahead_misses"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="rmat2m", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seed", type=int, default=824)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=25.0)
    ap.add_argument("--full-graph", action="store_true", help="rmat2m-embed: embed every node id")
    ap.add_argument("--embed-merge", type=int, default=2,
                    help="rmat2m-embed: reference batches per device launch (1 = one batch per launch)")
    ap.add_argument("--sustain", type=int, default=200,
                    help="steady-state steps after the measured ones (samplers running ahead), reported as `sustained`")
    ap.add_argument("--ar-buckets", type=int, default=None, choices=(1, 2),
                    help="N > 1: gradient all-reduce buckets (2, the default at N > 1: upper layers + classifier "
                         "under the layer-1 dW GEMM, then W1 in the row chunks its chunked dW GEMM completes, "
                         "GS_AR_W1_CHUNKS=2; 1: one all-reduce after the backward)")
    ap.add_argument("--ref-stream-steps", type=int, default=60,
                    help="N = 1: steps of the `reference_stream` window (the reference's single seed-824 random "
                         "stream, S = 1 with helper threads; 0 = skip)")
    ap.add_argument("--sampler-streams", type=int, default=None,
                    help="independent bit-exact sampler streams per GPU (1 = the reference's single stream; "
                         "default with helpers: min(8, (host cores per GPU - 2) / 2), two cores left for the "
                         "issuing thread and the HIP runtime / RCCL's proxy; without: min(12, cores per GPU - 3))")
    ap.add_argument("--no-warm", action="store_true",
                    help="skip the sampler threads' throwaway warm-up batch (A/B of the cold first batches)")
    ap.add_argument("--sampler", default="host", choices=("host", "device"),
                    help="device: every stream samples on the GPU (gs_dsampler, SURVEY §8 f-4), no host sampler "
                         "threads; default 1 stream (the reference's single random stream)")
    ap.add_argument("--sampler-depth", type=int, default=4,
                    help="pinned pack slots per sampler stream (how far each stream may run ahead)")
    ap.add_argument("--sampler-helpers", type=int, default=None,
                    help="helper threads per sampler stream (same draws; lower per-batch latency); "
                         "default 0: more streams instead (profiles/r06_sampler_layout_ab.txt)")
    args = ap.parse_args()
    per_gpu = host_cores() // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    # as given on the command line, before the training runner's defaults below
    # (the pubmed loop and the inference runner pick their own)
    args.helpers_cli, args.streams_cli, args.per_gpu = args.sampler_helpers, args.sampler_streams, per_gpu
    if args.sampler == "device":
        args.sampler_helpers = 0
        if args.sampler_streams is None:
            args.sampler_streams = 1
    if args.sampler_helpers is None:
        # streams without helpers: a helper shortens one batch (0.31-0.33 against
        # 0.45-0.48 ms in-bench) but halves the streams the cores hold, and at a
        # ~50 us step the pipeline needs batches per second, not latency: 12 streams
        # give 12.8-13.6 M roots/s of capacity against 10.8-11.7 M for 7 streams
        # + 7 helpers, at the same step rate (profiles/r06_sampler_layout_ab.txt)
        args.sampler_helpers = 0
    if args.sampler_streams is None:
        if args.sampler_helpers:  # two threads per stream, two cores for the issuing thread and the runtime
            args.sampler_streams = max(1, min(8, (per_gpu - 2) // (1 + args.sampler_helpers)))
        else:
            args.sampler_streams = max(1, min(12, per_gpu - 3))

    # the training layout needs S streams x (1 + helpers) sampler threads plus
    # two cores (the issuing thread, the HIP runtime / RCCL proxy); with fewer
    # host cores per GPU the sampler, not the GPU, sets the pace
    args.layout_cores = args.sampler_streams * (1 + args.sampler_helpers) + 2 if args.sampler == "host" else 2
    args.layout_short = args.sampler == "host" and (per_gpu < 8 or per_gpu < args.layout_cores)
    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["batch"] = args.batch
    if cfg.get("loop") == "apply_model":
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            raise SystemExit("the apply_model configs (pubmed, cora) run on one GPU")
        return run_apply_model_loop(args, cfg)
    if cfg.get("loop") == "embed":
        return run_embed(args, cfg)
    rank, world = train.init_distributed()
    if args.ar_buckets is None:
        args.ar_buckets = 2 if world > 1 else 1
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    wl = build_workload(cfg, device, args.seed, world)
    trainer = train.NativeTrainer(wl["graph"], wl["X"], wl["labels"], cfg["classes"], num_layers=2,
                                  hidden=128, fanouts=cfg["fanouts"], agg_func=cfg["agg"], seed=args.seed)
    rngs = [train.make_rng(args.seed, rank, w) for w in range(args.sampler_streams)]
    calib = min(50, args.steps)  # untimed steps after the measured ones that time the other kernels
    sustain = max(0, args.sustain)  # then a steady-state window (sampler threads running ahead)
    total_steps = args.warmup + 2 * args.steps + calib + sustain  # warmup, cold and steady windows, calib, sustain
    batches = []
    epoch = 0
    while len(batches) < total_steps:
        batches.extend(train.rank_batches(wl["candidates"], cfg["batch"], rank, world, args.seed + 1000, epoch))
        epoch += 1
    batches = batches[:total_steps]
    comm = train.Communicator(rank, world, device) if world > 1 else None
    # hold=True: the sampler threads start no batch past the release mark, so the
    # timed steps' batches are sampled inside the timed region (presampled_at_t0)
    runner = train.Runner(trainer, wl["graph"], batches, rngs, cfg["fanouts"], gcn=False,
                          fail_empty=cfg["agg"] == "MAX", comm=comm, hold=True, ar_buckets=args.ar_buckets,
                          helpers=args.sampler_helpers, warm=not args.no_warm, sampler=args.sampler,
                          depth=args.sampler_depth)
    elem = 2 if cfg["dtype"] == "bf16" else 4
    L = len(cfg["fanouts"])
    lib = gs._lib.lib()

    # warmup: every timer site armed; the site with the longest median launch
    # is the dominant kernel, the one timed inside the measured steps
    runner.release(args.warmup)
    gs._lib.check(lib.gs_trainer_time_kernels(trainer._h, (1 << len(SITES)) - 1, args.warmup))
    runner.run(args.warmup)
    torch.cuda.synchronize()
    warm = {site: kernel_times_ms(trainer, args.warmup, site) for site in SITES}
    names = {site: lib.gs_trainer_kernel_name(trainer._h, site).decode() for site in SITES}
    # dominant: the timed site with the largest average duration in the committed
    # rocprofv3 summary of this config (a stable choice: fwd, dW and top launches
    # lie within ~1 us of each other under events), else the longest warmup median
    prof_avg = {site: load_rocprof_avg(args.config, cfg["batch"], names[site]) for site in SITES}
    if all(prof_avg[site] for site in SITES if len(warm[site])):
        dominant = max((site for site in SITES if len(warm[site])), key=lambda site: prof_avg[site]["avg_us"])
        dominant_by = f"largest average launch in the committed rocprofv3 summary ({prof_avg[dominant]['source']})"
    else:
        dominant = max(SITES, key=lambda site: float(np.median(warm[site])) if len(warm[site]) else -1.0)
        dominant_by = "longest median launch (HIP events) over the warmup steps"
    if world > 1:
        dist.barrier()
    runner.stats(reset=True)
    no_timer = bool(os.environ.get("GS_BENCH_NO_TIMER"))  # A/B of the in-window timer's cost
    # an event-bound launch idles the queue a few us on either side of it
    # (rocprofv3 trace: 4.4 us each side): time one launch in `every` of the
    # measured steps, spread over both windows, not all of them (one in 4 cost
    # the 20-step line 2.4 % against no timer: 7.74 against 7.93 M, medians of
    # six rounds; one in 8 leaves 6 timed launches over the two 20-step windows)
    every = max(8, args.steps // 16)
    gs._lib.check(lib.gs_trainer_time_kernels_every(trainer._h, 0 if no_timer else 1 << dominant, 2 * args.steps,
                                                    every))

    def timed_window(wait_sampled):
        """K steps between barrier + synchronize on both sides; with
        wait_sampled the clock also runs until the sampler threads have
        finished as many new batches as the window consumed."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        s0, c0 = runner.progress()
        ta = time.perf_counter()
        if not wait_sampled:  # cold: the sampler threads start the window's batches now
            runner.release(total_steps)
        runner.run(args.steps)
        if wait_sampled:
            want = min(s0 + args.steps, total_steps)
            deadline = time.perf_counter() + 60.0
            # spin (no sleep: a 50 us sleep overshot the condition by up to ~0.1 ms of a
            # ~1.3 ms window); the sampler threads are native and need no GIL
            nap = float(os.environ.get("GS_BENCH_POLL_SLEEP", "0"))  # A/B of the poll
            while runner.progress()[0] < want:
                if time.perf_counter() > deadline:
                    raise SystemExit("bench: sampler threads stalled inside the timed window")
                if nap:
                    time.sleep(nap)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - ta
        s1, c1 = runner.progress()
        tt = torch.tensor([el], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item()), {"presampled_at_t0": s0 - c0, "sampled_in_timed_region": s1 - s0,
                                  "sampled_ahead_at_t1": s1 - c1}

    thr0 = cgroup_throttle()
    # cold window: nothing past the warmup batches sampled before t0, so the
    # window pays the pipeline fill (the first batch's whole sampling latency)
    cold_elapsed, cold_proof = timed_window(wait_sampled=False)
    cst = runner.stats(reset=True)  # the cold window's host stats; the line's own are the steady window's
    cold_proof.update(lookahead_misses=cst["lookahead_misses"], max_step_ms=round(1e3 * cst["max_step_s"], 3))
    # steady window (`value`): straight after it, the pipeline running as in
    # any later step of a training run; the clock stops only once the window
    # has also sampled as many new batches as it consumed, so the sampling
    # work of every step it counts is inside the timed region
    elapsed, proof = timed_window(wait_sampled=True)
    thr1 = cgroup_throttle()
    st = runner.stats()
    times = {} if no_timer else {dominant: kernel_times_ms(trainer, 2 * args.steps // every, dominant)}
    blocks = {} if no_timer else {dominant: block_stats_us(trainer, 2 * args.steps // every, dominant)}
    # calibration steps after the measured ones time the other sites (an
    # event-bound launch costs the stream a little: never inside the timed steps)
    runner.release(total_steps)
    others = sum(1 << site for site in SITES if site != dominant or no_timer)
    gs._lib.check(lib.gs_trainer_time_kernels(trainer._h, others, calib))
    runner.run(calib)
    torch.cuda.synchronize()
    for site in SITES:
        if site not in times:
            times[site] = kernel_times_ms(trainer, calib, site)
            blocks[site] = block_stats_us(trainer, calib, site)
    loss = float(trainer.loss.item())
    # steady state: the remaining batches, with the sampler threads free to run
    # ahead (released since the calibration steps); reported beside `value`
    # with its proof that the window sampled at least the batches it consumed
    sus = None
    if sustain:
        if world > 1:
            dist.barrier()
        runner.stats(reset=True)
        sthr0 = cgroup_throttle()
        ss0, sc0 = runner.progress()
        ts = time.perf_counter()
        runner.run(sustain)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        te = time.perf_counter() - ts
        ss1, sc1 = runner.progress()
        tt = torch.tensor([te], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        te = float(tt.item())
        sthr1 = cgroup_throttle()
        sst = runner.stats()
        ns = max(1, sst["steps"])
        sus = {"value": round(cfg["batch"] * sustain * world / te, 1), "unit": "root nodes/s", "steps": sustain,
               "ms_per_step": round(te / sustain * 1e3, 4), "sampled_ahead_at_start": ss0 - sc0,
               "sampled_in_window": ss1 - ss0, "sampled_ahead_at_end": ss1 - sc1,
               "lookahead_misses": sst["lookahead_misses"], "max_step_ms": round(1e3 * sst["max_step_s"], 3),
               "host_ms_per_step": {k: round(1e3 * sst[k + "_s"] / ns, 4)
                                    for k in ("sample", "wait", "wait_sample", "wait_ring", "wait_gather", "issue")},
               "cgroup_throttled_ms": (round((sthr1 - sthr0) / 1e3, 3) if sthr0 is not None else None)}
    value = cfg["batch"] * args.steps * world / elapsed
    sizes = st["hop_sizes_sum"] / max(1, st["steps"])  # mean (n_dst, n_pos, n_src, n_nbr) per hop
    ref_stream = None
    if world == 1 and args.ref_stream_steps > 0 and args.sampler == "host":
        runner.close()  # its sampler threads are done (the batch list is consumed)
        runner = None
        ref_stream = reference_stream_window(trainer, wl, cfg, args, batches)
    n_edges = float(sizes[:L, 1].sum()) * args.steps
    n1, e1 = float(sizes[L - 1, 0]), float(sizes[L - 1, 1])
    # the runner reserves id slots for the last hop's fanout: resolve, then agg_ids_kernel (timed)
    agg_bytes = agg1_ids_bytes(n1, e1, cfg["feat"], elem, cfg["fanouts"][-1])
    gemm_flops = 2.0 * n1 * (2 * cfg["feat"]) * 128  # 2·|L1|·2F·H per layer-1 GEMM

    # the BASELINE metric literally: sampled nodes (B + |L1| + |L0|, the
    # reference's nodes_batch_layers) per second over the steady window's batches
    w0 = args.warmup + args.steps  # the steady window's first batch
    fr = replay_frontiers(wl["graph"], batches, args.sampler_streams, cfg["fanouts"], args.seed, rank,
                          w0 + args.steps)[w0:]
    nodes_t = torch.tensor([float(fr.sum())], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(nodes_t)
    sampled_nodes_per_s = float(nodes_t.item()) / elapsed
    # sampler capacity: S streams, each a batch per mean sampling time
    per_batch_s = st["sample_s"] / max(1, st["steps"])
    cap_batches = args.sampler_streams / per_batch_s if per_batch_s > 0 else float("inf")
    produced = proof["sampled_in_timed_region"] / elapsed
    sampler_bound = args.layout_short or cap_batches * cfg["batch"] < 1.05 * value / world
    if sampler_bound and rank == 0:
        print(f"warning: sampler-bound layout: {args.per_gpu} host cores per GPU for {args.sampler_streams} "
              f"streams x (1 + {args.sampler_helpers}) threads + 2 (needs {args.layout_cores}); sampler capacity "
              f"{cap_batches * cfg['batch']:.0f} roots/s per GPU", file=sys.stderr)

    if rank == 0:
        rooflines = {}
        for site in SITES:
            tt = times.get(site)
            if tt is None or not len(tt):
                continue
            us = float(np.mean(tt)) * 1e3
            if site in (0, 3):
                nb = agg_bytes if site == 0 else top_bytes(cfg["batch"], float(sizes[0, 3]), 128, cfg["classes"])
                peak, unit, bound, scale = HBM_PEAK_GBS, "GB/s", "hbm", float(nb) / 1e9
                work = {"algo_bytes_per_launch": int(nb)}
            else:
                # the peak of the MFMA the kernel issues: the forward runs the config
                # dtype's MFMA (bf16 16x16x32 for bf16 features); the dW GEMM widens
                # bf16 operands to fp32 and runs the fp32 16x16x4 MFMA (exact
                # products), so its ceiling is the fp32 peak -- the config dtype's
                # peak and fraction are reported beside it
                mfma_dt = "fp32" if site == 2 else cfg["dtype"]
                peak, unit, bound, scale = MFMA_PEAK_TFS[mfma_dt], "TFLOP/s", "mfma", gemm_flops / 1e12
                work = {"algo_flops_per_launch": int(gemm_flops), "mfma_dtype": mfma_dt}
                if mfma_dt != cfg["dtype"]:
                    work.update(peak_config_dtype=MFMA_PEAK_TFS[cfg["dtype"]],
                                frac_config_dtype=round(scale / (us * 1e-6) / MFMA_PEAK_TFS[cfg["dtype"]], 4))
                mb = load_mfma_busy(args.config, names[site])
                work.update(mfma_busy=(mb["mfma_util"] if mb else None), mfma_busy_source=(mb["source"] if mb else None),
                            mfma_busy_dispatches=(mb["dispatches"] if mb else None))
            # `achieved` / `frac` on this run's own in-step timing of the kernel;
            # beside it the committed rocprofv3 average of the same kernel (the
            # same command under --kernel-trace --stats, profiles/) and whether
            # the two agree within ROCPROF_TOL (a stale profile or a slower
            # build shows up as a disagreement, never in `frac`)
            achieved = scale / (us * 1e-6)
            rp = prof_avg[site]
            achieved_rp = scale / (rp["avg_us"] * 1e-6) if rp else None
            tr = load_traffic(args.config, cfg["batch"], names[site])
            rooflines[SITE_NAMES[site]] = dict(
                bound=bound, achieved=round(achieved, 2), peak=peak, unit=unit, frac=round(achieved / peak, 4),
                traffic=(tr["hbm_bytes"] if tr else None), traffic_source=(tr["source"] if tr else None),
                traffic_dispatches=(tr["dispatches"] if tr else None),
                achieved_from="live in-step timing (avg_launch_us)",
                rocprof=rp,
                achieved_rocprof=(round(achieved_rp, 2) if rp else None),
                frac_rocprof=(round(achieved_rp / peak, 4) if rp else None),
                rocprof_agrees=(abs(us - rp["avg_us"]) <= ROCPROF_TOL * rp["avg_us"] if rp else None),
                kernel=names[site],
                role=SITE_ROLES[site], avg_launch_us=round(us, 2),
                timer=("kernel span (per-workgroup s_memrealtime stamps, min start .. max end)"
                       if site in (1, 2, 3) else "kernel-bound HIP events (hipExtLaunchKernelGGL)"),
                timed_in=(f"{len(tt)} of the measured steps of both windows (one in {every})" if site == dominant else f"{calib} calibration steps after them"),
                warmup_median_us=round(float(np.median(warm[site])) * 1e3, 2) if len(warm[site]) else None,
                workgroup_us=blocks.get(site), **work)
        roof = dict(rooflines[SITE_NAMES[dominant]])
        roof["dominant_by"] = dominant_by
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(wl, cfg, args.cpu_budget, args.seed)
        out = {
            "metric": "sampled nodes/sec (2-layer, fanout 25,10) at 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "root nodes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "sampled_nodes_per_s": round(sampled_nodes_per_s, 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": cfg["dtype"],
            "data": "synthetic (R-MAT graph, hashed U(-1,1) features, labels id%16)",
            "config": {"workload": f"{args.config}: R-MAT scale {cfg['scale']} "
                                   f"({wl['n']} ids), {cfg['pairs']} pairs, feat {cfg['feat']}, "
                                   f"fanout {tuple(cfg['fanouts'])}, {cfg['agg']}, B={cfg['batch']}/GPU",
                       "global_batch": cfg["batch"] * world, "parallelism": f"dp{world}",
                       "sampler_kind": args.sampler,
                       "sampler_streams_per_gpu": args.sampler_streams,
                       "sampler_helpers_per_stream": args.sampler_helpers,
                       "sampler_depth_per_stream": args.sampler_depth,
                       "sampler_contexts_warmed": not args.no_warm,
                       "sampled_nodes": {"per_step_mean": [round(float(x), 1) for x in fr.mean(0)],
                                         "fields": "B, |L1|, |L0| (unique frontiers, models.py:246-251)",
                                         "per_s": round(sampled_nodes_per_s, 1)},
                       "sampler": {"host_cores_per_gpu": args.per_gpu, "layout_cores": args.layout_cores,
                                   "ms_per_batch": round(per_batch_s * 1e3, 4),
                                   "capacity_batches_per_s": round(cap_batches, 1),
                                   "capacity_roots_per_s": round(cap_batches * cfg["batch"], 1),
                                   "produced_batches_per_s_in_window": round(produced, 1),
                                   "sampler_bound": bool(sampler_bound)},
                       "window": "steady (after a cold window of the same length; the clock waits until the "
                                 "window has sampled as many new batches as it consumed)",
                       **proof,
                       "cold_start": {"value": round(cfg["batch"] * args.steps * world / cold_elapsed, 1),
                                      "ms_per_step": round(cold_elapsed / args.steps * 1e3, 4), **cold_proof},
                       "allreduce_buckets": args.ar_buckets if world > 1 else 0,
                       "allreduce_w1_chunks": (int(os.environ.get("GS_AR_W1_CHUNKS", "2"))
                                               if world > 1 and args.ar_buckets == 2 else 0),
                       "sampled_edges_per_s": round(n_edges * world / elapsed, 1),
                       "graph_build_s": round(wl["t_graph"], 2), "final_loss": round(loss, 5),
                       "host_csr": "one per node, /dev/shm image mapped by every rank" if wl["csr_shared"]
                       else "built in-process",
                       "host_ms_per_step": {"sampler": round(1e3 * st["sample_s"] / max(1, st["steps"]), 3),
                                            "wait_for_batch": round(1e3 * st["wait_s"] / max(1, st["steps"]), 3),
                                            "issue": round(1e3 * st["issue_s"] / max(1, st["steps"]), 3),
                                            "wait_sample": round(1e3 * st["wait_sample_s"] / max(1, st["steps"]), 3),
                                            "wait_ring": round(1e3 * st["wait_ring_s"] / max(1, st["steps"]), 3),
                                            "wait_gather": round(1e3 * st["wait_gather_s"] / max(1, st["steps"]), 3),
                                            "lookahead_misses": st["lookahead_misses"],
                                            "issue_fwd_bwd": round(1e3 * st["fwd_bwd_s"] / max(1, st["steps"]), 3),
                                            "issue_update": round(1e3 * st["update_s"] / max(1, st["steps"]), 3),
                                            "max_step": round(1e3 * st["max_step_s"], 3)},
                       "cgroup_throttled_ms": (round((thr1 - thr0) / 1e3, 3) if thr0 is not None else None)},
            "roofline": roof,
            "roofline_kernels": rooflines,
            "sustained": sus,
            "reference_stream": ref_stream,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if runner is not None:
        runner.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
