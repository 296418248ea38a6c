"""Native supervised training step — the reference's per-batch loop
(utils.py:144-191: forward, log_softmax + NLL mean, backward, clip_grad_norm_(5)
per model, SGD lr=0.7) as one stream of HIP kernels over flat parameter and
gradient buffers, fed by a sampler thread, data-parallel over RCCL.

Parameter layout (one flat fp32 buffer, one all-reduce per step):
    [sage_layer1.weight | ... | sage_layerL.weight | layer.0.weight | layer.0.bias]
    groups for clipping: GraphSage = all SageLayer weights, Classification = rest
    (utils.py:185-186 clip each model separately).
Initialisation reproduces the reference modules' init under torch.manual_seed
(SageLayer xavier_uniform_ per layer, then Linear + xavier on its weight).
"""
import ctypes
import os
import queue
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from . import hip_ops as ops
from ._lib import check, lib
from .models import Classification, DeviceSample, SageLayer
from .sampler import RNG, sample


def reference_init(num_layers, input_size, hidden, n_classes, gcn=False, seed=824):
    """Weights exactly as main.py:41-58 would create them after torch.manual_seed(seed)."""
    torch.manual_seed(seed)
    layers = [SageLayer(input_size if i == 1 else hidden, hidden, gcn=gcn) for i in range(1, num_layers + 1)]
    cls = Classification(hidden, n_classes)
    return [l.weight.detach().clone() for l in layers], cls.layer[0].weight.detach().clone(), \
        cls.layer[0].bias.detach().clone()


class FlatParams:
    """Contiguous parameter + gradient buffers with named views."""

    def __init__(self, tensors, names, groups, device):
        sizes = [t.numel() for t in tensors]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self.params = torch.empty(int(self.offsets[-1]), dtype=torch.float32, device=device)
        self.grads = torch.zeros_like(self.params)
        self.names = names
        self.shapes = [tuple(t.shape) for t in tensors]
        for i, t in enumerate(tensors):
            self.view(i).copy_(t.to(device=device, dtype=torch.float32))
        self.group_off = np.array([self.offsets[g] for g in groups] + [self.offsets[-1]], np.int64)

    def view(self, i, grad=False):
        buf = self.grads if grad else self.params
        return buf[int(self.offsets[i]):int(self.offsets[i + 1])].view(self.shapes[i])

    def state_dict(self):
        return {n: self.view(i).detach().clone() for i, n in enumerate(self.names)}


class NativeTrainer:
    """Fused supervised GraphSAGE step on one GPU (one rank of data parallel)."""

    def __init__(self, graph, features, labels, n_classes, num_layers=2, hidden=128, fanouts=(10, 10),
                 agg_func="MEAN", gcn=False, lr=0.7, max_norm=5.0, seed=824, weights=None):
        if not features.is_cuda:
            raise RuntimeError("NativeTrainer runs on a HIP device")
        self.device = features.device
        self.graph, self.X = graph, features
        self.labels = labels.to(device=self.device, dtype=torch.int32)
        self.L, self.H, self.C = num_layers, hidden, n_classes
        self.fanouts = list(fanouts)
        self.agg, self.gcn, self.lr, self.max_norm = agg_func, gcn, lr, max_norm
        if weights is None:
            weights = reference_init(num_layers, features.shape[1], hidden, n_classes, gcn, seed)
        sage_w, cls_w, cls_b = weights
        names = [f"sage_layer{i}.weight" for i in range(1, num_layers + 1)] + ["layer.0.weight", "layer.0.bias"]
        self.p = FlatParams(list(sage_w) + [cls_w, cls_b], names, [0, num_layers], self.device)
        self.row_ptr, self.col = graph.device_csr(self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.clip_ws = torch.empty(65 * 2, dtype=torch.float32, device=self.device)
        X = self.X
        cfg = _lib.TrainerConfig(
            n_layers=num_layers, hidden=hidden, n_classes=n_classes, agg=ops.agg_op(agg_func), gcn=int(gcn),
            feat_dtype=_lib.GS_BF16 if X.dtype == torch.bfloat16 else _lib.GS_F32,
            feat_dim=X.shape[1], feat_ld=X.stride(0), X=X.data_ptr(), row_ptr=self.row_ptr.data_ptr(),
            col=self.col.data_ptr(), labels=self.labels.data_ptr(), params=self.p.params.data_ptr(),
            grads=self.p.grads.data_ptr(), lr=lr, max_norm=max_norm)
        h = ctypes.c_void_p()
        check(lib().gs_trainer_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        if lib().gs_trainer_n_params(h) != self.p.params.numel():
            raise RuntimeError("flat parameter layout mismatch")
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)

    def weights(self):
        return [self.p.view(i) for i in range(self.L)]

    def forward_backward(self, ds, roots_dev):
        """Loss (device scalar) and gradients into self.p.grads for one batch:
        one native call that issues every kernel of the step on the stream."""
        sizes, offs = ds.native_sizes()
        self._reserve_ws(sizes)
        check(lib().gs_trainer_forward_backward(
            self._h, ds.buf.data_ptr(), sizes.ctypes.data, offs.ctypes.data, roots_dev.data_ptr(),
            roots_dev.numel(), self._ws.data_ptr(), self._ws.numel(), self.loss.data_ptr(),
            _lib.stream_ptr(self.device)))
        return self.loss

    def _reserve_ws(self, sizes):
        need = int(lib().gs_trainer_ws_bytes(self._h, sizes.ctypes.data))
        if need < 0:
            check(_lib.GS_EINVAL)
        if self._ws.numel() < need:
            self._ws = torch.empty(int(need * 1.25) + (1 << 20), dtype=torch.uint8, device=self.device)

    def forward(self, ds, out):
        """GraphSage forward alone (models.py:241-269): the batch's embeddings
        into `out` ([n_roots, hidden] fp32, contiguous); no loss or backward."""
        if not (out.is_contiguous() and out.dtype == torch.float32 and out.shape[1] == self.H):
            raise ValueError("out must be a contiguous fp32 [n_roots, hidden] tensor")
        sizes, offs = ds.native_sizes()
        if out.shape[0] != sizes[0]:
            raise ValueError("out rows != batch roots")
        self._reserve_ws(sizes)
        check(lib().gs_trainer_forward(self._h, ds.buf.data_ptr(), sizes.ctypes.data, offs.ctypes.data,
                                       self._ws.data_ptr(), self._ws.numel(), out.data_ptr(),
                                       _lib.stream_ptr(self.device)))
        return out

    _OPTIONS = {"fused_bwd": _lib.GS_TOPT_FUSED_BWD, "top_launch": _lib.GS_TOPT_TOP_LAUNCH,
                "self_rows": _lib.GS_TOPT_SELF_ROWS, "defer_update": _lib.GS_TOPT_DEFER_UPDATE,
                "top_pair": _lib.GS_TOPT_TOP_PAIR}

    def set_option(self, name, value):
        """gs_trainer_set_option: switch an alternative of the step (fused_bwd,
        top_launch, self_rows, defer_update, top_pair; default all on except
        top_pair).
        fused_bwd, self_rows and defer_update are bitwise the default;
        top_launch and top_pair match it within fp32 rounding of their
        split-K orders."""
        check(lib().gs_trainer_set_option(self._h, self._OPTIONS[name], int(bool(value))))
        return self

    def capture(self, n_steps, batch):
        """Parity capture (tests): the next n_steps training steps' root
        embeddings [n_steps, batch, hidden] and flat gradients before their
        clip + SGD [n_steps, n_params] (gs_trainer_capture); returns both
        tensors, filled in stream order as the steps run."""
        emb = torch.zeros(n_steps, batch, self.H, dtype=torch.float32, device=self.device)
        grads = torch.zeros(n_steps, self.p.params.numel(), dtype=torch.float32, device=self.device)
        self._cap = (emb, grads)  # kept alive while the trainer may write them
        check(lib().gs_trainer_capture(self._h, emb.data_ptr(), batch * self.H, grads.data_ptr(), n_steps))
        return emb, grads

    def captured(self):
        return int(lib().gs_trainer_captured(self._h))

    def update(self, grad_scale=1.0):
        """gs_trainer_update: grads *= grad_scale, clip per model, SGD — what
        every rank runs after the gradient all-reduce (grad_scale = 1/world)."""
        check(lib().gs_trainer_update(self._h, float(grad_scale), self.clip_ws.data_ptr(),
                                      _lib.stream_ptr(self.device)))

    def defer(self, on):
        """gs_trainer_defer: from now on each update(1/W) after the gradient
        all-reduce is left pending and applied by the next forward (the
        runner's communicator path); defer(False) applies a pending update.
        Returns whether deferring took effect for this step shape."""
        active = ctypes.c_int32(0)
        check(lib().gs_trainer_defer(self._h, int(bool(on)), ctypes.byref(active), _lib.stream_ptr(self.device)))
        return bool(active.value)

    def apply_update(self, world_size=1, group=None):
        """All-reduce (sum) the flat gradients over ranks, then clip + SGD with 1/world."""
        if world_size > 1:
            dist.all_reduce(self.p.grads, group=group)
            check(lib().gs_trainer_update(self._h, 1.0 / world_size, self.clip_ws.data_ptr(),
                                          _lib.stream_ptr(self.device)))
        else:
            check(lib().gs_trainer_update_local(self._h, _lib.stream_ptr(self.device)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_trainer_destroy(h)
            self._h = None

    def step(self, ds, roots_dev, world_size=1, group=None):
        loss = self.forward_backward(ds, roots_dev)
        self.apply_update(world_size, group)
        return loss


# ------------------------------------------------------------ data pipeline
def rank_batches(candidates, batch_size, rank, world_size, seed, epoch=0):
    """Shuffle candidate roots (numpy, like sklearn.shuffle at utils.py:127) and
    deal batch i*world+rank to this rank: disjoint across ranks, B per rank."""
    perm = np.random.RandomState(seed + epoch).permutation(np.asarray(candidates, np.int64))
    n_steps = len(perm) // (batch_size * world_size)
    for i in range(n_steps):
        b = i * world_size + rank
        yield perm[b * batch_size:(b + 1) * batch_size]


def rank_seed(seed, rank, stream=0):
    """Sampler stream (rank, stream): random.seed(seed + rank + 64 * stream);
    rank 0 stream 0 is exactly the reference's random.seed(seed) stream."""
    return seed + rank + 64 * stream


class SampleInfo:
    """Sizes / pack offsets of one packed batch (what DeviceSample needs)."""

    def __init__(self, n_hops, sizes, offsets, used, n_roots):
        self.n_hops = n_hops
        self._sizes = [tuple(int(x) for x in sizes[4 * j:4 * j + 4]) for j in range(n_hops)]
        self.offsets = offsets.reshape(_lib.GS_MAX_HOPS, _lib.GS_PK_NFIELDS)[:n_hops].tolist()
        self.pack_total = int(used) - n_roots
        self.n_roots = n_roots

    def sizes(self, j):
        return self._sizes[j - 1]


class _SamplerWorker:
    """One RNG stream: samples its batches in order on a host thread (the GIL
    is released for the whole native sample+pack call) into a ring of pinned
    buffers; the consumer copies each to the device and recycles the slot."""

    def __init__(self, graph, rng, batches, fanouts, flags, depth):
        self.graph, self.rng, self.batches, self.flags = graph, rng, batches, flags
        self.fan = np.array([(-1 if k is None else int(k)) for k in fanouts], np.int32)
        self.q = queue.Queue(maxsize=depth)
        self.slots = [None] * (depth + 1)
        self.events = [None] * (depth + 1)
        self.free = queue.Queue()
        for i in range(depth + 1):
            self.free.put(i)
        self.sample_s = []
        self.stop = False
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        L = len(self.fan)
        try:
            for roots in self.batches:
                if self.stop:
                    break
                roots = np.ascontiguousarray(roots, dtype=np.int64)
                bound = int(lib().gs_sample_pack_bound(self.graph.handle, len(roots), self.fan.ctypes.data, L))
                slot = self.free.get()
                ev = self.events[slot]
                if ev is not None:
                    ev.synchronize()  # the previous H2D copy out of this slot is done
                buf = self.slots[slot]
                if buf is None or buf.numel() < bound:
                    buf = self.slots[slot] = torch.empty(bound, dtype=torch.int32, pin_memory=True)
                sizes = np.empty(4 * L, np.int64)
                offs = np.empty(_lib.GS_MAX_HOPS * _lib.GS_PK_NFIELDS, np.int64)
                used = ctypes.c_int64()
                t0 = time.perf_counter()
                check(lib().gs_sample_pack_run(self.graph.handle, self.rng._h, roots.ctypes.data, len(roots),
                                               self.fan.ctypes.data, L, self.flags, buf.data_ptr(), buf.numel(),
                                               sizes.ctypes.data, offs.ctypes.data, ctypes.byref(used)))
                self.sample_s.append(time.perf_counter() - t0)
                self.q.put((slot, SampleInfo(L, sizes, offs, used.value, len(roots)), offs, sizes))
        except BaseException as e:  # surface sampler errors in the consumer
            self.q.put(e)
        self.q.put(None)


class Prefetcher:
    """Host sampling pipelined with the GPU.  With one RNG (the default) the
    batches are sampled in order from that single stream — exactly the
    reference's sequence.  With `rngs` = S streams, stream w samples batches
    w, w+S, ... (each stream individually bit-exact with the reference seeded
    the same way, like S data-parallel ranks sharing this GPU); batches are
    still consumed in order."""

    def __init__(self, graph, rng, batches, fanouts, gcn, device, depth=3, rngs=None, fail_empty=False):
        self.device = torch.device(device)
        rngs = list(rngs) if rngs is not None else [rng]
        S = len(rngs)
        batches = list(batches)
        flags = (_lib.GS_SAMPLE_GCN if gcn else 0) | (4 if fail_empty else 0)
        self.workers = [_SamplerWorker(graph, rngs[w], batches[w::S], fanouts, flags, depth) for w in range(S)]
        self.i = 0

    @property
    def sample_s(self):
        return [t for w in self.workers for t in w.sample_s]

    def next(self):
        w = self.workers[self.i % len(self.workers)]
        item = w.q.get()
        if item is None:
            raise StopIteration
        if isinstance(item, BaseException):
            raise item
        self.i += 1
        slot, info, offs, sizes = item
        used = info.pack_total + info.n_roots
        dev = w.slots[slot][:used].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        w.events[slot] = ev
        w.free.put(slot)
        ds = DeviceSample(info, self.device, buf=dev)
        ds._native = (sizes, offs)
        return ds, dev[info.pack_total:used], info

    def __iter__(self):
        return self

    def __next__(self):
        return self.next()

    def close(self):
        for w in self.workers:
            w.stop = True


def init_distributed():
    """torch.distributed from torchrun env (RCCL on HIP devices); (rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not dist.is_initialized():
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend=backend)
    return rank, world


def make_rng(seed, rank=0, stream=0):
    return RNG(rank_seed(seed, rank, stream))


# ------------------------------------------------------------ native runner
class Communicator:
    """Native RCCL communicator for the runner's gradient all-reduce; the
    128-byte id is created on rank 0 and broadcast over torch.distributed."""

    def __init__(self, rank, world, device):
        self.world = world
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            check(lib().gs_comm_unique_id(uid.numpy().ctypes.data))
        if world > 1:
            t = uid.to(device)
            dist.broadcast(t, 0)
            uid = t.cpu().contiguous()
        h = ctypes.c_void_p()
        check(lib().gs_comm_create(uid.numpy().ctypes.data, world, rank, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h is not None and self._h.value:
            lib().gs_comm_destroy(self._h)
        self._h = None


class Runner:
    """The training loop as one native pipeline (gs_runner): S sampler
    threads, pinned pack rings, the next batch's device pull and layer-1
    gather on a high-priority side stream, and the fused
    step, all without Python per step.  `batches`: iterable of equal-size
    int64 root arrays consumed in order; `rngs`: one RNG per sampler stream
    (stream w samples batches w, w+S, ...).  Forward-only (`embed_out`) with
    `merge` = m > 1: each step is m consecutive batches in one pack and one
    forward; step u (batches u·m .. u·m+m-1) is sampled by stream u % S.
    `hold`: no batch is sampled before `release(mark)` allows it (measurement:
    proves a timed region sampled its own batches).  `ar_buckets=2` (with a
    communicator): the upper layers' + classifier gradients are all-reduced on
    a comm stream under the layer-1 weight-gradient GEMM, W1's after it.
    `helpers`: helper threads per sampler stream (gs_team; same draws, lower
    per-batch latency).  `warm`: every sampler thread samples one throwaway
    batch (its last, from a copy of its rng) before the constructor returns,
    so measured batches never pay a cold sampling context.
    `sampler="device"`: the streams sample on the GPU instead (SURVEY §8 f-4,
    gs_dsampler: one per stream, each on its own HIP stream), writing every
    pack straight into the device ring — no host sampler threads; the same
    packs and stream consumption as the host sampler.  The rngs are updated
    at ``sync_rngs()`` and ``close()``."""

    def __init__(self, trainer, graph, batches, rngs, fanouts, gcn=False, fail_empty=False, depth=4,
                 comm=None, embed_out=None, merge=1, hold=False, ar_buckets=1, helpers=0, warm=False,
                 sampler="host"):
        if sampler not in ("host", "device"):
            raise ValueError("sampler must be 'host' or 'device'")
        self.sampler = sampler
        self.trainer, self.graph = trainer, graph
        self.embed_out = embed_out
        self.rngs = list(rngs)
        self.batches = np.ascontiguousarray(np.stack([np.asarray(b, np.int64) for b in batches]))
        self.fanouts = np.ascontiguousarray(fanouts, dtype=np.int32)
        self._rng_ptrs = (ctypes.c_void_p * len(self.rngs))(*[r._h.value for r in self.rngs])
        self.comm = comm
        flags = (_lib.GS_SAMPLE_GCN if gcn else 0) | (4 if fail_empty else 0)
        cfg = _lib.RunnerConfig(
            graph=graph._h.value, trainer=trainer._h.value, batches=self.batches.ctypes.data,
            n_batches=self.batches.shape[0], batch=self.batches.shape[1], fanouts=self.fanouts.ctypes.data,
            n_hops=len(self.fanouts), flags=flags, n_streams=len(self.rngs),
            rngs=ctypes.cast(self._rng_ptrs, ctypes.c_void_p), depth=depth,
            comm=comm._h.value if comm is not None else None, world=comm.world if comm is not None else 1,
            hold=int(bool(hold)), ar_buckets=int(ar_buckets), helpers=int(helpers), warm=int(bool(warm)),
            device_sampler=int(sampler == "device"))
        if embed_out is not None:
            n_rows = self.batches.shape[0] * self.batches.shape[1]
            if not (embed_out.is_contiguous() and embed_out.dtype == torch.float32
                    and embed_out.device == trainer.device and embed_out.dim() == 2
                    and embed_out.shape[0] >= n_rows and embed_out.shape[1] == trainer.H):
                raise ValueError("embed_out must be a contiguous fp32 [n_batches * batch, hidden] device tensor")
            cfg.embed_out = embed_out.data_ptr()
            cfg.embed_ld = trainer.H
            cfg.merge = max(1, int(merge))
        elif merge > 1:
            raise ValueError("merge > 1 needs embed_out (forward-only)")
        self.merge = max(1, int(merge)) if embed_out is not None else 1
        h = ctypes.c_void_p()
        check(lib().gs_runner_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    def run(self, n_steps):
        """Issue the next n_steps steps (asynchronous on the device): training
        steps, or forward-only steps (of `merge` batches each) into embed_out."""
        check(lib().gs_runner_run(self._h, int(n_steps), self.trainer.loss.data_ptr(),
                                  _lib.stream_ptr(self.trainer.device)))
        return self.embed_out if self.embed_out is not None else self.trainer.loss

    def sync_rngs(self):
        """sampler="device": copy the device streams' states back into the rngs
        (every batch sampled so far, consumed or not)."""
        check(lib().gs_runner_sync_rngs(self._h))

    def release(self, mark):
        """hold=True runners: let the sampler threads start batches < mark."""
        check(lib().gs_runner_release(self._h, int(mark)))

    def progress(self):
        """(batches sampled so far, steps issued so far)."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check(lib().gs_runner_progress(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def stats(self, reset=False):
        st = _lib.RunnerStats()
        check(lib().gs_runner_stats_get(self._h, ctypes.byref(st)))
        if reset:
            lib().gs_runner_stats_reset(self._h)
        sizes = np.array(st.hop_sizes[:], dtype=np.float64).reshape(_lib.GS_MAX_HOPS, 4)
        return {"steps": st.steps, "wait_s": st.wait_s, "issue_s": st.issue_s, "sample_s": st.sample_s,
                "wait_sample_s": st.wait_sample_s, "wait_ring_s": st.wait_ring_s,
                "wait_gather_s": st.wait_gather_s, "fwd_bwd_s": st.fwd_bwd_s, "update_s": st.update_s,
                "max_step_s": st.max_step_s, "lookahead_misses": st.lookahead_misses, "hop_sizes_sum": sizes}

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_runner_destroy(h)
        self._h = None

    def __del__(self):
        self.close()


# ------------------------------------------------------- full-graph inference
class Embedder:
    """get_gnn_embeddings (utils.py:59-78) as one native pipeline: the
    training runner in forward-only mode (gs_runner_config.embed_out) over
    batches of `batch` ids, S sampler streams, the next batch's pull + layer-1
    gather under the current forward, embeddings written in place.

    `merge` = m consecutive batches share one pack and one forward launch
    sequence (each still sampled on its own, so each row equals its own
    batch's forward): the runner is host-issue bound at one 500-id batch per
    launch.  Stream w of `rngs` samples the groups w, w+S, ... (batch i on
    stream (i // m) % S); a trailing partial batch is sampled afterwards by
    the stream whose turn it is and run through NativeTrainer.forward.  With
    one stream that is exactly the reference's sequence of GraphSage calls on
    one `random` stream, for any m."""

    def __init__(self, graph, features, weights, fanouts, agg_func="MEAN", gcn=False, depth=4, merge=2, helpers=0):
        weights = [w.detach() for w in weights]
        H = weights[0].shape[0]
        dev = features.device
        dummy_cls = (torch.zeros(1, H, device=dev), torch.zeros(1, device=dev))
        self.trainer = NativeTrainer(graph, features, torch.zeros(1, dtype=torch.int32), 1,
                                     num_layers=len(weights), hidden=H, fanouts=fanouts, agg_func=agg_func,
                                     gcn=gcn, weights=(weights, *dummy_cls))
        self.graph, self.fanouts, self.gcn, self.agg = graph, list(fanouts), gcn, agg_func
        self.depth = depth
        self.merge = max(1, int(merge))
        self.helpers = int(helpers)  # gs_team helper threads per sampler stream (same draws)
        self.last_stats = None

    def embed(self, nodes, batch, rngs):
        """[len(nodes), hidden] fp32 embeddings on the device, row i = nodes[i]."""
        nodes = np.ascontiguousarray(nodes, dtype=np.int64).reshape(-1)
        rngs = list(rngs)
        n_full = len(nodes) // batch
        out = torch.empty(len(nodes), self.trainer.H, dtype=torch.float32, device=self.trainer.device)
        if n_full:
            r = Runner(self.trainer, self.graph, nodes[:n_full * batch].reshape(n_full, batch), rngs, self.fanouts,
                       gcn=self.gcn, fail_empty=self.agg == "MAX", depth=self.depth, embed_out=out,
                       merge=self.merge, helpers=self.helpers)
            try:
                r.run(-(-n_full // self.merge))
                self.last_stats = r.stats()
            finally:
                r.close()  # joins the sampler threads: every rng has advanced past its batches
        rest = nodes[n_full * batch:]
        if len(rest):
            s = sample(self.graph, rngs[(n_full // self.merge) % len(rngs)], rest, self.fanouts, gcn=self.gcn)
            if self.agg == "MAX" and any(s.n_empty(j) for j in range(1, s.n_hops + 1)):
                raise IndexError("MAX aggregation over an empty neighbourhood (reference: models.py:321-325)")
            self.trainer.forward(DeviceSample(s, self.trainer.device), out[n_full * batch:])
        return out
