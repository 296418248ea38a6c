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
        need = int(lib().gs_trainer_ws_bytes(self._h, sizes.ctypes.data))
        if need < 0:
            check(_lib.GS_EINVAL)
        if self._ws.numel() < need:
            self._ws = torch.empty(int(need * 1.25) + (1 << 20), dtype=torch.uint8, device=self.device)
        check(lib().gs_trainer_forward_backward(
            self._h, ds.buf.data_ptr(), sizes.ctypes.data, offs.ctypes.data, roots_dev.data_ptr(),
            roots_dev.numel(), self._ws.data_ptr(), self._ws.numel(), self.loss.data_ptr(),
            _lib.stream_ptr(self.device)))
        return self.loss

    def apply_update(self, world_size=1, group=None):
        """All-reduce (sum) the flat gradients over ranks, then clip + SGD with 1/world."""
        if world_size > 1:
            dist.all_reduce(self.p.grads, group=group)
        check(lib().gs_trainer_update(self._h, 1.0 / world_size, self.clip_ws.data_ptr(),
                                      _lib.stream_ptr(self.device)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
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


def rank_seed(seed, rank):
    """Sampler stream of a rank: random.seed(seed + rank) — rank 0 == the reference's stream."""
    return seed + rank


class Prefetcher:
    """Samples batch i+1.. on a host thread (GIL released inside the native
    sampler) into a ring of pinned buffers while the GPU runs batch i."""

    def __init__(self, graph, rng, batches, fanouts, gcn, device, depth=3):
        self.graph, self.rng, self.fanouts, self.gcn = graph, rng, list(fanouts), gcn
        self.device = torch.device(device)
        self.q = queue.Queue(maxsize=depth)
        self.slots = [None] * (depth + 1)
        self.events = [None] * (depth + 1)
        self.free = queue.Queue()
        for i in range(depth + 1):
            self.free.put(i)
        self._it = iter(batches)
        self._stop = False
        self.sample_s = []  # host sampler seconds per batch
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        try:
            for roots in self._it:
                if self._stop:
                    break
                t0 = time.perf_counter()
                s = sample(self.graph, self.rng, roots, self.fanouts, gcn=self.gcn)
                self.sample_s.append(time.perf_counter() - t0)
                slot = self.free.get()
                ev = self.events[slot]
                if ev is not None:
                    ev.synchronize()  # the previous H2D copy out of this slot is done
                need = s.pack_total + len(roots)
                buf = self.slots[slot]
                if buf is None or buf.numel() < need:
                    buf = self.slots[slot] = torch.empty(int(need * 1.25) + 1024, dtype=torch.int32,
                                                         pin_memory=True)
                s.pack_into(buf)
                buf[s.pack_total:need].copy_(torch.from_numpy(np.asarray(roots, np.int32)))
                self.q.put((s, slot, need, len(roots)))
        except BaseException as e:  # surface sampler errors in the consumer
            self.q.put(e)
        self.q.put(None)

    def next(self):
        item = self.q.get()
        if item is None:
            raise StopIteration
        if isinstance(item, BaseException):
            raise item
        s, slot, need, B = item
        dev = self.slots[slot][:need].to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[slot] = ev
        self.free.put(slot)
        ds = DeviceSample(s, self.device, buf=dev)
        return ds, dev[s.pack_total:need], s

    def __iter__(self):
        return self

    def __next__(self):
        return self.next()

    def close(self):
        self._stop = True


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


def make_rng(seed, rank=0):
    return RNG(rank_seed(seed, rank))
