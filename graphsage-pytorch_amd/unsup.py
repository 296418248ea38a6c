"""Drop-in ``UnsupervisedLoss`` (the reference's src/models.py:45-186).

``extend_nodes`` runs natively (host/unsup.cpp): the random walks, the
5-hop balls and ``random.sample`` over ``set(train) - ball`` draw from the
module-global ``random`` stream exactly as the reference does (same words, same
CPython set orders), so a GraphSage forward that follows sees the reference's
state.  ``get_loss_sage`` / ``get_loss_margin`` run as HIP kernels
(kernels/unsup.hip) over an index plan of the pairs, with a deterministic
backward into the embedding rows.

The pair containers the reference exposes (``positive_pairs``,
``negtive_pairs``, ``node_positive_pairs``, ``node_negtive_pairs``) are built
lazily from the native arrays on first access.
"""
import ctypes
import os
import random as _pyrandom

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr
from .graph import CSRGraph
from .sampler import RNG

KIND_SAGE, KIND_MARGIN = 0, 1
PARTS_WALKS, PARTS_NEG, PARTS_BOTH = 1, 2, 3


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def _pairs_list(arr):
    return [(int(a), int(b)) for a, b in arr.tolist()] if len(arr) else []


def _per_node(nodes, arr, cnt, keep=None):
    """dict node -> its slice of pairs, reference dict semantics (key at the
    first occurrence, value from the last)."""
    out = {}
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    pairs = arr.tolist()
    for i, v in enumerate(nodes.tolist()):
        if keep is not None and not keep[i]:
            continue
        out[int(v)] = [tuple(p) for p in pairs[off[i]:off[i + 1]]]
    return out


# Below this many ids the host's bit-parallel BFS beats the device one, whose
# launches and host round trips cost ~1 ms per batch (apply_model phases, num_neg
# 100, 16 host threads: Cora 2,708 ids host 0.44 ms / device 1.30 ms; Pubmed
# 19,717 ids host 8.7 ms / device 3.3 ms; tools/lab/pubmed_phases.py).  Both
# paths give identical results and leave the same stream state.
DEVICE_BALLS_MIN_NODES = 8192


def device_balls_default(device, n_nodes):
    """extend_nodes' balls on the GPU: HIP device and a graph of at least DEVICE_BALLS_MIN_NODES ids."""
    return torch.device(device).type == "cuda" and int(n_nodes) >= DEVICE_BALLS_MIN_NODES


class UnsupervisedLoss:
    """UnsupervisedLoss(adj_lists, train_nodes, device) — models.py:45-186.

    adj_lists may be the reference's dict of sets (adopted with its set
    layouts) or a CSRGraph.  ``rng``: a sampler.RNG to draw from instead of the
    module-global ``random`` (the reference always uses the global stream).
    ``device_balls``: grow extend_nodes' 5-hop balls and pick the far-list
    negatives on the GPU (gs_unsup_attach_device; same results and stream);
    default: when ``device`` is a HIP device and the graph has at least
    DEVICE_BALLS_MIN_NODES ids (``device_balls_default``)."""

    def __init__(self, adj_lists, train_nodes, device, *, rng=None, n_threads=None, device_balls=None):
        self.Q = 10
        self.N_WALKS = 6
        self.WALK_LEN = 1
        self.N_WALK_LEN = 5
        self.MARGIN = 3
        self.adj_lists = adj_lists
        self.train_nodes = train_nodes
        self.device = device
        self.target_nodes = None
        self.unique_nodes_batch = []
        self.rng = rng
        self.n_threads = n_threads or _threads()
        dev = torch.device(device) if device is not None else torch.device("cpu")
        self._reset_pairs()
        if isinstance(adj_lists, CSRGraph):
            self.graph = adj_lists
        else:
            keys = list(adj_lists.keys()) if hasattr(adj_lists, "keys") else range(len(adj_lists))
            tr = np.asarray(train_nodes, np.int64).reshape(-1)
            n = max(max(keys, default=-1), int(tr.max(initial=-1))) + 1
            self.graph = CSRGraph.from_adj_lists(adj_lists, n_nodes=n)
        self.device_balls = (device_balls_default(dev, self.graph.n_nodes) if device_balls is None
                             else bool(device_balls))
        self._h = None
        self._make_handle()

    # ------------------------------------------------------------ native
    def _make_handle(self):
        tr = np.ascontiguousarray(np.asarray(self.train_nodes, np.int64).reshape(-1))
        h = ctypes.c_void_p()
        check(lib().gs_unsup_create(self.graph.handle, ptr(tr), len(tr), self.N_WALKS, self.WALK_LEN,
                                    self.N_WALK_LEN, ctypes.byref(h)))
        self._h = h
        if self.device_balls:
            # the device half allocates on, and owns a stream of, the current
            # device: make it this module's device
            dev = torch.device(self.device)
            with torch.cuda.device(dev if dev.index is not None else torch.cuda.current_device()):
                check(lib().gs_unsup_attach_device(h, None))
        self._params = (self.N_WALKS, self.WALK_LEN, self.N_WALK_LEN)

    def _run(self, nodes, num_neg, parts):
        if self._params != (self.N_WALKS, self.WALK_LEN, self.N_WALK_LEN):
            lib().gs_unsup_destroy(self._h)
            self._make_handle()
        nodes = np.ascontiguousarray(np.asarray(nodes, np.int64).reshape(-1))
        rng = self.rng if self.rng is not None else RNG.from_python(_pyrandom)
        sizes = np.zeros(4, np.int64)
        try:
            check(lib().gs_unsup_extend(self._h, rng._h, ptr(nodes), len(nodes), int(num_neg), parts,
                                        self.n_threads, ptr(sizes)))
        finally:
            if self.rng is None:
                rng.to_python(_pyrandom)
        U, P, N, ok = (int(x) for x in sizes)
        uniq = np.zeros(max(U, 1), np.int64)
        pos = np.zeros((max(P, 1), 2), np.int64)
        neg = np.zeros((max(N, 1), 2), np.int64)
        pc, nc = np.zeros(max(len(nodes), 1), np.int64), np.zeros(max(len(nodes), 1), np.int64)
        hp = np.zeros(max(len(nodes), 1), np.uint8)
        check(lib().gs_unsup_fetch(self._h, ptr(uniq), ptr(pos), ptr(neg), ptr(pc), ptr(nc), ptr(hp)))
        n = len(nodes)
        return dict(nodes=nodes, unique=uniq[:U], pos=pos[:P], neg=neg[:N], pos_cnt=pc[:n], neg_cnt=nc[:n],
                    has_pos=hp[:n].astype(bool), ok=bool(ok))

    def _reset_pairs(self):
        self._pos_parts, self._neg_parts = [], []
        self._pos_cache = self._neg_cache = self._npos_cache = self._nneg_cache = None
        self._plan = None

    # --------------------------------------------- reference attributes
    # unique_nodes_batch (models.py:146) is the list the reference keeps; the
    # last extend_nodes holds it as an int64 array and builds the list on first
    # read (a 10k-id tolist is ~0.2 ms of a Pubmed step that never reads it).
    @property
    def unique_nodes_batch(self):
        if self._uniq_list is None:
            self._uniq_list = self._uniq_arr.tolist()
        return self._uniq_list

    @unique_nodes_batch.setter
    def unique_nodes_batch(self, v):
        self._uniq_list, self._uniq_arr = list(v), None

    def _unique_array(self):
        # once the list has been handed out it is the reference's attribute and
        # may have been edited in place: the losses read it, as models.py does
        if self._uniq_list is not None:
            self._uniq_arr = np.asarray(self._uniq_list, np.int64).reshape(-1)
        return self._uniq_arr

    @property
    def positive_pairs(self):
        if self._pos_cache is None:
            self._pos_cache = [p for r in self._pos_parts for p in _pairs_list(r["pos"])]
        return self._pos_cache

    @positive_pairs.setter
    def positive_pairs(self, v):
        self._pos_parts, self._pos_cache = [], list(v)

    @property
    def negtive_pairs(self):
        if self._neg_cache is None:
            self._neg_cache = [p for r in self._neg_parts for p in _pairs_list(r["neg"])]
        return self._neg_cache

    @negtive_pairs.setter
    def negtive_pairs(self, v):
        self._neg_parts, self._neg_cache = [], list(v)

    @property
    def node_positive_pairs(self):
        if self._npos_cache is None:
            d = {}
            for r in self._pos_parts:
                d.update(_per_node(r["nodes"], r["pos"], r["pos_cnt"], r["has_pos"]))
            self._npos_cache = d
        return self._npos_cache

    @node_positive_pairs.setter
    def node_positive_pairs(self, v):
        self._npos_cache = dict(v)

    @property
    def node_negtive_pairs(self):
        if self._nneg_cache is None:
            d = {}
            for r in self._neg_parts:
                d.update(_per_node(r["nodes"], r["neg"], r["neg_cnt"]))
            self._nneg_cache = d
        return self._nneg_cache

    @node_negtive_pairs.setter
    def node_negtive_pairs(self, v):
        self._nneg_cache = dict(v)

    # ------------------------------------------------ reference methods
    def extend_nodes(self, nodes, num_neg=6):
        """models.py:135-147: the batch extended by its walk positives and
        far negatives, as list(set(pos) | set(neg))."""
        self._extend(nodes, num_neg)
        return self.unique_nodes_batch

    def extend_nodes_array(self, nodes, num_neg=6):
        """extend_nodes with unique_nodes_batch returned as an int64 array (the
        same ids in the same order, no Python list; utils.train_step's path).
        The array is a read-only view: the losses read the ids back through
        the same buffer, so a caller cannot change them under the plan."""
        self._extend(nodes, num_neg)
        view = self._uniq_arr.view()
        view.flags.writeable = False
        return view

    def _extend(self, nodes, num_neg):
        self._reset_pairs()
        self.target_nodes = nodes
        r = self._run(nodes, num_neg, PARTS_BOTH)
        self._pos_parts, self._neg_parts = [r], [r]
        self._last = r
        self._uniq_arr, self._uniq_list = r["unique"], None
        assert r["ok"], "set(target_nodes) < set(unique_nodes_batch) failed (models.py:147)"

    def get_positive_nodes(self, nodes):
        return self._run_random_walks(nodes)

    def get_negtive_nodes(self, nodes, num_neg):
        r = self._run(nodes, num_neg, PARTS_NEG)
        self._neg_parts.append(r)
        self._neg_cache = self._nneg_cache = None
        self._plan = None
        return self.negtive_pairs

    def _run_random_walks(self, nodes):
        r = self._run(nodes, 0, PARTS_WALKS)
        self._pos_parts.append(r)
        self._pos_cache = self._npos_cache = None
        self._plan = None
        return self.positive_pairs

    # ------------------------------------------------------------ losses
    def _device_plan(self, device):
        """(plan int32 tensor on device, dims) for the last extend_nodes."""
        if self._plan is not None and self._plan[0].device == device:
            return self._plan
        if len(self._pos_parts) != 1 or len(self._neg_parts) != 1 or self._pos_parts[0] is not self._neg_parts[0]:
            raise RuntimeError("device losses need the pairs of one extend_nodes call")
        dims = np.zeros(6, np.int64)
        used = ctypes.c_int64()
        check(lib().gs_unsup_loss_plan(self._h, None, 0, ptr(dims), ctypes.byref(used)))
        host = torch.empty(max(int(used.value), 1), dtype=torch.int32,
                           pin_memory=torch.device(device).type == "cuda")
        check(lib().gs_unsup_loss_plan(self._h, ptr(host), host.numel(), ptr(dims), ctypes.byref(used)))
        self._plan = (host.to(device, non_blocking=True), dims)
        return self._plan

    def _loss(self, embeddings, nodes, kind):
        uniq = self._unique_array()
        assert len(embeddings) == len(uniq)
        nodes = np.asarray(nodes).reshape(-1)
        if len(nodes) > len(uniq):  # the reference indexes unique_nodes_batch[i] for every i
            raise IndexError("list index out of range")
        assert np.array_equal(nodes.astype(np.int64), uniq[:len(nodes)])
        if not isinstance(embeddings, torch.Tensor) or not embeddings.is_cuda:
            raise RuntimeError("UnsupervisedLoss losses run on a HIP device (cuda embeddings)")
        plan, dims = self._device_plan(embeddings.device)
        M, P, N, U, n_pos_keys, n_neg_keys = (int(x) for x in dims)
        assert n_pos_keys == n_neg_keys
        if M == 0:
            raise ValueError("torch.cat(): expected a non-empty list of Tensors")
        loss = _UnsupLossFn.apply(embeddings, plan, (M, P, N, U), kind, float(self.Q), float(self.MARGIN))
        return loss if kind == KIND_SAGE else loss.view(1)

    def get_loss_sage(self, embeddings, nodes):
        """models.py:65-96."""
        return self._loss(embeddings, nodes, KIND_SAGE)

    def get_loss_margin(self, embeddings, nodes):
        """models.py:98-132."""
        return self._loss(embeddings, nodes, KIND_MARGIN)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_unsup_destroy(h)
            self._h = None


class _UnsupLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb, plan, dims, kind, q, margin):
        M, P, N, U = dims
        E = emb.detach()
        if E.dtype != torch.float32:
            raise TypeError("embeddings must be float32")
        if E.stride(1) != 1 or E.stride(0) % 4 or E.data_ptr() % 16:
            E = E.contiguous()
        D = E.shape[1]
        ws = torch.empty(int(lib().gs_unsup_loss_ws_floats(M, P, N)), dtype=torch.float32, device=E.device)
        loss = torch.empty((), dtype=torch.float32, device=E.device)
        check(lib().gs_unsup_loss_fwd(kind, M, P, N, U, D, E.data_ptr(), E.stride(0), plan.data_ptr(), q, margin,
                                      loss.data_ptr(), ws.data_ptr(), _lib.stream_ptr(E.device)))
        ctx.save_for_backward(E, plan, ws)
        ctx.dims = dims
        return loss

    @staticmethod
    def backward(ctx, dloss):
        E, plan, ws = ctx.saved_tensors
        M, P, N, U = ctx.dims
        dl = dloss.detach().reshape(1).to(torch.float32).contiguous()
        dE = torch.empty_like(E)
        check(lib().gs_unsup_loss_bwd(M, P, N, U, E.shape[1], E.data_ptr(), E.stride(0), plan.data_ptr(),
                                      ws.data_ptr(), dl.data_ptr(), dE.data_ptr(), dE.stride(0),
                                      _lib.stream_ptr(E.device)))
        return dE, None, None, None, None, None
