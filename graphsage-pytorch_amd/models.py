"""Drop-in replacements for the reference's src/models.py modules.

Same constructor signatures, attributes, state_dict keys and forward contracts
as ``SageLayer`` (models.py:189-220), ``GraphSage`` (models.py:222-330) and
``Classification`` (models.py:8-27); the work runs through the native sampler
and the gfx950 kernels:

  GraphSage.forward(nodes_batch)
    host : sample all hops (bit-exact with the reference's `random` stream and
           set order; the module-global `random` state is consumed exactly as
           the reference consumes it), pack one int32 image, one H2D copy
    HIP  : per layer, segmented gather-aggregate (K-agg) + MFMA SageLayer
           (K-sage-linear); backward through the transposed neighbourhoods.

There is no CPU execution path: raw_features must live on a HIP device.
"""
import ctypes
import random as _pyrandom

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import hip_ops as ops
from .graph import CSRGraph
from .sampler import RNG, sample

PK = {  # field ids of the device pack
    "pos_ptr": _lib.GS_PK_POS_PTR, "pos": _lib.GS_PK_POS, "dst_ids": _lib.GS_PK_DST_IDS,
    "nbr_ptr": _lib.GS_PK_NBR_PTR, "nbr": _lib.GS_PK_NBR, "self": _lib.GS_PK_SELF,
    "tptr": _lib.GS_PK_TPTR, "tidx": _lib.GS_PK_TIDX,
}


class DeviceSample:
    """One batch's sampled computation graph resident on the device."""

    def __init__(self, s, device, buf=None):
        self.n_hops = s.n_hops
        self.sizes = [s.sizes(j) for j in range(1, s.n_hops + 1)]
        self.offsets = s.offsets
        if buf is None:
            host = s.pack(pin=torch.device(device).type == "cuda")
            buf = host.to(device, non_blocking=True)
        self.buf = buf

    def native_sizes(self):
        """(hop sizes [L][4], pack offsets [GS_MAX_HOPS][NFIELDS]) as int64 arrays."""
        if getattr(self, "_native", None) is None:
            sizes = np.array(self.sizes, np.int64).reshape(-1)
            offs = np.full((_lib.GS_MAX_HOPS, _lib.GS_PK_NFIELDS), -1, np.int64)
            offs[:self.n_hops] = np.array(self.offsets, np.int64)
            self._native = (sizes, offs.reshape(-1))
        return self._native

    def field(self, hop, name):
        """int32 view of `name` for hop (1-based)."""
        n_dst, n_pos, n_src, n_nbr = self.sizes[hop - 1]
        n = {"pos_ptr": n_dst + 1, "pos": n_pos, "dst_ids": n_dst, "nbr_ptr": n_dst + 1,
             "nbr": n_nbr, "self": n_dst, "tptr": n_src + 1, "tidx": n_nbr + n_dst}[name]
        off = self.offsets[hop - 1][PK[name]]
        if off < 0:
            raise KeyError(f"hop {hop} has no '{name}' on the device")
        return self.buf[off:off + n]


class _PackInfo:
    """Hop sizes / pack offsets of a pack written by gs_sample_pack_run*."""

    def __init__(self, n_hops, sizes, offsets):
        self.n_hops = n_hops
        self._sizes = [tuple(int(x) for x in sizes[4 * j:4 * j + 4]) for j in range(n_hops)]
        self.offsets = offsets.reshape(_lib.GS_MAX_HOPS, _lib.GS_PK_NFIELDS)[:n_hops].tolist()

    def sizes(self, j):
        return self._sizes[j - 1]


# ------------------------------------------------------------ shared compute
def sage_forward(ds, X, weights, agg_func, gcn, row_ptr, col, weights_lowp=None):
    """Bottom-up forward (models.py:255-267) over a DeviceSample.

    Returns (h_list, agg_list, argmax_list); h_list[-1] is [len(roots), H]."""
    L = ds.n_hops
    hs, aggs, ams = [], [], []
    # layer 1 reads the raw features through the last hop, expanded on device
    n_dst = ds.sizes[L - 1][0]
    dst = ds.field(L, "dst_ids")
    a1 = torch.empty(n_dst, X.shape[1], dtype=X.dtype, device=X.device)
    W1 = weights_lowp[0] if weights_lowp is not None else weights[0]
    h = torch.empty(n_dst, weights[0].shape[0], dtype=torch.float32, device=X.device)
    W1c = W1.detach().contiguous()
    if (ops.sage1_supported(X.dtype, X.shape[1], W1c.shape[0], gcn) and X.stride(1) == 1
            and X.stride(0) % (16 // X.element_size()) == 0 and X.data_ptr() % 16 == 0):
        # gather + concat-linear in one launch; the pack holds absolute CSR entries
        ops.sage1_fwd(agg_func, X, ds.field(L, "pos_ptr"), ds.field(L, "pos"), col, dst, W1c, a1, h, gcn=gcn)
    else:
        ops.agg_fwd(agg_func, X, ds.field(L, "pos_ptr"), ds.field(L, "pos"), a1,
                    row_ptr=None, col=col, dst_ids=dst, gcn=gcn)
        ops.sage_linear_fwd(a1, W1, h, Xs=None if gcn else X, sidx=dst)
    hs.append(h)
    aggs.append(a1)
    ams.append(None)
    for layer in range(2, L + 1):
        j = L - layer + 1
        n_dst = ds.sizes[j - 1][0]
        prev = hs[-1]
        a = torch.empty(n_dst, prev.shape[1], dtype=torch.float32, device=X.device)
        am = (torch.empty(n_dst, prev.shape[1], dtype=torch.int32, device=X.device)
              if agg_func == "MAX" else None)
        ops.agg_fwd(agg_func, prev, ds.field(j, "nbr_ptr"), ds.field(j, "nbr"), a, argmax=am)
        h = torch.empty(n_dst, weights[layer - 1].shape[0], dtype=torch.float32, device=X.device)
        ops.sage_linear_fwd(a, weights[layer - 1], h, Xs=None if gcn else prev, sidx=ds.field(j, "self"))
        hs.append(h)
        aggs.append(a)
        ams.append(am)
    return hs, aggs, ams


def sage_backward(ds, X, weights, agg_func, gcn, hs, aggs, ams, dout, dWs):
    """Autograd of sage_forward for the weights (raw features get no grad,
    models.py:234).  dWs[l] receives layer l+1's weight gradient."""
    L = ds.n_hops
    dH = dout
    relu = True
    for layer in range(L, 0, -1):
        j = L - layer + 1
        if layer == 1:
            x_in, sidx = X, ds.field(L, "dst_ids")
        else:
            x_in, sidx = hs[layer - 2], ds.field(j, "self")
        ops.sage_linear_bwd_weight(aggs[layer - 1], dH, hs[layer - 1], dWs[layer - 1],
                                   Xs=None if gcn else x_in, sidx=sidx, relu=relu)
        if layer == 1:
            break
        n_dst = ds.sizes[j - 1][0]
        H_in = hs[layer - 2].shape[1]
        dIn = torch.empty(n_dst, H_in if gcn else 2 * H_in, dtype=torch.float32, device=X.device)
        dSelf = None if gcn else dIn[:, :H_in]
        dA = dIn if gcn else dIn[:, H_in:]
        ops.sage_linear_bwd_input(dH, hs[layer - 1], weights[layer - 1], dA, dSelf=dSelf, relu=relu)
        dprev = torch.empty_like(hs[layer - 2])
        ops.agg_bwd(agg_func, ds.field(j, "tptr"), ds.field(j, "tidx"), ds.field(j, "nbr_ptr"), dA,
                    dprev, dSelf=dSelf, argmax=ams[layer - 1], Hprev=hs[layer - 2])
        dH = dprev
        relu = False  # dprev is already masked by relu'(h_{layer-1})


class _GraphSageFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ds, row_ptr, col, agg_func, gcn, X, *weights):
        lowp = None
        if X.dtype == torch.bfloat16:
            lowp = [ops.cast_bf16(weights[0].detach().contiguous(),
                                  torch.empty(weights[0].shape, dtype=torch.bfloat16, device=X.device))]
        ws = [w.detach().contiguous() for w in weights]
        hs, aggs, ams = sage_forward(ds, X, ws, agg_func, gcn, row_ptr, col, lowp)
        ctx.ds, ctx.agg, ctx.gcn = ds, agg_func, gcn
        ctx.save_for_backward(X, *ws)
        ctx.acts = (hs, aggs, ams)
        return hs[-1]

    @staticmethod
    def backward(ctx, dout):
        X, *ws = ctx.saved_tensors
        hs, aggs, ams = ctx.acts
        dWs = [torch.empty_like(w) for w in ws]
        sage_backward(ctx.ds, X, ws, ctx.agg, ctx.gcn, hs, aggs, ams, dout.contiguous().float(), dWs)
        ctx.acts = None
        return (None, None, None, None, None, None, *dWs)


class _SageLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, self_feats, agg_feats, weight, gcn):
        A = agg_feats.contiguous()
        Xs = None if gcn else self_feats.contiguous()
        W = weight.detach().contiguous()
        Wd = W if A.dtype == torch.float32 else W.to(A.dtype)
        out = torch.empty(A.shape[0], W.shape[0], dtype=torch.float32, device=A.device)
        ops.sage_linear_fwd(A, Wd, out, Xs=Xs)
        ctx.gcn = gcn
        ctx.save_for_backward(Xs if Xs is not None else A, A, W, out)
        return out

    @staticmethod
    def backward(ctx, dout):
        Xs, A, W, out = ctx.saved_tensors
        gcn = ctx.gcn
        dout = dout.contiguous().float()
        dW = torch.empty_like(W)
        ops.sage_linear_bwd_weight(A, dout, out, dW, Xs=None if gcn else Xs)
        d_self = d_agg = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            F = A.shape[1]
            dIn = torch.empty(A.shape[0], F if gcn else 2 * F, dtype=torch.float32, device=A.device)
            dS = None if gcn else dIn[:, :F]
            dA = dIn if gcn else dIn[:, F:]
            ops.sage_linear_bwd_input(dout, out, W, dA, dSelf=dS)
            d_agg = dA.to(A.dtype)
            d_self = None if gcn else dS.to(Xs.dtype)
        return d_self, d_agg, dW, None


class _AggregateFn(torch.autograd.Function):
    """GraphSage.aggregate on explicit neighbourhoods (API path)."""

    @staticmethod
    def forward(ctx, agg_func, X, nptr, nidx, tptr, tidx):
        n = nptr.numel() - 1
        out = torch.empty(n, X.shape[1], dtype=X.dtype, device=X.device)
        am = (torch.empty(n, X.shape[1], dtype=torch.int32, device=X.device)
              if agg_func == "MAX" and X.dtype == torch.float32 else None)
        ops.agg_fwd(agg_func, X, nptr, nidx, out, argmax=am)
        ctx.agg, ctx.n_src = agg_func, X.shape[0]
        ctx.save_for_backward(nptr, tptr, tidx)
        ctx.am = am
        return out

    @staticmethod
    def backward(ctx, dout):
        nptr, tptr, tidx = ctx.saved_tensors
        if ctx.agg == "MAX" and ctx.am is None:
            raise RuntimeError("MAX aggregate backward is implemented for float32 inputs")
        dX = torch.empty(ctx.n_src, dout.shape[1], dtype=torch.float32, device=dout.device)
        ops.agg_bwd(ctx.agg, tptr, tidx, nptr, dout.contiguous().float(), dX, argmax=ctx.am)
        return None, dX, None, None, None, None


# ------------------------------------------------------------------ modules
class SageLayer(nn.Module):
    """Encodes a node's features the 'convolutional' GraphSage way (models.py:189-220)."""

    def __init__(self, input_size, out_size, gcn=False):
        super().__init__()
        self.input_size = input_size
        self.out_size = out_size
        self.gcn = gcn
        self.weight = nn.Parameter(torch.FloatTensor(out_size, self.input_size if self.gcn else 2 * self.input_size))
        self.init_params()

    def init_params(self):
        for param in self.parameters():
            nn.init.xavier_uniform_(param)

    def forward(self, self_feats, aggregate_feats, neighs=None):
        return _SageLinearFn.apply(self_feats, aggregate_feats, self.weight, self.gcn)


class GraphSage(nn.Module):
    """GraphSage encoder (models.py:222-330) on the native sampler + HIP kernels.

    Extra keyword arguments (all optional, defaults reproduce the reference):
      fanouts : num_sample per hop, roots first (reference: 10 at every hop,
                models.py:277); None entries mean "all neighbours".
      rng     : a sampler.RNG to draw from instead of the module-global
                `random` (the reference always uses the global stream).
      sampler_helpers : helper threads for the forward's sampling (gs_team:
                the same draws from the same stream, bit-identical pack; the
                per-node sets and neighbour lists are built beside the draws).
                0 = none.  MAX keeps the team-less path, whose sample is
                complete before the empty-neighbourhood IndexError.
      device_sampler : sample on the GPU (sampler.DeviceSampler):
                the stream's state moves to the device and back around each
                forward, the pack is written in device memory — the same
                draws, pack and `random` state as the host sampler (fanouts
                1..32 before the last hop, <= 32 at it).  For large batches
                (an apply_model forward over an extended batch).
    """

    def __init__(self, num_layers, input_size, out_size, raw_features, adj_lists, device, gcn=False,
                 agg_func='MEAN', *, fanouts=None, rng=None, sampler_helpers=0, device_sampler=False):
        super().__init__()
        self.input_size = input_size
        self.out_size = out_size
        self.num_layers = num_layers
        self.gcn = gcn
        self.device = device
        self.agg_func = agg_func
        self.raw_features = raw_features
        self.adj_lists = adj_lists
        self.fanouts = list(fanouts) if fanouts is not None else [10] * num_layers
        if len(self.fanouts) != num_layers:
            raise ValueError("need one fanout per layer")
        self.rng = rng
        self.sampler_helpers = int(sampler_helpers)
        self._team = None       # gs_team handle (lazy)
        self._pin = None        # pinned pack buffer of the team path
        self._pin_ev = None     # its last H2D copy
        self._graph = adj_lists if isinstance(adj_lists, CSRGraph) else None
        self.device_sampler = bool(device_sampler)
        if self.device_sampler:
            ks = self.fanouts
            if any(k is None or int(k) > 32 for k in ks) or any(int(k) < 1 for k in ks[:-1]):
                raise ValueError("device_sampler: fanouts must be <= 32 (and >= 1 before the last hop)")
        self._dsampler = None   # sampler.DeviceSampler (lazy, grown with the batch)
        for index in range(1, num_layers + 1):
            layer_size = out_size if index != 1 else input_size
            setattr(self, 'sage_layer' + str(index), SageLayer(layer_size, out_size, gcn=self.gcn))

    def __getstate__(self):
        """Pickle support for torch.save(models) (utils.py:52): the native CSR
        is a derived cache and is rebuilt from adj_lists after loading."""
        if isinstance(self.adj_lists, CSRGraph) or self.rng is not None:
            raise TypeError("GraphSage built on a native CSRGraph / RNG handle cannot be pickled; "
                            "save its state_dict() instead")
        state = self.__dict__.copy()
        state["_graph"] = None
        state["_team"] = state["_pin"] = state["_pin_ev"] = state["_dsampler"] = None
        return state

    def __del__(self):
        t = getattr(self, "_team", None)
        if t is not None and t.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_team_destroy(t)
            self._team = None

    # -------------------------------------------------------------- helpers
    @property
    def graph(self):
        if self._graph is None:
            self._graph = CSRGraph.from_adj_lists(self.adj_lists, n_nodes=len(self.raw_features))
        return self._graph

    def _draw(self, roots, fanouts, full=False):
        rng = self.rng if self.rng is not None else RNG.from_python(_pyrandom)
        s = sample(self.graph, rng, roots, fanouts, gcn=self.gcn, full=full)
        if self.rng is None:
            rng.to_python(_pyrandom)
        return s

    def _draw_pack(self, roots, device):
        """The forward's sample as a device pack, drawn with the helper team
        (gs_sample_pack_run_multi_team) into a pinned buffer and copied
        up; the same draws and the same pack as DeviceSample(self._draw(...))."""
        lib = _lib.lib()
        if self._team is None:
            t = ctypes.c_void_p()
            _lib.check(lib.gs_team_create(self.sampler_helpers, ctypes.byref(t)))
            self._team = t
        fan = np.array([(-1 if k is None else int(k)) for k in self.fanouts], np.int32)
        roots = np.ascontiguousarray(roots, np.int64)
        L, n = len(fan), len(roots)
        bound = int(lib.gs_sample_pack_bound(self.graph.handle, n, fan.ctypes.data, L))
        if self._pin_ev is not None:
            self._pin_ev.synchronize()  # the previous copy out of the pinned buffer is done
        if self._pin is None or self._pin.numel() < bound:
            self._pin = torch.empty(bound, dtype=torch.int32, pin_memory=True)
        sizes = np.empty(4 * L, np.int64)
        offs = np.empty(_lib.GS_MAX_HOPS * _lib.GS_PK_NFIELDS, np.int64)
        used = ctypes.c_int64()
        rng = self.rng if self.rng is not None else RNG.from_python(_pyrandom)
        flags = _lib.GS_SAMPLE_GCN if self.gcn else 0
        _lib.check(lib.gs_sample_pack_run_multi_team(self.graph.handle, rng._h, roots.ctypes.data, n, n,
                                                     fan.ctypes.data, L, flags, self._pin.data_ptr(),
                                                     self._pin.numel(), sizes.ctypes.data, offs.ctypes.data,
                                                     ctypes.byref(used), self._team))
        if self.rng is None:
            rng.to_python(_pyrandom)
        dev = self._pin[:used.value].to(device, non_blocking=True)
        self._pin_ev = torch.cuda.Event()
        self._pin_ev.record()
        ds = DeviceSample(_PackInfo(L, sizes, offs), device, buf=dev)
        ds._native = (sizes, offs)
        return ds

    def _draw_device(self, roots, device):
        """The forward's sample drawn on the GPU (gs_dsampler): the stream's
        state in, the pack in device memory, the advanced state out — the
        draws, pack and `random` state of the host sampler."""
        from .sampler import DeviceSampler
        n = len(roots)
        dev = torch.device(device)
        if self._dsampler is None or self._dsampler_cap < n or self._dsampler.device != dev:
            cap = max(n, 512)
            self._dsampler = DeviceSampler(self.graph, self.fanouts, cap, gcn=self.gcn,
                                           fail_empty=self.agg_func == "MAX", device=dev)
            self._dsampler_cap = cap
        ds = self._dsampler
        rng = self.rng if self.rng is not None else RNG.from_python(_pyrandom)
        ds.set_rng(rng)
        try:
            pack, sizes, offs, used = ds.run(roots)
        except _lib.DeviceLimit:
            # the batch outgrew a device capacity (its rejection windows widen
            # with the frontier): `rng` is untouched, so the host sampler
            # draws the same sample from the same state
            return None
        except IndexError:
            # MAX over an empty neighbourhood: the reference raises after its
            # sampling consumed the stream (models.py:321-325)
            rng.setstate(*ds.get_rng())
            if self.rng is None:
                rng.to_python(_pyrandom)
            raise IndexError("MAX aggregation over an empty neighbourhood (reference: models.py:321-325)")
        rng.setstate(*ds.get_rng())
        if self.rng is None:
            rng.to_python(_pyrandom)
        L = len(self.fanouts)
        hs = np.zeros(4 * L, np.int64)
        hs[:] = np.asarray(sizes, np.int64).reshape(-1)[:4 * L]
        out = DeviceSample(_PackInfo(L, hs, np.asarray(offs, np.int64).reshape(-1)), device, buf=pack[:used])
        out._native = (hs, np.asarray(offs, np.int64).reshape(-1))
        return out

    @staticmethod
    def _roots(nodes_batch):
        if isinstance(nodes_batch, torch.Tensor):
            return nodes_batch.detach().cpu().numpy().astype(np.int64).reshape(-1)
        if isinstance(nodes_batch, np.ndarray):  # no per-element list (a 10k-id batch: ~1 ms)
            return np.ascontiguousarray(nodes_batch, dtype=np.int64).reshape(-1)
        return np.asarray(list(nodes_batch), dtype=np.int64).reshape(-1)

    # -------------------------------------------------------------- forward
    def forward(self, nodes_batch):
        """Embeddings [len(nodes_batch), out_size]; row i is nodes_batch[i]."""
        roots = self._roots(nodes_batch)
        X = self.raw_features
        if not isinstance(X, torch.Tensor) or not X.is_cuda:
            raise RuntimeError("graphsage_amd.GraphSage runs on a HIP device: raw_features must be a "
                               "cuda tensor (the reference's --cuda path, main.py:52)")
        if self.agg_func not in ("MEAN", "MAX"):
            raise ValueError(f"agg_func must be 'MEAN' or 'MAX', got {self.agg_func!r}")
        # the device sampler returns None for a batch past its capacities
        ds = self._draw_device(roots, X.device) if self.device_sampler else None
        if ds is None and self.sampler_helpers > 0 and self.agg_func == "MEAN":
            ds = self._draw_pack(roots, X.device)
        elif ds is None:
            s = self._draw(roots, self.fanouts)
            if self.agg_func == "MAX":
                for j in range(1, s.n_hops + 1):
                    if s.n_empty(j):
                        raise IndexError("MAX aggregation over an empty neighbourhood "
                                         "(reference: models.py:321-325)")
            ds = DeviceSample(s, X.device)
        row_ptr, col = self.graph.device_csr(X.device)
        weights = [getattr(self, 'sage_layer' + str(i)).weight for i in range(1, self.num_layers + 1)]
        Xc = X if X.is_contiguous() else X.contiguous()
        return _GraphSageFn.apply(ds, row_ptr, col, self.agg_func, self.gcn, Xc, *weights)

    # ------------------------------------------------ reference helper API
    def _nodes_map(self, nodes, hidden_embs, neighs):
        layer_nodes, samp_neighs, layer_nodes_dict = neighs
        assert len(samp_neighs) == len(nodes)
        return [layer_nodes_dict[x] for x in nodes]

    def _get_unique_neighs_list(self, nodes, num_sample=10):
        """(samp_neighs list of sets, {id: pos}, unique list) — models.py:277-289."""
        s = self._draw(self._roots(nodes), [num_sample], full=True)
        h = s.hop(1)
        samp = [set(x) for x in h.sets()]
        uniq = h.src_ids.tolist()
        return samp, dict(zip(uniq, range(len(uniq)))), uniq

    def aggregate(self, nodes, pre_hidden_embs, pre_neighs, num_sample=10):
        """models.py:291-330 on explicit neighbourhoods (API path)."""
        unique_nodes_list, samp_neighs, unique_nodes = pre_neighs
        assert len(nodes) == len(samp_neighs)
        assert all(nodes[i] in samp_neighs[i] for i in range(len(samp_neighs)))
        if not self.gcn:
            samp_neighs = [samp_neighs[i] - {nodes[i]} for i in range(len(samp_neighs))]
        direct = len(pre_hidden_embs) == len(unique_nodes)  # :300-303
        cols = [sorted(unique_nodes[n] for n in sn) for sn in samp_neighs]
        if self.agg_func == "MAX" and any(len(c) == 0 for c in cols):
            raise IndexError("MAX aggregation over an empty neighbourhood")
        rows = [c if direct else [unique_nodes_list[x] for x in c] for c in cols]
        nptr = np.zeros(len(rows) + 1, np.int32)
        nptr[1:] = np.cumsum([len(r) for r in rows])
        nidx = np.array([x for r in rows for x in r], np.int32)
        n_src = len(pre_hidden_embs)
        tcnt = np.zeros(n_src + 1, np.int64)
        np.add.at(tcnt, nidx.astype(np.int64) + 1, 1)
        tptr = np.cumsum(tcnt).astype(np.int32)
        order = np.argsort(nidx, kind="stable")
        dsts = np.repeat(np.arange(len(rows), dtype=np.int32), np.diff(nptr))
        tidx = dsts[order].astype(np.int32)
        dev = pre_hidden_embs.device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        X = pre_hidden_embs if pre_hidden_embs.is_contiguous() else pre_hidden_embs.contiguous()
        return _AggregateFn.apply(self.agg_func, X, t(nptr), t(nidx if len(nidx) else np.zeros(1, np.int32)),
                                  t(tptr), t(tidx if len(tidx) else np.zeros(1, np.int32)))


class Classification(nn.Module):
    """log_softmax(Linear(emb)) head (models.py:8-27); plain torch ops."""

    def __init__(self, emb_size, num_classes):
        super().__init__()
        self.layer = nn.Sequential(nn.Linear(emb_size, num_classes))
        self.init_params()

    def init_params(self):
        for param in self.parameters():
            if len(param.size()) == 2:
                nn.init.xavier_uniform_(param)

    def forward(self, embeds):
        return torch.log_softmax(self.layer(embeds), 1)
