"""Bit-exact neighbour sampling (models.py:277-289) behind the C-ABI.

``RNG`` is an MT19937 stream interchangeable with CPython's ``random``
(``from_python`` / ``to_python`` move the module-global state in and out, so
a forward consumes exactly the words the reference's forward would, also when
interleaved with other ``random`` users such as UnsupervisedLoss).

``sample`` runs every hop of a forward; the result holds the host views
(frontiers in CPython set order, sampled sets) and packs the int32 image the
kernels read into one buffer for a single host->device copy.
"""
import array as _array
import ctypes
import random as _pyrandom

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr


class RNG:
    """CPython 3.10 ``random.Random`` word stream (native)."""

    def __init__(self, seed=None):
        h = ctypes.c_void_p()
        check(lib().gs_rng_create(ctypes.byref(h)))
        self._h = h
        if seed is not None:
            self.seed(seed)

    def seed(self, n):
        """random.seed(n) for an int n (init_by_array over abs(n)'s 32-bit words)."""
        n = abs(int(n))
        words = []
        while True:
            words.append(n & 0xFFFFFFFF)
            n >>= 32
            if n == 0:
                break
        key = np.array(words, np.uint32)
        check(lib().gs_rng_seed_words(self._h, ptr(key), len(key)))
        return self

    def getstate(self):
        mt = np.zeros(624, np.uint32)
        pos = ctypes.c_int64()
        check(lib().gs_rng_get_state(self._h, ptr(mt), ctypes.byref(pos)))
        return mt, int(pos.value)

    def setstate(self, mt, pos):
        mt = np.ascontiguousarray(mt, dtype=np.uint32)
        if mt.shape != (624,):
            raise ValueError("MT19937 state must have 624 words")
        check(lib().gs_rng_set_state(self._h, ptr(mt), int(pos)))
        return self

    @classmethod
    def from_python(cls, r=_pyrandom):
        ver, internal, _gauss = r.getstate()
        if ver != 3:
            raise ValueError("unsupported random state version")
        out = cls()
        # array.array('I') takes the tuple's ints in one C loop (np.array: ~3x slower)
        out.setstate(np.frombuffer(_array.array("I", internal[:624]), np.uint32), internal[624])
        return out

    def to_python(self, r=_pyrandom):
        ver, _old, gauss = r.getstate()
        mt, pos = self.getstate()
        r.setstate((ver, tuple(mt.tolist()) + (pos,), gauss))

    # ----- known-answer helpers (tests / extend_nodes host code)
    def getrandbits(self, k, count=1):
        out = np.zeros(count, np.uint32)
        check(lib().gs_rng_getrandbits(self._h, int(k), int(count), ptr(out)))
        return out

    def randbelow(self, n, count=1):
        out = np.zeros(count, np.uint32)
        check(lib().gs_rng_randbelow(self._h, int(n), int(count), ptr(out)))
        return out

    def sample_positions(self, n, k):
        out = np.zeros(max(int(k), 1), np.int64)
        check(lib().gs_rng_sample_positions(self._h, int(n), int(k), ptr(out)))
        return out[:int(k)]

    def choice_position(self, n):
        out = ctypes.c_int64()
        check(lib().gs_rng_choice_position(self._h, int(n), ctypes.byref(out)))
        return int(out.value)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_rng_destroy(h)
            self._h = None


def pyset_union_of_lists(lists):
    """list(set.union(*[set(l) for l in lists])) via the native emulator."""
    lens = [len(l) for l in lists]
    p = np.zeros(len(lists) + 1, np.int64)
    p[1:] = np.cumsum(lens)
    items = np.array([x for l in lists for x in l], np.int64) if p[-1] else np.zeros(1, np.int64)
    out = np.zeros(max(int(p[-1]), 1), np.int64)
    n = ctypes.c_int64()
    check(lib().gs_pyset_union_of_lists(ptr(items), ptr(p), len(lists), ptr(out), ctypes.byref(n)))
    return out[:n.value]


def _arr(p, n, ct):
    if n <= 0 or not p:
        return np.zeros(0, np.int64 if ct is ctypes.c_int64 else np.int32)
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ct)), shape=(n,)).copy()


class Hop:
    """Host view of one hop (numpy copies)."""

    def __init__(self, v):
        self.n_dst, self.n_pos = int(v.n_dst), int(v.n_pos)
        self.n_src, self.n_nbr = int(v.n_src), int(v.n_nbr)
        self.n_empty = int(v.n_empty)
        self.dst_ids = _arr(v.dst_ids, self.n_dst, ctypes.c_int64)
        self.pos_ptr = _arr(v.pos_ptr, self.n_dst + 1, ctypes.c_int32)
        self.pos = _arr(v.pos, self.n_pos, ctypes.c_int32)
        self.materialised = self.n_src >= 0
        if self.materialised:
            self.src_ids = _arr(v.src_ids, self.n_src, ctypes.c_int64)
            self.nbr_ptr = _arr(v.nbr_ptr, self.n_dst + 1, ctypes.c_int32)
            self.nbr = _arr(v.nbr, self.n_nbr, ctypes.c_int32)
            self.self_local = _arr(v.self_local, self.n_dst, ctypes.c_int32)
            self.set_ptr = _arr(v.set_ptr, self.n_dst + 1, ctypes.c_int32)
            n_items = int(self.set_ptr[-1]) if self.n_dst else 0
            self.set_items = _arr(v.set_items, n_items, ctypes.c_int64)

    def sets(self):
        """samp_neighs as ordered lists (iteration order of the reference's sets)."""
        return [self.set_items[self.set_ptr[i]:self.set_ptr[i + 1]].tolist() for i in range(self.n_dst)]


class Sample:
    """All hops of one forward's sampling (a native gs_sample handle)."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)
        nh = ctypes.c_int32()
        check(lib().gs_sample_n_hops(self._h, ctypes.byref(nh)))
        self.n_hops = int(nh.value)
        self._hops = {}
        lay = _lib.PackLayout()
        check(lib().gs_sample_pack_layout(self._h, ctypes.byref(lay)))
        self.pack_total = int(lay.total)
        self.offsets = [[int(lay.off[j][f]) for f in range(_lib.GS_PK_NFIELDS)]
                        for j in range(self.n_hops)]
        self._sizes = []
        self._empty = []
        for j in range(1, self.n_hops + 1):
            v = _lib.HopView()
            check(lib().gs_sample_hop(self._h, j, ctypes.byref(v)))
            self._sizes.append((int(v.n_dst), int(v.n_pos), int(v.n_src), int(v.n_nbr)))
            self._empty.append(int(v.n_empty))

    def hop(self, j):
        """Host view of hop j (1 = the roots' hop)."""
        if j not in self._hops:
            v = _lib.HopView()
            check(lib().gs_sample_hop(self._h, int(j), ctypes.byref(v)))
            self._hops[j] = Hop(v)
        return self._hops[j]

    def sizes(self, j):
        """(n_dst, n_pos, n_src, n_nbr) of hop j."""
        return self._sizes[j - 1]

    def n_empty(self, j):
        """Destinations of hop j with an empty neighbourhood after the self rule."""
        return self._empty[j - 1]

    def pack_into(self, buf):
        """Write the device image into `buf` (int32 tensor / array, >= pack_total)."""
        if buf.numel() < self.pack_total:
            raise ValueError("pack buffer too small")
        check(lib().gs_sample_pack(self._h, ptr(buf), int(buf.numel())))

    def pack(self, pin=False):
        buf = torch.empty(max(self.pack_total, 1), dtype=torch.int32, pin_memory=pin)
        self.pack_into(buf)
        return buf

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_sample_destroy(h)
            self._h = None


def sample(graph, rng, roots, fanouts, gcn=False, full=False):
    """Sample every hop of one forward from `roots` (consumes `rng`)."""
    roots = np.ascontiguousarray(np.asarray(roots).reshape(-1), dtype=np.int64)
    fan = np.array([(-1 if k is None else int(k)) for k in fanouts], np.int32)
    flags = (_lib.GS_SAMPLE_GCN if gcn else 0) | (_lib.GS_SAMPLE_FULL if full else 0)
    h = ctypes.c_void_p()
    check(lib().gs_sample_run(graph.handle, rng._h, ptr(roots), len(roots), ptr(fan), len(fan),
                              flags, ctypes.byref(h)))
    return Sample(h.value)


class DeviceSampler:
    """The hop loop of GraphSage.forward (models.py:246-251 over
    _get_unique_neighs_list, :277-289) on the GPU: a device
    copy of the graph and a device MT19937 stream produce the same int32 pack
    as ``sample(...).pack()`` — bit for bit — directly in device memory, and
    advance the stream exactly as the reference's ``random`` would.

    ``rng`` moves between host and device with ``set_rng`` / ``get_rng``
    (``RNG`` objects or ``random.getstate()``-style (mt, pos) pairs)."""

    def __init__(self, graph, fanouts, max_roots, gcn=False, fail_empty=False, device=None):
        from ._lib import GS_SAMPLE_GCN
        self.fanouts = np.ascontiguousarray(fanouts, np.int32)
        flags = (GS_SAMPLE_GCN if gcn else 0) | (4 if fail_empty else 0)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("DeviceSampler runs on a HIP device")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().gs_dsampler_create(graph._h, ptr(self.fanouts), len(self.fanouts), int(max_roots), flags,
                                           ctypes.byref(h)))
        self._h = h
        self.graph = graph  # keep the host graph alive (pack bounds)
        self.n_hops = len(self.fanouts)

    def set_rng(self, rng):
        mt, pos = rng.getstate() if isinstance(rng, RNG) else rng
        mt = np.ascontiguousarray(mt, np.uint32)
        check(lib().gs_dsampler_set_rng(self._h, ptr(mt), int(pos), _lib.stream_ptr(self.device)))

    def get_rng(self):
        mt = np.zeros(624, np.uint32)
        pos = ctypes.c_int64()
        check(lib().gs_dsampler_get_rng(self._h, ptr(mt), ctypes.byref(pos), _lib.stream_ptr(self.device)))
        return mt, int(pos.value)

    def words(self, n):
        out = np.zeros(max(int(n), 1), np.uint32)
        check(lib().gs_dsampler_words(self._h, int(n), ptr(out), _lib.stream_ptr(self.device)))
        return out[:int(n)]

    def pack_bound(self, n_roots):
        return int(lib().gs_dsampler_pack_bound(self._h, int(n_roots)))

    def run(self, roots, pack=None):
        """Sample one batch; returns (pack, hop_sizes[n_hops, 4], offsets[8, 8], used)."""
        if not isinstance(roots, torch.Tensor):
            roots = torch.as_tensor(np.asarray(roots, np.int64).astype(np.int32))
        # device pointers only: a CPU or strided roots tensor would hand the
        # kernels host memory or the wrong ids
        roots = roots.to(device=self.device, dtype=torch.int32).contiguous().view(-1)
        n = int(roots.numel())
        if pack is None:
            pack = torch.zeros(self.pack_bound(n), dtype=torch.int32, device=self.device)
        elif not (isinstance(pack, torch.Tensor) and pack.dtype == torch.int32 and pack.is_contiguous()
                  and pack.device == self.device):
            raise ValueError(f"pack must be a contiguous int32 tensor on {self.device}")
        check(lib().gs_dsampler_run(self._h, ptr(roots), n, ptr(pack), int(pack.numel()), _lib.stream_ptr(self.device)))
        hs = np.zeros(4 * _lib.GS_MAX_HOPS, np.int64)
        off = np.zeros(_lib.GS_MAX_HOPS * _lib.GS_PK_NFIELDS, np.int64)
        used = ctypes.c_int64()
        check(lib().gs_dsampler_result(self._h, ptr(hs), ptr(off), ctypes.byref(used)))
        return pack, hs.reshape(-1, 4)[:self.n_hops], off.reshape(_lib.GS_MAX_HOPS, _lib.GS_PK_NFIELDS), \
            int(used.value)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_dsampler_destroy(h)
            self._h = None
