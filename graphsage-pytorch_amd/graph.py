"""Adjacency for the sampler: CSR rows in CPython-set iteration order.

The reference keeps the graph as ``defaultdict(set)`` filled by
``adj[p1].add(p2); adj[p2].add(p1)`` in file order (dataCenter.py:33-41,
:77-86).  Because ``random.sample(adj_set, k)`` samples ``tuple(adj_set)``
(models.py:282), each set's *iteration order* is part of the sampling
semantics, and for rows with fewer than k neighbours the set's *table layout*
decides the frontier order of the union (models.py:285-286).  ``CSRGraph``
keeps both, built natively (libgraphsage_amd ``gs_graph_build``), and mirrors
the CSR to the GPU for the device-side expansion of the last hop.
"""
import ctypes
import mmap
import os
import sys

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


class CSRGraph:
    """Native adjacency handle (host) + lazily mirrored device CSR."""

    def __init__(self, handle, n_nodes):
        self._h = ctypes.c_void_p(handle)
        self.n_nodes = int(n_nodes)
        n, e, md = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().gs_graph_dims(self._h, ctypes.byref(n), ctypes.byref(e), ctypes.byref(md)))
        self.n_entries = int(e.value)
        self.max_degree = int(md.value)
        self._dev = {}

    # ------------------------------------------------------------ builders
    @classmethod
    def from_pairs(cls, src, dst, n_nodes=None, n_threads=None):
        """adj[a].add(b); adj[b].add(a) for every pair, in order."""
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        if src.shape != dst.shape or src.ndim != 1:
            raise ValueError("src/dst must be 1-D arrays of equal length")
        if n_nodes is None:
            n_nodes = int(max(src.max(initial=-1), dst.max(initial=-1)) + 1)
        h = ctypes.c_void_p()
        check(lib().gs_graph_build(ptr(src), ptr(dst), len(src), int(n_nodes),
                                   int(n_threads or _threads()), ctypes.byref(h)))
        return cls(h.value, n_nodes)

    @classmethod
    def from_adj_lists(cls, adj_lists, n_nodes=None):
        """Adopt a caller-built dict of int sets (the drop-in path).

        Each set's table is read from the live CPython object (PySetObject:
        fill, used, mask, table of {key, hash}), and checked against the set's
        own iteration order, so the sampler replays exactly the layout the
        reference would see.  CPython 3.10 only — the reference itself relies on
        random.sample(set) which 3.11 removed (models.py:282).
        """
        if sys.implementation.name != "cpython" or sys.version_info[:2] != (3, 10):
            raise RuntimeError("from_adj_lists reads CPython 3.10 set tables; use from_pairs")
        if n_nodes is None:
            n_nodes = (max(adj_lists.keys()) + 1) if len(adj_lists) else 0
        n_nodes = int(n_nodes)
        row_ptr = np.zeros(n_nodes + 1, np.int64)
        cols, slots = [], []
        log2 = np.full(n_nodes, 3, np.uint8)
        dirty = np.zeros(n_nodes, np.uint8)
        get = adj_lists.get if hasattr(adj_lists, "get") else (lambda k, d=None: adj_lists[k])
        for v in range(n_nodes):
            s = get(v, None)
            if s is None or len(s) == 0:
                row_ptr[v + 1] = row_ptr[v]
                if s is not None:
                    fill, used, mask, _ = _set_header(s)
                    log2[v] = int(mask + 1).bit_length() - 1
                    dirty[v] = fill != used
                continue
            fill, used, mask, table = _set_header(s)
            raw = np.frombuffer(ctypes.string_at(table, 16 * (mask + 1)), dtype=np.int64).reshape(-1, 2)
            live = (raw[:, 0] != 0) & (raw[:, 1] != -1)
            sl = np.nonzero(live)[0]
            keys = raw[sl, 1]
            if len(keys) != used or list(keys) != list(s):
                raise ValueError(f"adj_lists[{v}]: set table does not match its iteration order "
                                 "(non-int or negative keys?)")
            cols.append(keys.astype(np.int32))
            slots.append(sl.astype(np.uint32))
            row_ptr[v + 1] = row_ptr[v] + len(keys)
            log2[v] = int(mask + 1).bit_length() - 1
            dirty[v] = fill != used
        col = np.concatenate(cols) if cols else np.zeros(0, np.int32)
        slot = np.concatenate(slots) if slots else np.zeros(0, np.uint32)
        h = ctypes.c_void_p()
        check(lib().gs_graph_from_tables(n_nodes, ptr(row_ptr), ptr(col), ptr(slot), ptr(log2),
                                         ptr(dirty), ctypes.byref(h)))
        return cls(h.value, n_nodes)

    # ------------------------------------------------- node-wide sharing
    def write_image(self, path):
        """Write this graph's flat image to `path` (atomically: a temporary
        file renamed into place), for other processes to map (``from_image``)."""
        nb = int(lib().gs_graph_image_bytes(self._h))
        if nb <= 0:
            raise RuntimeError("gs_graph_image_bytes failed")
        tmp = f"{path}.tmp{os.getpid()}"
        with open(tmp, "wb+") as f:
            f.truncate(nb)
            mm = mmap.mmap(f.fileno(), nb)
            try:
                buf = (ctypes.c_char * nb).from_buffer(mm)
                check(lib().gs_graph_write_image(self._h, ctypes.addressof(buf), nb))
                del buf
                mm.flush()
            finally:
                mm.close()
        os.replace(tmp, path)
        return nb

    @classmethod
    def from_image(cls, path):
        """Adopt the image at `path` mapped read-only (no copy): the graph's
        arrays are the mapping's pages, shared by every process that maps it."""
        with open(path, "rb") as f:
            nb = os.fstat(f.fileno()).st_size
            mm = mmap.mmap(f.fileno(), nb, prot=mmap.PROT_READ)
        view = np.frombuffer(mm, dtype=np.uint8)  # read-only; its address is the mapping's
        h = ctypes.c_void_p()
        check(lib().gs_graph_from_image(view.ctypes.data, nb, ctypes.byref(h)))
        n = ctypes.c_int64()
        check(lib().gs_graph_dims(h, ctypes.byref(n), None, None))
        g = cls(h.value, n.value)
        g._mapping = (mm, view)  # keep the pages mapped for the handle's lifetime
        return g

    @classmethod
    def shared(cls, build, path, local_rank, barrier):
        """One graph per node: local rank 0 runs ``build()`` and writes its
        image to ``path``; after ``barrier()`` every other rank maps it.  Rank
        0 keeps its built graph (identical bytes)."""
        g = None
        if local_rank == 0:
            g = build()
            g.write_image(path)
        barrier()
        if g is None:
            g = cls.from_image(path)
        return g

    # --------------------------------------------------------------- views
    def row_ptr(self):
        p = lib().gs_graph_row_ptr(self._h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int64)),
                                     shape=(self.n_nodes + 1,)).copy()

    def col(self):
        if self.n_entries == 0:
            return np.zeros(0, np.int32)
        p = lib().gs_graph_col(self._h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int32)),
                                     shape=(self.n_entries,)).copy()

    def degrees(self):
        return np.diff(self.row_ptr())

    def row(self, v):
        rp = self.row_ptr()
        return self.col()[rp[v]:rp[v + 1]]

    def device_csr(self, device):
        """(row_ptr int64, col int32) on `device`, uploaded once."""
        key = str(torch.device(device))
        if key not in self._dev:
            rp = torch.from_numpy(self.row_ptr()).to(device)
            cl = torch.from_numpy(self.col()).to(device)
            if cl.numel() == 0:
                cl = torch.zeros(1, dtype=torch.int32, device=device)
            self._dev[key] = (rp, cl)
        return self._dev[key]

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and getattr(_lib, "_lib", None) is not None:  # _lib is None at interpreter exit
            _lib._lib.gs_graph_destroy(h)
            self._h = None


def _set_header(s):
    """(fill, used, mask, table*) of a CPython 3.10 PySetObject."""
    base = id(s)
    rd = ctypes.c_ssize_t.from_address
    fill, used, mask = rd(base + 16).value, rd(base + 24).value, rd(base + 32).value
    table = ctypes.c_void_p.from_address(base + 40).value
    if used != len(s) or mask < 7 or (mask + 1) & mask:
        raise RuntimeError("unexpected PySetObject layout (not CPython 3.10?)")
    return fill, used, mask, table


def rmat_pairs(scale, n_pairs, a=0.57, b=0.19, c=0.19, seed=824, permute=True, n_threads=None):
    """R-MAT(a, b, c, 1-a-b-c) pairs, self pairs dropped."""
    src = np.empty(int(n_pairs), np.int64)
    dst = np.empty(int(n_pairs), np.int64)
    kept = ctypes.c_int64()
    check(lib().gs_rmat_pairs(int(scale), int(n_pairs), float(a), float(b), float(c),
                              int(seed) & 0xFFFFFFFFFFFFFFFF, int(bool(permute)),
                              int(n_threads or _threads()), ptr(src), ptr(dst), ctypes.byref(kept)))
    return src[:kept.value], dst[:kept.value]
