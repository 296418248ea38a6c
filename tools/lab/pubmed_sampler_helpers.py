"""Host sampler (gs_sample_pack_run_multi_team) on a Pubmed-sized forward batch: 9,700 random roots,
fanouts 10,10, by helper count (argv[1]); ms per batch, median of 25."""
import sys, importlib, time, ctypes, random
sys.path.insert(0, ".")
import numpy as np
gs = importlib.import_module("graphsage-pytorch_amd")
_lib = importlib.import_module("graphsage-pytorch_amd._lib")
S = importlib.import_module("graphsage-pytorch_amd.sampler")
g = np.load("tests/golden/graphs.npz")
src, dst, n = g["pubmed_src"].astype(np.int64), g["pubmed_dst"].astype(np.int64), int(g["pubmed_n"][0])
graph = gs.CSRGraph.from_pairs(src, dst, n)
lib = _lib.lib()
H = int(sys.argv[1]) if len(sys.argv) > 1 else 7
t = ctypes.c_void_p(); _lib.check(lib.gs_team_create(H, ctypes.byref(t)))
fan = np.array([10, 10], np.int32)
rs = np.random.RandomState(0)
rng = S.RNG(824)
T = []
for it in range(30):
    roots = np.ascontiguousarray(rs.permutation(n)[:9700], np.int64)
    bound = int(lib.gs_sample_pack_bound(graph.handle, len(roots), fan.ctypes.data, 2))
    buf = np.empty(bound, np.int32)
    sizes = np.empty(8, np.int64); offs = np.empty(_lib.GS_MAX_HOPS * _lib.GS_PK_NFIELDS, np.int64); used = ctypes.c_int64()
    t0 = time.perf_counter()
    _lib.check(lib.gs_sample_pack_run_multi_team(graph.handle, rng._h, roots.ctypes.data, len(roots), len(roots), fan.ctypes.data, 2, 0, buf.ctypes.data, bound, sizes.ctypes.data, offs.ctypes.data, ctypes.byref(used), t))
    T.append(time.perf_counter() - t0)
print("helpers", H, "ms median", np.median(T[5:]) * 1e3, "sizes", sizes[:8])
