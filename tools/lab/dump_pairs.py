"""Write a graph of tests/golden/graphs.npz (argv[1]: pubmed / cora) as the
sampler bench's pair file (int64 n, int64 count, src ids, dst ids) to argv[2]."""
import sys
import numpy as np
g = np.load("tests/golden/graphs.npz")
name = sys.argv[1]
src, dst = g[f"{name}_src"].astype(np.int64), g[f"{name}_dst"].astype(np.int64)
with open(sys.argv[2], "wb") as f:
    np.array([int(g[f"{name}_n"][0]), len(src)], np.int64).tofile(f)
    src.tofile(f)
    dst.tofile(f)
