"""Deterministic synthetic inputs shared by the golden capture script, the
tests and the benchmark (the reference ships no feature files:
/root/reference/.MISSING_LARGE_BLOBS).  Pure numpy, no RNG state consumed."""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform_features(seed, n_rows, n_cols, row0=0):
    """U(-1,1) table: the same counter hash as the device kernel gs_fill_uniform
    (kernels/misc.hip uniform_hash)."""
    with np.errstate(over="ignore"):
        r = np.arange(row0, row0 + n_rows, dtype=np.uint64)[:, None]
        c = np.arange(n_cols, dtype=np.uint64)[None, :]
        z = (np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + r * np.uint64(0xBF58476D1CE4E5B9)
             + c * np.uint64(0x94D049BB133111EB))
        z = _mix(z)
    m = (z >> np.uint64(40)).astype(np.int64) - (1 << 23)
    return (m.astype(np.float32) * np.float32(1.0 / 8388608.0)).astype(np.float32)


def hashed_binary_features(n_rows, n_cols):
    """Cora-like sparse binary bag-of-words (≈1.27 % density)."""
    i = np.arange(n_rows, dtype=np.int64)[:, None]
    j = np.arange(n_cols, dtype=np.int64)[None, :]
    return (((i * 1315423911 + j * 2654435761) % 1000003) % 79 == 0).astype(np.float32)


def tiny_rmat_pairs(scale=9, n_pairs=6000, seed=17):
    """Small skewed graph for sampling/forward fixtures (numpy only)."""
    rs = np.random.RandomState(seed)
    a, b, c = 0.57, 0.19, 0.19
    u = np.zeros(n_pairs, np.int64)
    v = np.zeros(n_pairs, np.int64)
    for _ in range(scale):
        r = rs.random_sample(n_pairs)
        bu = (r >= a + b).astype(np.int64)
        bv = (((r >= a) & (r < a + b)) | (r >= a + b + c)).astype(np.int64)
        u = (u << 1) | bu
        v = (v << 1) | bv
    keep = u != v
    u, v = u[keep], v[keep]
    # compact ids to the touched nodes (first appearance), so every node has an edge
    ids = {}
    src = np.empty(len(u), np.int64)
    dst = np.empty(len(v), np.int64)
    for t, (x, y) in enumerate(zip(u.tolist(), v.tolist())):
        for z in (x, y):
            if z not in ids:
                ids[z] = len(ids)
        src[t], dst[t] = ids[x], ids[y]
    return src, dst, len(ids)


def labels_mod(n, n_classes):
    return (np.arange(n, dtype=np.int64) % n_classes).astype(np.int64)
