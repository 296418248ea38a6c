"""Native host side (no GPU needed): C-ABI exports, RNG / set known answers,
CSR builder order, multi-hop sampler bit-exactness vs the reference's vectors
and vs the oracle, error behaviour, and the device pack layout."""
import ctypes
import json
import os
import random
import re

import numpy as np
import pytest

from oracle import Adjacency, sample_layers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def test_library_exports_every_declared_symbol(gs):
    hdr = open(os.path.join(ROOT, "include", "graphsage_amd.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|void|const char\*|const int64_t\*|const int32_t\*)\s+\**(gs_\w+)\(",
                              hdr, re.M))
    assert len(declared) > 30
    L = gs._lib.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert set(gs._lib.exported_symbols()) >= declared
    assert b"gfx950" in L.gs_version()


def test_rng_known_answers(gs):
    for rec in json.load(open(os.path.join(G, "rng.json"))):
        r = gs.RNG(rec["seed"])
        assert r.getrandbits(32, 8).tolist() == rec["bits32"]
        for k, v in rec["bits_k"]:
            assert int(r.getrandbits(k)[0]) == v
        for s in rec["samples"]:
            assert r.sample_positions(s["n"], s["k"]).tolist() == s["out"], (rec["seed"], s["n"], s["k"])
        for n, v in rec["choice"]:
            assert r.choice_position(n) == v
        for n, v in rec["randbelow"]:
            assert int(r.randbelow(n)[0]) == v
        mt, pos = r.getstate()
        assert mt.tolist() + [pos] == rec["state_after"]


def test_rng_python_state_roundtrip(gs):
    random.seed(99)
    random.random()
    r = gs.RNG.from_python()
    a = r.getrandbits(32, 5).tolist()
    b = [random.getrandbits(32) for _ in range(5)]
    assert a == b
    r.to_python()
    assert random.getrandbits(32) == int(r.getrandbits(32)[0])


def test_sample_errors(gs):
    r = gs.RNG(1)
    with pytest.raises(ValueError, match="Sample larger"):
        r.sample_positions(3, 4)
    with pytest.raises(ValueError):
        r.choice_position(0)


def test_pyset_known_answers(gs):
    for case in json.load(open(os.path.join(G, "pyset.json"))):
        assert gs.pyset_union_of_lists(case["lists"]).tolist() == case["union"]


def _graph(gs, name):
    g = np.load(os.path.join(G, "graphs.npz"))
    return gs.CSRGraph.from_pairs(g[f"{name}_src"], g[f"{name}_dst"], int(g[f"{name}_n"][0])), g


@pytest.mark.parametrize("name", ["cora", "pubmed", "rmat"])
def test_csr_rows_in_reference_set_order(gs, name):
    G_, g = _graph(gs, name)
    assert np.array_equal(G_.row_ptr(), g[f"{name}_row_ptr"])
    assert np.array_equal(G_.col(), g[f"{name}_col"])


@pytest.mark.parametrize("name", ["cora", "pubmed", "rmat"])
@pytest.mark.parametrize("full", [False, True])
def test_sampler_matches_reference_vectors(gs, name, full):
    G_, _ = _graph(gs, name)
    S = np.load(os.path.join(G, f"sample_{name}.npz"))
    for key in sorted({k.split("__")[0] for k in S.files}):
        seed = int(key.split("_")[0][1:])
        fan = [int(x) for x in key.split("_f")[1].split("-")]
        r = gs.RNG(seed)
        s = gs.sample(G_, r, S[key + "__roots"], fan, full=full)
        for j in range(1, len(fan) + 1):
            h = s.hop(j)
            if j < len(fan) or full:
                assert np.array_equal(h.src_ids, S[f"{key}__h{j}_union"]), (key, j)
                assert np.array_equal(h.set_ptr, S[f"{key}__h{j}_set_ptr"])
                assert np.array_equal(h.set_items, S[f"{key}__h{j}_set_items"])
        mt, pos = r.getstate()
        assert np.array_equal(np.append(mt.astype(np.int64), pos), S[key + "__state"])


def test_adj_lists_adoption_matches_pairs(gs):
    from collections import defaultdict
    g = np.load(os.path.join(G, "graphs.npz"))
    adj = defaultdict(set)
    for a, b in zip(g["pubmed_src"].tolist(), g["pubmed_dst"].tolist()):
        adj[a].add(b)
        adj[b].add(a)
    G1 = gs.CSRGraph.from_adj_lists(adj, int(g["pubmed_n"][0]))
    G2, _ = _graph(gs, "pubmed")
    assert np.array_equal(G1.col(), G2.col()) and np.array_equal(G1.row_ptr(), G2.row_ptr())
    # a set with dummies (after discard) still reproduces the reference's frontier
    adj[7].discard(next(iter(adj[7])))
    G3 = gs.CSRGraph.from_adj_lists(adj, int(g["pubmed_n"][0]))
    roots = [7] + list(range(100, 140))
    random.seed(3)
    want = sample_layers(adj, roots, [10, 10])
    s = gs.sample(G3, gs.RNG(3), roots, [10, 10], full=True)
    assert s.hop(1).src_ids.tolist() == want[0][3]
    assert s.hop(2).src_ids.tolist() == want[1][3]


def test_sampler_vs_oracle_random_graphs(gs):
    """Random skewed graphs, many seeds, fanouts incl. None (take all) and >setsize."""
    rs = np.random.RandomState(0)
    for trial in range(6):
        n = int(rs.randint(50, 400))
        m = int(rs.randint(n, 12 * n))
        hub = rs.randint(0, n, size=m) * (rs.random_sample(m) < 0.3)
        src = np.where(hub > 0, hub % 7, rs.randint(0, n, size=m))
        dst = rs.randint(0, n, size=m)
        keep = src != dst
        src, dst = src[keep], dst[keep]
        Gn = gs.CSRGraph.from_pairs(src, dst, n)
        adj = Adjacency(src, dst, n)
        deg = Gn.degrees()
        roots = [int(v) for v in rs.permutation(np.nonzero(deg)[0])[:int(rs.randint(1, 60))]]
        for fan in ([25, 10], [10, 10], [3, None], [100], [2, 2, 2]):
            seed = int(rs.randint(0, 10 ** 6))
            random.seed(seed)
            want = sample_layers(adj, roots, fan)
            s = gs.sample(Gn, gs.RNG(seed), roots, fan, full=True)
            for j, (_, samp, _, union) in enumerate(want, start=1):
                h = s.hop(j)
                assert h.src_ids.tolist() == union
                assert h.sets() == [list(x) for x in samp]
            r2 = gs.RNG(seed)
            gs.sample(Gn, r2, roots, fan)
            assert r2.getstate()[0].tolist() + [r2.getstate()[1]] == list(random.getstate()[1])


def test_sampler_duplicate_roots_vs_oracle(gs):
    """nodes_batch with repeated ids: the reference samples every occurrence
    (drawing from `random` each time, models.py:282) and unions the results;
    the same per occurrence here, and the same words consumed."""
    rs = np.random.RandomState(5)
    n = 300
    src = rs.randint(0, n, 3000)
    dst = (src + 1 + rs.randint(0, n - 1, 3000)) % n
    Gn = gs.CSRGraph.from_pairs(src, dst, n)
    adj = Adjacency(src, dst, n)
    base = [int(v) for v in rs.permutation(np.nonzero(Gn.degrees())[0])[:20]]
    roots = base + base[:7] + [base[3]] * 3
    for fan in ([25, 10], [4, 3], [None, 5]):
        random.seed(9)
        want = sample_layers(adj, roots, fan)
        s = gs.sample(Gn, gs.RNG(9), roots, fan, full=True)
        for j, (_, samp, _, union) in enumerate(want, start=1):
            h = s.hop(j)
            assert h.dst_ids.tolist() == (roots if j == 1 else want[j - 2][3])
            assert h.src_ids.tolist() == union
            assert h.sets() == [list(x) for x in samp]
        r2 = gs.RNG(9)
        gs.sample(Gn, r2, roots, fan)
        assert r2.getstate()[0].tolist() + [r2.getstate()[1]] == list(random.getstate()[1])


def test_sample_pack_layout(gs):
    G_, _ = _graph(gs, "cora")
    s = gs.sample(G_, gs.RNG(824), list(range(0, 200, 7)), [10, 10])
    buf = s.pack()
    assert buf.numel() >= s.pack_total
    for j in range(1, 3):
        for f in s.offsets[j - 1]:
            assert f == -1 or f % 4 == 0  # 16-byte aligned arrays
    h1, h2 = s.hop(1), s.hop(2)
    off = s.offsets
    b = buf.numpy()
    assert np.array_equal(b[off[0][gs._lib.GS_PK_NBR_PTR]:][:h1.n_dst + 1], h1.nbr_ptr)
    assert np.array_equal(b[off[0][gs._lib.GS_PK_NBR]:][:h1.n_nbr], h1.nbr)
    rs = G_.row_ptr()[h2.dst_ids]  # the pack holds absolute entries row_ptr[dst] + pos
    assert np.array_equal(b[off[1][gs._lib.GS_PK_POS]:][:h2.n_pos], np.repeat(rs, np.diff(h2.pos_ptr)) + h2.pos)
    assert np.array_equal(b[off[1][gs._lib.GS_PK_DST_IDS]:][:h2.n_dst], h1.src_ids)
    tp = b[off[0][gs._lib.GS_PK_TPTR]:][:h1.n_src + 1]
    ti = b[off[0][gs._lib.GS_PK_TIDX]:][:h1.n_nbr + h1.n_dst]
    # every (dst, src) edge and every self row appears exactly once in the transpose
    pairs = sorted((c, int(t)) for c in range(h1.n_src) for t in ti[tp[c]:tp[c + 1]])
    want = sorted([(int(h1.self_local[r]), -(r + 1)) for r in range(h1.n_dst)] +
                  [(int(c), r) for r in range(h1.n_dst) for c in h1.nbr[h1.nbr_ptr[r]:h1.nbr_ptr[r + 1]]])
    assert pairs == want


def test_unknown_node_raises(gs):
    G_, _ = _graph(gs, "cora")
    with pytest.raises(IndexError):
        gs.sample(G_, gs.RNG(1), [5, 10 ** 6], [10, 10])


def test_rmat_generator_deterministic(gs):
    a = gs.rmat_pairs(12, 50000, seed=5, n_threads=1)
    b = gs.rmat_pairs(12, 50000, seed=5, n_threads=7)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert (a[0] != a[1]).all() and a[0].max() < 4096
    deg = np.bincount(np.concatenate(a), minlength=4096)
    assert deg.max() > 20 * max(1, np.median(deg))  # power-law skew


def test_pack_run_matches_sample_pack(gs):
    """The streaming sample+pack call equals sample() + pack() and leaves the rng identical."""
    import torch
    G_, _ = _graph(gs, "rmat")
    L = gs._lib
    roots = np.nonzero(G_.degrees())[0][:40].astype(np.int64)
    fan = np.array([25, 10], np.int32)
    bound = int(L.lib().gs_sample_pack_bound(G_.handle, len(roots), fan.ctypes.data, 2))
    buf = np.full(bound, -7, np.int32)
    sizes = np.empty(8, np.int64)
    offs = np.empty(L.GS_MAX_HOPS * L.GS_PK_NFIELDS, np.int64)
    used = ctypes.c_int64()
    r1 = gs.RNG(42)
    L.check(L.lib().gs_sample_pack_run(G_.handle, r1._h, roots.ctypes.data, len(roots), fan.ctypes.data, 2, 0,
                                       buf.ctypes.data, bound, sizes.ctypes.data, offs.ctypes.data,
                                       ctypes.byref(used)))
    r2 = gs.RNG(42)
    s = gs.sample(G_, r2, roots, [25, 10])
    assert s.pack_total + len(roots) == used.value
    assert [tuple(sizes[4 * j:4 * j + 4]) for j in range(2)] == [s.sizes(1), s.sizes(2)]
    ref = s.pack().numpy()
    for j in range(2):
        for f in range(L.GS_PK_NFIELDS):
            o = offs[j * L.GS_PK_NFIELDS + f]
            assert o == s.offsets[j][f]
    h1, h2 = s.hop(1), s.hop(2)
    for j, f, n in [(0, L.GS_PK_NBR, h1.n_nbr), (0, L.GS_PK_TIDX, h1.n_nbr + h1.n_dst), (1, L.GS_PK_POS, h2.n_pos)]:
        o = s.offsets[j][f]
        assert np.array_equal(buf[o:o + n], ref[o:o + n])
    assert np.array_equal(buf[s.pack_total:used.value], roots.astype(np.int32))
    assert r1.getstate()[0].tolist() == r2.getstate()[0].tolist() and r1.getstate()[1] == r2.getstate()[1]
    with pytest.raises(ValueError):  # below the bound: refused before any rng word is drawn
        L.check(L.lib().gs_sample_pack_run(G_.handle, r1._h, roots.ctypes.data, len(roots), fan.ctypes.data, 2,
                                           0, buf.ctypes.data, 10, sizes.ctypes.data, offs.ctypes.data,
                                           ctypes.byref(used)))


def _pack_run(gs, G_, rng, roots, fan, group=None):
    L = gs._lib
    nh = len(fan)
    if group is None:
        bound = int(L.lib().gs_sample_pack_bound(G_.handle, len(roots), fan.ctypes.data, nh))
    else:
        bound = int(L.lib().gs_sample_pack_bound_multi(G_.handle, len(roots), group, fan.ctypes.data, nh))
    buf = np.full(bound, -7, np.int32)
    sizes = np.empty(4 * nh, np.int64)
    offs = np.empty(L.GS_MAX_HOPS * L.GS_PK_NFIELDS, np.int64)
    used = ctypes.c_int64()
    if group is None:
        L.check(L.lib().gs_sample_pack_run(G_.handle, rng._h, roots.ctypes.data, len(roots), fan.ctypes.data, nh,
                                           0, buf.ctypes.data, bound, sizes.ctypes.data, offs.ctypes.data,
                                           ctypes.byref(used)))
    else:
        L.check(L.lib().gs_sample_pack_run_multi(G_.handle, rng._h, roots.ctypes.data, len(roots), group,
                                                 fan.ctypes.data, nh, 0, buf.ctypes.data, bound, sizes.ctypes.data,
                                                 offs.ctypes.data, ctypes.byref(used)))
    offs = offs.reshape(L.GS_MAX_HOPS, L.GS_PK_NFIELDS)
    return buf[:used.value], sizes.reshape(nh, 4), offs, used.value


@pytest.mark.parametrize("n_roots,group", [(40, 15), (45, 15), (12, 15), (3, 1)])
def test_pack_run_multi_rebases_groups(gs, n_roots, group):
    """Several batches in one pack (the merged inference steps): the same
    draws as one gs_sample_pack_run per group on one stream, and every field
    the concatenation of the groups' fields with pointers and frontier
    indices rebased (TIDX keeps its self encoding -(r+1))."""
    G_, _ = _graph(gs, "rmat")
    L = gs._lib
    roots = np.nonzero(G_.degrees())[0][5:5 + n_roots].astype(np.int64)
    fan = np.array([25, 10], np.int32)
    r1, r2 = gs.RNG(9), gs.RNG(9)
    parts = [_pack_run(gs, G_, r1, roots[lo:lo + group], fan) for lo in range(0, n_roots, group)]
    buf, sizes, offs, used = _pack_run(gs, G_, r2, roots, fan, group)
    assert r1.getstate()[0].tolist() == r2.getstate()[0].tolist() and r1.getstate()[1] == r2.getstate()[1]
    if len(parts) == 1:
        assert np.array_equal(buf, parts[0][0])
        return
    assert np.array_equal(sizes[:, :2], sum(p[1][:, :2] for p in parts))
    assert np.array_equal(sizes[0, 2:], sum(p[1][0, 2:] for p in parts)) and (sizes[1, 2:] == -1).all()

    def field(p, j, f, n):
        o = p[2][j, f]
        return p[0][o:o + n]

    def cat_ptr(j, f, nd_col, n_col):
        out, base = [], 0
        for p in parts:
            v = field(p, j, f, p[1][j, nd_col] + 1)
            out.append(v[:-1] + base)
            base += p[1][j, n_col]
        return np.concatenate(out + [np.array([base])])

    def cat_idx(j, f, n_col, base_col, neg=False):
        out, base = [], 0
        for p in parts:
            v = field(p, j, f, p[1][j, n_col]).astype(np.int64)
            out.append(np.where(v >= 0, v + base, v - base) if neg else v + base)
            base += p[1][j, base_col]
        return np.concatenate(out)

    got = lambda j, f, n: field((buf, sizes, offs), j, f, n)
    # hop 1 (roots -> F1): explicit lists into the src frontier, transposed lists over it
    nd, nn, ns = sizes[0, 0], sizes[0, 3], sizes[0, 2]
    assert np.array_equal(got(0, L.GS_PK_NBR_PTR, nd + 1), cat_ptr(0, L.GS_PK_NBR_PTR, 0, 3))
    assert np.array_equal(got(0, L.GS_PK_NBR, nn), cat_idx(0, L.GS_PK_NBR, 3, 2))
    assert np.array_equal(got(0, L.GS_PK_SELF, nd), cat_idx(0, L.GS_PK_SELF, 0, 2))
    tptr, base = [], 0
    for p in parts:
        v = field(p, 0, L.GS_PK_TPTR, p[1][0, 2] + 1)
        tptr.append(v[:-1] + base)
        base += v[-1]
    assert np.array_equal(got(0, L.GS_PK_TPTR, ns + 1), np.concatenate(tptr + [np.array([base])]))
    tidx, base_d = [], 0
    for p in parts:
        v = field(p, 0, L.GS_PK_TIDX, p[1][0, 3] + p[1][0, 0]).astype(np.int64)
        tidx.append(np.where(v >= 0, v + base_d, v - base_d))
        base_d += p[1][0, 0]
    assert np.array_equal(got(0, L.GS_PK_TIDX, nn + nd), np.concatenate(tidx))
    # hop 2 (F1 -> F0, the layer-1 gather): absolute CSR entries and global ids need no rebasing
    nd2, npos = sizes[1, 0], sizes[1, 1]
    assert nd2 == ns
    assert np.array_equal(got(1, L.GS_PK_POS_PTR, nd2 + 1), cat_ptr(1, L.GS_PK_POS_PTR, 0, 1))
    assert np.array_equal(got(1, L.GS_PK_POS, npos), np.concatenate([field(p, 1, L.GS_PK_POS, p[1][1, 1]) for p in parts]))
    assert np.array_equal(got(1, L.GS_PK_DST_IDS, nd2),
                          np.concatenate([field(p, 1, L.GS_PK_DST_IDS, p[1][1, 0]) for p in parts]))
    assert np.array_equal(buf[used - n_roots:], roots.astype(np.int32))


def test_stream_seeds_are_reference_seeds(gs):
    """Stream (rank, w) draws exactly what random.seed(seed + rank + 64 w) would."""
    import importlib
    train = importlib.import_module("graphsage-pytorch_amd.train")
    assert train.rank_seed(824, 0, 0) == 824
    G_, g = _graph(gs, "cora")
    adj = Adjacency(g["cora_src"], g["cora_dst"], int(g["cora_n"][0]))
    batches = list(train.rank_batches(np.arange(2708), 20, 1, 2, 5))[:6]
    S = 2
    for w in range(S):
        seed = train.rank_seed(824, 1, w)
        r = train.make_rng(824, 1, w)
        random.seed(seed)
        for roots in batches[w::S]:
            s = gs.sample(G_, r, roots, [10, 10], full=True)
            want = sample_layers(adj, roots.tolist(), [10, 10])
            assert s.hop(2).src_ids.tolist() == want[1][3]
        assert r.getstate()[0].tolist() + [r.getstate()[1]] == list(random.getstate()[1])


def test_sample_positions_match_cpython_random_sample(gs):
    """random.sample over both branches (pool / selected-set, incl. the
    chunked k <= 32 scan) and across MT block refills: positions and the
    stream state must equal CPython's own random.Random."""
    rs = np.random.RandomState(7)
    ks = [1, 2, 5, 6, 10, 16, 25, 31, 32, 33, 40]
    for seed in (0, 1, 824):
        py = random.Random(seed)
        r = gs.RNG(seed)
        for _ in range(2500):
            k = int(rs.choice(ks))
            n = int(rs.choice([k, k + 1, 50, 85, 86, 100, 128, 129, 277, 278, 1000, 65536, 100003, (1 << 20) + 3]))
            if n < k:
                continue
            assert r.sample_positions(n, k).tolist() == py.sample(range(n), k), (seed, n, k)
        mt, pos = r.getstate()
        st = py.getstate()[1]
        assert mt.tolist() == list(st[:624]) and pos == st[624]


@pytest.mark.parametrize("helpers", [1, 3])
@pytest.mark.parametrize("fan,group", [((25, 10), None), ((10, 10, 5), None), ((25, 10), 150)])
def test_team_pack_equals_single_thread(gs, helpers, fan, group):
    """Helper threads (gs_team) split a batch's set builds and run each hop's
    neighbour / transposed lists under the next hop's draws: the pack image,
    sizes and rng state must equal the team-less call's bit for bit, batch
    after batch on one stream (3 hops: two materialised hops, so a lists job
    overlaps the next hop's set builds too)."""
    L = gs._lib
    G_, _ = _graph(gs, "rmat")
    fan = np.array(fan, np.int32)
    nh = len(fan)
    team = ctypes.c_void_p()
    L.check(L.lib().gs_team_create(helpers, ctypes.byref(team)))
    try:
        cand = np.nonzero(G_.degrees())[0]
        rs = np.random.RandomState(5)
        r1, r2 = gs.RNG(77), gs.RNG(77)
        for _ in range(6):
            roots = rs.choice(cand, 300).astype(np.int64)
            want = _pack_run(gs, G_, r1, roots, fan, group)
            g = group if group is not None else len(roots)
            bound = int(L.lib().gs_sample_pack_bound_multi(G_.handle, len(roots), g, fan.ctypes.data, nh))
            buf = np.full(bound, -7, np.int32)
            sizes = np.empty(4 * nh, np.int64)
            offs = np.empty(L.GS_MAX_HOPS * L.GS_PK_NFIELDS, np.int64)
            used = ctypes.c_int64()
            L.check(L.lib().gs_sample_pack_run_multi_team(G_.handle, r2._h, roots.ctypes.data, len(roots), g,
                                                          fan.ctypes.data, nh, 0, buf.ctypes.data, bound,
                                                          sizes.ctypes.data, offs.ctypes.data, ctypes.byref(used),
                                                          team))
            assert used.value == want[3]
            assert np.array_equal(buf[:used.value], want[0])
            assert np.array_equal(sizes.reshape(nh, 4), want[1])
            assert r1.getstate()[0].tolist() == r2.getstate()[0].tolist() and r1.getstate()[1] == r2.getstate()[1]
    finally:
        L.lib().gs_team_destroy(team)


@pytest.mark.parametrize("gcn", [False, True])
def test_team_lists_job_many_workers(gs, gcn):
    """A hop's lists job split over seven helpers (slot ranks, then chunks of
    32 destinations, then the transpose beside the pack copy): 2,000-root
    batches (63 chunks) with and without gcn give the team-less pack bit for
    bit, batch after batch."""
    L = gs._lib
    G_, _ = _graph(gs, "rmat")
    fan = np.array((10, 10), np.int32)
    nh = len(fan)
    flags = L.GS_SAMPLE_GCN if gcn else 0
    cand = np.nonzero(G_.degrees())[0]
    rs = np.random.RandomState(11)
    team = ctypes.c_void_p()
    L.check(L.lib().gs_team_create(7, ctypes.byref(team)))
    r1, r2 = gs.RNG(5), gs.RNG(5)

    def run(rng, roots, t):
        bound = int(L.lib().gs_sample_pack_bound(G_.handle, len(roots), fan.ctypes.data, nh))
        buf = np.full(bound, -7, np.int32)
        sizes = np.empty(4 * nh, np.int64)
        offs = np.empty(L.GS_MAX_HOPS * L.GS_PK_NFIELDS, np.int64)
        used = ctypes.c_int64()
        if t is None:
            L.check(L.lib().gs_sample_pack_run(G_.handle, rng._h, roots.ctypes.data, len(roots), fan.ctypes.data,
                                               nh, flags, buf.ctypes.data, bound, sizes.ctypes.data,
                                               offs.ctypes.data, ctypes.byref(used)))
        else:
            L.check(L.lib().gs_sample_pack_run_multi_team(G_.handle, rng._h, roots.ctypes.data, len(roots),
                                                          len(roots), fan.ctypes.data, nh, flags, buf.ctypes.data,
                                                          bound, sizes.ctypes.data, offs.ctypes.data,
                                                          ctypes.byref(used), t))
        return buf[:used.value].copy(), sizes.copy()

    try:
        for _ in range(3):
            roots = rs.choice(cand, 2000).astype(np.int64)
            want, got = run(r1, roots, None), run(r2, roots, team)
            assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
            assert r1.getstate()[0].tolist() == r2.getstate()[0].tolist() and r1.getstate()[1] == r2.getstate()[1]
    finally:
        L.lib().gs_team_destroy(team)


def test_shared_team_streams_equal_single_thread(gs):
    """Three sampling streams on three threads whose teams share one pool of
    helpers (gs_team_create_shared, the runner's GS_SHARED_HELPERS layout):
    a helper builds whichever stream's sets are posted, and every stream's
    packs must still equal its team-less run's bit for bit."""
    import threading
    L = gs._lib
    G_, _ = _graph(gs, "rmat")
    fan = np.array((25, 10), np.int32)
    nh = len(fan)
    cand = np.nonzero(G_.degrees())[0]
    n_streams, n_batches = 3, 5
    roots = [[np.random.RandomState(10 * w + b).choice(cand, 300).astype(np.int64) for b in range(n_batches)]
             for w in range(n_streams)]
    want = []
    for w in range(n_streams):
        r = gs.RNG(100 + w)
        want.append([_pack_run(gs, G_, r, roots[w][b], fan, None) for b in range(n_batches)])
    first = ctypes.c_void_p()
    L.check(L.lib().gs_team_create(2 * n_streams, ctypes.byref(first)))
    teams = [first]
    for _ in range(n_streams - 1):
        t = ctypes.c_void_p()
        L.check(L.lib().gs_team_create_shared(first, ctypes.byref(t)))
        teams.append(t)
    got = [[None] * n_batches for _ in range(n_streams)]
    errors = []

    def stream(w):
        try:
            r = gs.RNG(100 + w)
            bound = int(L.lib().gs_sample_pack_bound_multi(G_.handle, 300, 300, fan.ctypes.data, nh))
            for b in range(n_batches):
                buf = np.full(bound, -7, np.int32)
                sizes = np.empty(4 * nh, np.int64)
                offs = np.empty(L.GS_MAX_HOPS * L.GS_PK_NFIELDS, np.int64)
                used = ctypes.c_int64()
                L.check(L.lib().gs_sample_pack_run_multi_team(
                    G_.handle, r._h, roots[w][b].ctypes.data, 300, 300, fan.ctypes.data, nh, 0, buf.ctypes.data,
                    bound, sizes.ctypes.data, offs.ctypes.data, ctypes.byref(used), teams[w]))
                got[w][b] = (buf[:used.value].copy(), sizes.reshape(nh, 4).copy())
        except Exception as e:  # surfaced below
            errors.append(e)

    try:
        th = [threading.Thread(target=stream, args=(w,)) for w in range(n_streams)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for t in reversed(teams):
            L.lib().gs_team_destroy(t)
    assert not errors, errors
    for w in range(n_streams):
        for b in range(n_batches):
            assert np.array_equal(got[w][b][0], want[w][b][0]), (w, b)
            assert np.array_equal(got[w][b][1], want[w][b][1]), (w, b)


@pytest.mark.parametrize("scale,pairs,batch", [(12, 40_000, 64), (16, 600_000, 512)])
def test_runner_pack_matches_oracle_per_root(gs, scale, pairs, batch):
    """The pack the runner's sampler threads write (gs_sample_pack_run_multi_team
    with a helper team) decoded per root and per hop against
    oracle.sample_layers on the same stream — the check the GPU suite runs at
    the rmat2m / rmat16m sizes (tests/fullsize_parity.py)."""
    from tests.fullsize_parity import check_pack_vs_oracle
    src, dst = gs.rmat_pairs(scale, pairs, seed=5)
    n = 1 << scale
    graph = gs.CSRGraph.from_pairs(src, dst, n)
    adj = Adjacency(src, dst, n)
    cands = np.nonzero(graph.degrees() > 0)[0]
    roots = cands[np.random.default_rng(3).permutation(len(cands))[:batch]]
    check_pack_vs_oracle(graph, adj, roots, [25, 10], seed=77)
