"""Kernel-level parity on the MI355X: every HIP kernel against a plain torch
fp32 (or exact integer) statement of the same op, including ragged/empty
segments, hub rows, F not a multiple of 4/64, bf16 and gcn mode."""
import importlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ops = importlib.import_module("graphsage-pytorch_amd.hip_ops")
DEV = torch.device("cuda", 0)


def _rand_graph(gs, n, m, seed):
    rs = np.random.RandomState(seed)
    src = np.where(rs.random_sample(m) < 0.2, rs.randint(0, 5, m), rs.randint(0, n, m))
    dst = rs.randint(0, n, m)
    keep = src != dst
    return gs.CSRGraph.from_pairs(src[keep], dst[keep], n)


def _expand_ref(graph, s, hop, X, agg, gcn):
    """numpy statement of the layer-1 neighbourhood: sampled ids minus self (+ self in gcn)."""
    h = s.hop(hop)
    rp, col = graph.row_ptr(), graph.col()
    Xf = X.float().cpu()
    out = []
    for r in range(h.n_dst):
        v = int(h.dst_ids[r])
        ids = [int(col[rp[v] + p]) for p in h.pos[h.pos_ptr[r]:h.pos_ptr[r + 1]]]
        ids = [x for x in ids if x != v] + ([v] if gcn else [])
        rows = Xf[torch.tensor(ids, dtype=torch.long)] if ids else torch.zeros(0, X.shape[1])
        if agg == "MEAN":
            out.append(rows.sum(0) / len(ids) if ids else torch.full((X.shape[1],), float("nan")))
        else:
            out.append(rows.max(0)[0])
    return torch.stack(out)


@pytest.mark.parametrize("F", [256, 128, 100, 1433, 64, 8])
@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("gcn", [False, True])
def test_agg_fwd_expand(gs, F, agg, dtype, gcn):
    graph = _rand_graph(gs, 500, 6000, F)
    X = torch.randn(500, F, device=DEV).to(dtype)
    roots = np.nonzero(graph.degrees())[0][:80]
    s = gs.sample(graph, gs.RNG(F), roots, [25, 10], gcn=gcn)
    if agg == "MAX" and s.n_empty(2):
        pytest.skip("empty neighbourhood (MAX raises in the model layer)")
    models = importlib.import_module("graphsage-pytorch_amd.models")
    ds = models.DeviceSample(s, DEV)
    rp, cl = graph.device_csr(DEV)
    n_dst = s.sizes(2)[0]
    out = torch.empty(n_dst, F, dtype=dtype, device=DEV)
    ops.agg_fwd(agg, X, ds.field(2, "pos_ptr"), ds.field(2, "pos"), out, row_ptr=None, col=cl,
                dst_ids=ds.field(2, "dst_ids"), gcn=gcn)  # pack: absolute entries
    ref = _expand_ref(graph, s, 2, X, agg, gcn)
    got = out.float().cpu()
    if dtype == torch.float32:
        torch.testing.assert_close(got, ref, atol=1e-6, rtol=1e-5, equal_nan=True)
    else:
        torch.testing.assert_close(got, ref.to(torch.bfloat16).float(), atol=2e-2, rtol=1e-2, equal_nan=True)
    # relative positions through row_ptr (hop view layout)
    h = s.hop(2)
    pos_rel = torch.from_numpy(h.pos.astype(np.int32)).to(DEV)
    out.zero_()
    ops.agg_fwd(agg, X, ds.field(2, "pos_ptr"), pos_rel, out, row_ptr=rp, col=cl,
                dst_ids=ds.field(2, "dst_ids"), gcn=gcn)
    got = out.float().cpu()
    if dtype == torch.float32:
        torch.testing.assert_close(got, ref, atol=1e-6, rtol=1e-5, equal_nan=True)
    else:
        torch.testing.assert_close(got, ref.to(torch.bfloat16).float(), atol=2e-2, rtol=1e-2, equal_nan=True)


@pytest.mark.parametrize("F", [128, 100, 7])
def test_agg_fwd_explicit_max_argmax_first_index(gs, F):
    rs = np.random.RandomState(F)
    n_src, n_dst = 300, 120
    X = torch.from_numpy(rs.randint(-3, 4, (n_src, F)).astype(np.float32)).to(DEV)  # many ties
    lists = [sorted(rs.choice(n_src, rs.randint(1, 30), replace=False).tolist()) for _ in range(n_dst)]
    lists[0] = list(range(n_src))  # a hub row
    ptr = torch.tensor(np.cumsum([0] + [len(l) for l in lists]), dtype=torch.int32, device=DEV)
    idx = torch.tensor([x for l in lists for x in l], dtype=torch.int32, device=DEV)
    out = torch.empty(n_dst, F, device=DEV)
    am = torch.empty(n_dst, F, dtype=torch.int32, device=DEV)
    ops.agg_fwd("MAX", X, ptr, idx, out, argmax=am)
    Xc = X.cpu()
    for r, l in enumerate(lists):
        rows = Xc[torch.tensor(l)]
        v, i = rows.max(0)
        assert torch.equal(out[r].cpu(), v)
        # first maximum in ascending source order
        first = torch.tensor([l[int(torch.nonzero(rows[:, f] == v[f])[0])] for f in range(F)], dtype=torch.int32)
        assert torch.equal(am[r].cpu(), first)


@pytest.mark.parametrize("n,F,H", [(1, 256, 128), (37, 128, 128), (300, 100, 64), (4321, 256, 128),
                                   (50, 1433, 128), (64, 8, 16), (129, 256, 256), (5000, 64, 48),
                                   (3000, 20, 16)])
@pytest.mark.parametrize("gcn", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sage_linear_fwd_bwd(n, F, H, gcn, dtype):
    torch.manual_seed(n + F)
    n_src = n + 13
    Xs = torch.randn(n_src, F, device=DEV)
    A = torch.randn(n, F, device=DEV)
    sidx = torch.randint(0, n_src, (n,), dtype=torch.int32, device=DEV)
    K = F if gcn else 2 * F
    W = torch.randn(H, K, device=DEV) * 0.05
    Xd, Ad, Wd = Xs.to(dtype), A.to(dtype), W.to(dtype)
    out = torch.empty(n, H, device=DEV)
    ops.sage_linear_fwd(Ad, Wd, out, Xs=None if gcn else Xd, sidx=None if gcn else sidx)
    comb = Ad.float() if gcn else torch.cat([Xd.float()[sidx.long()], Ad.float()], 1)
    ref = torch.relu(comb.double() @ Wd.float().double().t()).float()
    tol = dict(atol=1e-4, rtol=1e-4) if dtype == torch.float32 else dict(atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(out, ref, **tol)
    # backward
    dout = torch.randn(n, H, device=DEV)
    dZ = dout * (ref > 0)
    dW = torch.empty(H, K, device=DEV)
    ops.sage_linear_bwd_weight(Ad, dout, out, dW, Xs=None if gcn else Xd, sidx=None if gcn else sidx)
    torch.testing.assert_close(dW, (dZ.double().t() @ comb.double()).float(), atol=2e-4, rtol=1e-4)
    dIn = torch.empty(n, K, device=DEV)
    ops.sage_linear_bwd_input(dout, out, W, dIn if gcn else dIn[:, F:], dSelf=None if gcn else dIn[:, :F])
    torch.testing.assert_close(dIn, (dZ.double() @ W.double()).float(), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("n,F,H", [(1, 256, 128), (37, 128, 128), (4321, 256, 128), (4400, 256, 128),
                                   (513, 128, 64), (100, 64, 32), (2048, 256, 256), (6200, 256, 128),
                                   (17, 256, 128)])
@pytest.mark.parametrize("gcn", [False, True])
def test_wide_forward_bitwise_equals_chunked_kernel(n, F, H, gcn):
    """The 32-row W-in-LDS forward (linear_fwd_wide_kernel, taken for 16-B
    aligned operands) feeds the same MFMA operands in the same order as the
    16-row chunked kernel (linear_fwd_kernel, taken here by an aggregate whose
    rows are not 16-B aligned): outputs bitwise equal, partial last tiles and
    the self-row gather included."""
    torch.manual_seed(n + F + H)
    n_src = n + 29
    Xs = torch.randn(n_src, F, device=DEV)
    A = torch.randn(n, F, device=DEV)
    A_odd = torch.empty(n, F + 1, device=DEV)[:, 1:]  # lda = F + 1, row 0 at +4 B: the chunked kernel
    A_odd.copy_(A)
    sidx = torch.randint(0, n_src, (n,), dtype=torch.int32, device=DEV)
    K = F if gcn else 2 * F
    W = torch.randn(H, K, device=DEV) * 0.05
    outs = []
    for a in (A, A_odd):
        out = torch.full((n, H), float("nan"), device=DEV)
        ops.sage_linear_fwd(a, W, out, Xs=None if gcn else Xs, sidx=None if gcn else sidx)
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
@pytest.mark.parametrize("F", [128, 36, 5])
def test_agg_bwd_matches_autograd(agg, F):
    rs = np.random.RandomState(F)
    n_src, n_dst = 200, 90
    lists = [sorted(rs.choice(n_src, rs.randint(1, 12), replace=False).tolist()) for _ in range(n_dst)]
    self_of = rs.permutation(n_src)[:n_dst]
    H = torch.randn(n_src, F, device=DEV)
    Hr = torch.relu(H)
    ptr = torch.tensor(np.cumsum([0] + [len(l) for l in lists]), dtype=torch.int32, device=DEV)
    idx = torch.tensor([x for l in lists for x in l], dtype=torch.int32, device=DEV)
    a = torch.empty(n_dst, F, device=DEV)
    am = torch.empty(n_dst, F, dtype=torch.int32, device=DEV) if agg == "MAX" else None
    ops.agg_fwd(agg, Hr, ptr, idx, a, argmax=am)
    # transposed lists incl. self edges (-(r+1))
    ent = [(c, r) for r, l in enumerate(lists) for c in l] + [(int(self_of[r]), -(r + 1)) for r in range(n_dst)]
    ent.sort(key=lambda t: (t[0], t[1] if t[1] >= 0 else -t[1] - 1))
    tptr = torch.tensor(np.searchsorted([c for c, _ in ent], np.arange(n_src + 1)), dtype=torch.int32, device=DEV)
    tidx = torch.tensor([r for _, r in ent], dtype=torch.int32, device=DEV)
    dA = torch.randn(n_dst, F, device=DEV)
    dS = torch.randn(n_dst, F, device=DEV)
    dH = torch.empty(n_src, F, device=DEV)
    ops.agg_bwd(agg, tptr, tidx, ptr, dA, dH, dSelf=dS, argmax=am, Hprev=Hr)
    # autograd reference
    Ht = H.detach().clone().requires_grad_(True)
    R = torch.relu(Ht)
    outs = []
    for l in lists:
        rows = R[torch.tensor(l, device=DEV)]
        outs.append(rows.mean(0) if agg == "MEAN" else rows.max(0)[0])
    ref_a = torch.stack(outs)
    torch.testing.assert_close(a, ref_a, atol=1e-6, rtol=1e-5)
    ((ref_a * dA).sum() + (R[torch.tensor(self_of, device=DEV)] * dS).sum()).backward()
    torch.testing.assert_close(dH, Ht.grad, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("B,D,C,use_roots,mask", [
    (512, 128, 16, False, False),
    (512, 128, 16, True, True),
    (37, 64, 7, True, False),        # ragged last block, Cora-sized head
    (100, 256, 200, True, True),     # Wc too large for LDS -> read from global
    (1, 8, 1, False, False),
    (9705, 128, 3, False, False),    # Pubmed's extended batch: 32 rows per block
    (6001, 128, 3, True, True),      # grown rows on the FAST path, ragged last block
])
def test_cls_nll_matches_torch(B, D, C, use_roots, mask):
    torch.manual_seed(0)
    n_nodes = 3 * B + 5
    H = torch.randn(B, D, device=DEV)
    E = (torch.relu(H) if mask else H).requires_grad_(True)
    Wc = (torch.randn(C, D, device=DEV) * 0.1).requires_grad_(True)
    bc = torch.randn(C, device=DEV, requires_grad=True)
    labels = torch.randint(0, C, (n_nodes,), device=DEV, dtype=torch.int32)
    roots = torch.randperm(n_nodes, device=DEV)[:B].int() if use_roots else None
    y = (labels[roots.long()] if use_roots else labels[:B]).long()
    logp = torch.log_softmax(E @ Wc.t() + bc, 1)
    loss = -torch.sum(logp[range(B), y], 0) / B
    loss.backward()
    dE_ref = E.grad * (E.detach() > 0) if mask else E.grad
    out = [torch.empty(1, device=DEV), torch.empty(B, D, device=DEV), torch.empty(C, D, device=DEV),
           torch.empty(C, device=DEV)]
    ws = ops.cls_nll_workspace(B, D, C, DEV)
    ops.cls_nll_fwd_bwd(E.detach(), Wc.detach(), bc.detach(), labels, *out, ws, roots=roots, mask_relu=mask)
    torch.testing.assert_close(out[0][0], loss.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out[1], dE_ref, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(out[2], Wc.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(out[3], bc.grad, atol=1e-6, rtol=1e-4)


def test_clip_sgd_matches_torch():
    torch.manual_seed(1)
    sizes = [1000, 333, 64, 7]
    p = torch.randn(sum(sizes), device=DEV)
    g = torch.randn(sum(sizes), device=DEV) * 3
    goff = np.array([0, 1333, sum(sizes)], np.int64)
    ref_p = p.clone()
    ref_g = g.clone() * 0.5
    for lo, hi in zip(goff[:-1], goff[1:]):
        nrm = ref_g[lo:hi].norm()
        ref_g[lo:hi] *= torch.clamp(5.0 / (nrm + 1e-6), max=1.0)
    ref_p -= 0.7 * ref_g
    ws = torch.empty(130, device=DEV)
    ops.clip_sgd(goff, p, g, 0.5, 5.0, 0.7, ws)
    torch.testing.assert_close(p, ref_p, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(g, ref_g, atol=1e-6, rtol=1e-5)


def test_fill_uniform_matches_host_hash():
    from tests.golden.synth import uniform_features
    X = torch.empty(1000, 77, device=DEV)
    ops.fill_uniform(X, 824)
    assert torch.equal(X.cpu(), torch.from_numpy(uniform_features(824, 1000, 77)))
    Xb = torch.empty(1000, 77, dtype=torch.bfloat16, device=DEV)
    ops.fill_uniform(Xb, 824)
    assert torch.equal(Xb.cpu(), X.cpu().to(torch.bfloat16))


@pytest.mark.parametrize("F,H", [(256, 128), (128, 64), (64, 256), (512, 128), (40, 16)])
@pytest.mark.parametrize("agg", ["MEAN", "MAX"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("gcn", [False, True])
def test_sage1_fused_equals_two_kernel_path(gs, F, H, agg, dtype, gcn):
    """gs_sage1_fwd == gs_agg_fwd (expand) + gs_sage_linear_fwd, bitwise."""
    if not ops.sage1_supported(dtype, F, H, gcn):
        pytest.skip("shape outside the fused kernel's LDS tile")
    graph = _rand_graph(gs, 700, 9000, F)
    X = torch.randn(700, F, device=DEV).to(dtype)
    roots = np.nonzero(graph.degrees())[0][:120]
    s = gs.sample(graph, gs.RNG(F + H), roots, [25, 70], gcn=gcn)  # > 64 entries per dst reach the slow path
    if agg == "MAX" and s.n_empty(2):
        pytest.skip("empty neighbourhood (MAX raises in the model layer)")
    models = importlib.import_module("graphsage-pytorch_amd.models")
    ds = models.DeviceSample(s, DEV)
    _, cl = graph.device_csr(DEV)
    n_dst = s.sizes(2)[0]
    K = F if gcn else 2 * F
    W = (torch.randn(H, K, device=DEV) * 0.05).to(dtype)
    ptr_, ent, dst = ds.field(2, "pos_ptr"), ds.field(2, "pos"), ds.field(2, "dst_ids")
    a_ref = torch.empty(n_dst, F, dtype=dtype, device=DEV)
    ops.agg_fwd(agg, X, ptr_, ent, a_ref, row_ptr=None, col=cl, dst_ids=dst, gcn=gcn)
    h_ref = torch.empty(n_dst, H, device=DEV)
    ops.sage_linear_fwd(a_ref, W, h_ref, Xs=None if gcn else X, sidx=dst)
    a = torch.empty_like(a_ref)
    h = torch.empty_like(h_ref)
    ops.sage1_fwd(agg, X, ptr_, ent, cl, dst, W, a, h, gcn=gcn)
    assert torch.equal(a.view(torch.int16) if dtype == torch.bfloat16 else a,
                       a_ref.view(torch.int16) if dtype == torch.bfloat16 else a_ref)
    assert torch.equal(h, h_ref)


@pytest.mark.parametrize("gcn", [False, True])
@pytest.mark.parametrize("H", [128, 64])
def test_sage1_explicit_equals_two_kernel_path(gs, gcn, H):
    """Explicit mode (layers >= 2): gs_sage1_fwd over the pack's NBR/SELF
    fields == gs_agg_fwd (explicit) + gs_sage_linear_fwd, bitwise."""
    graph = _rand_graph(gs, 600, 7000, 16)
    roots = np.nonzero(graph.degrees())[0][:100]
    s = gs.sample(graph, gs.RNG(H), roots, [25, 10], gcn=gcn)
    models = importlib.import_module("graphsage-pytorch_amd.models")
    ds = models.DeviceSample(s, DEV)
    n_src = s.sizes(1)[2]
    n_dst = s.sizes(1)[0]
    Hp = torch.randn(n_src, H, device=DEV)
    W = torch.randn(H, H if gcn else 2 * H, device=DEV) * 0.05
    ptr_, nbr, slf = ds.field(1, "nbr_ptr"), ds.field(1, "nbr"), ds.field(1, "self")
    a_ref = torch.empty(n_dst, H, device=DEV)
    ops.agg_fwd("MEAN", Hp, ptr_, nbr, a_ref)
    h_ref = torch.empty(n_dst, H, device=DEV)
    ops.sage_linear_fwd(a_ref, W, h_ref, Xs=None if gcn else Hp, sidx=slf)
    a, h = torch.empty_like(a_ref), torch.empty_like(h_ref)
    ops.sage1_fwd("MEAN", Hp, ptr_, nbr, None, slf, W, a, h, gcn=gcn)
    assert torch.equal(a, a_ref) and torch.equal(h, h_ref)
