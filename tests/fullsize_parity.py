"""Full-size sampling and embedding parity against the oracle (shared by
test_gpu_fullsize.py and test_gpu_fullsize16m.py).

The pack checked is the one the training runner's sampler threads produce:
gs_sample_pack_run_multi_team with a helper team (runtime/runner.hip's
sampler_loop calls exactly this), decoded field by field, against
oracle.sample_layers on the same `random` stream (models.py:246-251 over
_get_unique_neighs_list, :277-289):

* hop 1 (roots -> L1): every root's neighbourhood (its sampled set minus self,
  models.py:297-298) and self position, through the L1 frontier order — which
  must equal the oracle's union list element for element (CPython set order,
  :286); the transposed lists are the exact inverse of the neighbourhoods;
* hop 2 (L1 -> L0): the destinations are L1 in that order; each one's sampled
  CSR entries name exactly the oracle's sampled set minus self (the reference
  keeps the set, so membership is the bit-exact content); |L0| — the union of
  the frontier and every sample — equals the oracle's union;
* the stream consumed exactly the oracle's words (state equal afterwards).
"""
import ctypes
import importlib
import random

import numpy as np

import oracle

_lib = importlib.import_module("graphsage-pytorch_amd._lib")
sampler = importlib.import_module("graphsage-pytorch_amd.sampler")


def runner_pack(graph, rng, roots, fanouts, helpers=1):
    """The runner's pack of one batch: (buf, hop_sizes[L, 4], offsets[8, 9])."""
    lib = _lib.lib()
    roots = np.ascontiguousarray(roots, np.int64)
    fan = np.ascontiguousarray(fanouts, np.int32)
    L, n = len(fan), len(roots)
    bound = int(lib.gs_sample_pack_bound(graph.handle, n, fan.ctypes.data, L)) + n
    buf = np.zeros(bound, np.int32)
    sizes = np.zeros(4 * _lib.GS_MAX_HOPS, np.int64)
    offs = np.zeros(_lib.GS_MAX_HOPS * _lib.GS_PK_NFIELDS, np.int64)
    used = ctypes.c_int64()
    team = ctypes.c_void_p()
    _lib.check(lib.gs_team_create(helpers, ctypes.byref(team)))
    try:
        _lib.check(lib.gs_sample_pack_run_multi_team(graph.handle, rng._h, roots.ctypes.data, n, n, fan.ctypes.data,
                                                     L, 0, buf.ctypes.data, bound, sizes.ctypes.data,
                                                     offs.ctypes.data, ctypes.byref(used), team))
    finally:
        lib.gs_team_destroy(team)
    return buf[:used.value], sizes.reshape(-1, 4)[:L], offs.reshape(_lib.GS_MAX_HOPS, _lib.GS_PK_NFIELDS)


def check_pack_vs_oracle(graph, adj, roots, fanouts, seed):
    """Decode the runner's 2-hop pack for `roots` drawn from random.seed(seed)
    and compare it with the oracle's hops from the same stream; returns the
    oracle's hops (for the embedding check)."""
    assert len(fanouts) == 2
    rng = sampler.RNG(seed)
    buf, sizes, off = runner_pack(graph, rng, roots, fanouts)
    ref_rng = random.Random(seed)
    hops = oracle.sample_layers(adj, [int(x) for x in roots], fanouts, ref_rng)
    (f0, samp0, idx0, union0), (f1, samp1, idx1, union1) = hops
    n0, n1 = len(roots), len(union0)
    # hop 1: sizes, then the frontier L1 in CPython set order
    assert sizes[0, 0] == n0 and sizes[0, 2] == n1, (sizes, n0, n1)
    assert sizes[1, 0] == n1
    l1 = buf[off[1, _lib.GS_PK_DST_IDS]:off[1, _lib.GS_PK_DST_IDS] + n1]
    np.testing.assert_array_equal(l1, np.asarray(union0, np.int64))
    nptr = buf[off[0, _lib.GS_PK_NBR_PTR]:off[0, _lib.GS_PK_NBR_PTR] + n0 + 1]
    nbr = buf[off[0, _lib.GS_PK_NBR]:off[0, _lib.GS_PK_NBR] + int(nptr[-1])]
    slf = buf[off[0, _lib.GS_PK_SELF]:off[0, _lib.GS_PK_SELF] + n0]
    tptr = buf[off[0, _lib.GS_PK_TPTR]:off[0, _lib.GS_PK_TPTR] + n1 + 1]
    tidx = buf[off[0, _lib.GS_PK_TIDX]:off[0, _lib.GS_PK_TIDX] + int(tptr[-1])]
    for r, v in enumerate(roots):
        lst = nbr[nptr[r]:nptr[r + 1]]
        assert np.all(np.diff(lst) > 0)  # union-local ids ascending (the dense mask's column order)
        assert set(l1[lst].tolist()) == samp0[r] - {int(v)}, r
        assert int(l1[slf[r]]) == int(v)
    # transposed lists: the inverse of (neighbourhoods, self rows), destinations ascending
    inv = [[] for _ in range(n1)]
    for r in range(n0):
        inv[slf[r]].append(-(r + 1))
        for c in nbr[nptr[r]:nptr[r + 1]]:
            inv[c].append(r)
    for c in range(n1):
        got = tidx[tptr[c]:tptr[c + 1]].tolist()
        assert sorted(got) == sorted(inv[c]), c
    # hop 2: L1's sampled entries -> ids, against the oracle's sets; |L0|
    row_ptr = graph.row_ptr()
    col = graph.col()
    pptr = buf[off[1, _lib.GS_PK_POS_PTR]:off[1, _lib.GS_PK_POS_PTR] + n1 + 1]
    ent = buf[off[1, _lib.GS_PK_POS]:off[1, _lib.GS_PK_POS] + int(pptr[-1])]
    assert sizes[1, 1] == len(ent)
    ids = col[ent.astype(np.int64)]
    for r, v in enumerate(l1):
        e = ent[pptr[r]:pptr[r + 1]].astype(np.int64)
        assert np.all((e >= row_ptr[v]) & (e < row_ptr[v + 1])), r  # entries inside the destination's row
        assert set(ids[pptr[r]:pptr[r + 1]].tolist()) | {int(v)} == samp1[r], r
    assert set(ids.tolist()) | set(l1.tolist()) == set(union1)
    assert len(set(ids.tolist()) | set(l1.tolist())) == len(union1)
    # the stream: exactly the oracle's words
    mt, pos = rng.getstate()
    ver, internal, _ = ref_rng.getstate()
    assert pos == internal[624] and tuple(int(x) for x in mt) == internal[:624]
    return hops


def check_embeddings_vs_oracle(gs_models, graph, X, X_rows, hops, roots, fanouts, weights, seed, device,
                               tol=1e-5):
    """The drop-in module's forward of `roots` drawn from random.seed(seed)
    (models.py:241-269, its own sampling on its own stream) against
    oracle.forward_dense over the oracle's hops of the same stream (the
    dense-mask reference formulation, models.py:291-330) at `tol`.  X_rows
    indexes the feature table as the oracle needs (a CPU tensor or a row
    view of the device table)."""
    import torch
    H = weights[0].shape[0]
    m = gs_models.GraphSage(2, X.shape[1], H, X, graph, device, fanouts=list(fanouts),
                            rng=sampler.RNG(seed)).to(device)
    with torch.no_grad():
        for i in (1, 2):
            getattr(m, f"sage_layer{i}").weight.copy_(weights[i - 1])
        emb = m([int(x) for x in roots]).cpu()
        ref = oracle.forward_dense(hops, X_rows, [w.detach().cpu() for w in weights])
    assert emb.shape == ref.shape
    torch.testing.assert_close(emb, ref, atol=tol, rtol=tol)
    return emb


def check_timed_steps_vs_oracle(train, wl, adj, X_dev, X_rows, fanouts, classes, agg="MEAN", bf16=False,
                                tols=(1e-5, 1e-5), n_steps=2, streams=2, seed=824, hidden=128):
    """The bench's own training step against the oracle, step by step.

    The native path is exactly what bench.py times: NativeTrainer + Runner
    (`streams` sampler streams held until release, the resolved-id gather into
    the [self | agg] slot on the side stream, the layer-1 forward, the fused
    top launch, the layer-2 backward, the layer-1 dW and its slab sum), all
    n_steps in ONE gs_runner_run call — so every step after the first runs the
    layer-1 forward instance that applies the previous step's deferred clip +
    SGD (linear_fwd_wide_kernel<..., true>) and reads the speculative W1 the
    previous slab sum wrote.  gs_trainer_capture copies each step's root
    embeddings and its flat gradient [dW1 | dW2 | dWc | dbc] before the clip +
    SGD; oracle.train_step_dense (autograd over the dense-mask restatement,
    models.py:241-330, utils.py:157-187) runs the same batches on the same
    `random` streams and its weights carry over step to step.  tols[i]: the
    tolerance (atol = rtol) of step i's embeddings and gradients."""
    import time
    import torch
    B = len(wl["batches"][0])
    batches = wl["batches"][:n_steps]
    tr = train.NativeTrainer(wl["graph"], X_dev, wl["labels"], classes, fanouts=fanouts, agg_func=agg, seed=seed)
    emb, grads = tr.capture(n_steps, B)
    r = train.Runner(tr, wl["graph"], batches, [train.make_rng(seed, 0, w) for w in range(streams)], fanouts,
                     fail_empty=agg == "MAX", depth=2, hold=True)
    time.sleep(0.1)
    r.release(len(batches))
    r.run(n_steps)  # one call: the deferred update is pending between the steps
    torch.cuda.synchronize()
    r.close()
    assert tr.captured() == n_steps
    emb, grads = emb.cpu(), grads.cpu()
    labels = wl["labels"].cpu().long()
    feat = X_dev.shape[1]
    sage_w, cw, cb = train.reference_init(2, feat, hidden, classes, False, seed)
    W = [w.clone().requires_grad_(True) for w in sage_w]
    cw, cb = cw.clone().requires_grad_(True), cb.clone().requires_grad_(True)
    rngs = [random.Random(train.rank_seed(seed, 0, w)) for w in range(streams)]
    worst = []
    for i, roots in enumerate(batches):
        cap = {}
        oracle.train_step_dense(adj, roots.tolist(), fanouts, X_rows, W, cw, cb, labels[torch.from_numpy(roots)],
                                agg=agg, rng=rngs[i % streams], bf16_layer1=bf16, capture=cap)
        tol = tols[min(i, len(tols) - 1)]
        e_ref, g_ref = cap["emb"], cap["grads"]
        assert g_ref.numel() == grads.shape[1]
        torch.testing.assert_close(emb[i, :len(roots)], e_ref, atol=tol, rtol=tol, msg=lambda m: f"step {i} emb: {m}")
        torch.testing.assert_close(grads[i], g_ref, atol=tol, rtol=tol, msg=lambda m: f"step {i} grads: {m}")
        worst.append((float((emb[i, :len(roots)] - e_ref).abs().max()), float((grads[i] - g_ref).abs().max()),
                      float(g_ref.abs().max())))
    return worst
