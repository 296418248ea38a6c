"""torch-tensor front-end of the gfx950 kernels (C-ABI in include/graphsage_amd.h).

Every function checks shapes/dtypes/devices, then launches on torch's current
stream of the tensors' device.  There is deliberately no CPU path: tensors
that are not on a HIP device raise.
"""
import torch

from . import _lib
from ._lib import check, lib, ptr

_DT = {torch.float32: _lib.GS_F32, torch.bfloat16: _lib.GS_BF16}
_AGG = {"MEAN": _lib.GS_AGG_MEAN, "MAX": _lib.GS_AGG_MAX}


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("graphsage_amd kernels run on a HIP device; got a CPU tensor "
                               "(move raw_features / the model to cuda)")


def _stream(t):
    return _lib.stream_ptr(t.device)


def _i32(t):
    if t is not None and t.dtype != torch.int32:
        raise TypeError("index tensors must be int32")
    return t


def agg_op(agg_func):
    try:
        return _AGG[agg_func]
    except KeyError:
        raise ValueError(f"agg_func must be 'MEAN' or 'MAX', got {agg_func!r}") from None


def agg_fwd(agg_func, X, ptr_, idx, out, *, row_ptr=None, col=None, dst_ids=None, gcn=False,
            argmax=None):
    """Segmented mean/max of rows of X (models.py:291-330); see gs_agg_fwd."""
    _dev(X, ptr_, idx, out)
    if X.dtype not in _DT or out.dtype != X.dtype:
        raise TypeError("X/out must share dtype float32 or bfloat16")
    n_dst = ptr_.numel() - 1
    F = X.shape[1]
    if out.shape[0] < n_dst or out.shape[1] < F:
        raise ValueError("out too small")
    check(lib().gs_agg_fwd(agg_op(agg_func), _DT[X.dtype], ptr(X), X.stride(0), F, n_dst,
                           ptr(_i32(ptr_)), ptr(_i32(idx)), ptr(row_ptr), ptr(_i32(col)),
                           ptr(_i32(dst_ids)), int(bool(gcn)), ptr(out), _DT[out.dtype],
                           out.stride(0), ptr(_i32(argmax)), _stream(X)))
    return out


def sage_linear_fwd(A, Wd, out, *, Xs=None, sidx=None, relu=True):
    """relu([Xs[sidx] | A] · Wᵀ) (models.py:209-220); Xs=None is the gcn form."""
    _dev(A, Wd, out, Xs)
    n, F = A.shape
    H = Wd.shape[0]
    K = 2 * F if Xs is not None else F
    if Wd.shape[1] != K or Wd.dtype != A.dtype or (Xs is not None and Xs.dtype != A.dtype):
        raise ValueError(f"weight must be [{H}, {K}] in the activation dtype")
    if out.dtype != torch.float32 or out.shape[0] < n or out.shape[1] < H:
        raise ValueError("out must be fp32 [n, H]")
    check(lib().gs_sage_linear_fwd(_DT[A.dtype], n, F, H, ptr(Xs), Xs.stride(0) if Xs is not None else 0,
                                   ptr(_i32(sidx)), ptr(A), A.stride(0), ptr(Wd), ptr(out),
                                   out.stride(0), int(bool(relu)), _stream(A)))
    return out


def sage1_supported(dtype, F, H, gcn):
    return bool(lib().gs_sage1_fwd_supported(_DT[dtype], F, H, int(bool(gcn))))


def sage1_fwd(agg_func, X, ptr_, ent, col, dst_ids, W, agg_out, out, *, gcn=False, relu=True):
    """Fused layer 1 (gs_sage1_fwd): gather-aggregate over absolute CSR
    entries + relu([X[dst] | agg] · Wᵀ); fills agg_out and out."""
    _dev(X, ptr_, ent, col, dst_ids, W, agg_out, out)  # col None: explicit lists (layers >= 2)
    n_dst = ptr_.numel() - 1
    F = X.shape[1]
    H = W.shape[0]
    if W.dtype != X.dtype or agg_out.dtype != X.dtype or out.dtype != torch.float32:
        raise TypeError("W / agg_out must share X's dtype; out is fp32")
    check(lib().gs_sage1_fwd(agg_op(agg_func), _DT[X.dtype], ptr(X), X.stride(0), F, H, n_dst, ptr(_i32(ptr_)),
                             ptr(_i32(ent)), ptr(_i32(col)), ptr(_i32(dst_ids)), int(bool(gcn)), ptr(W),
                             ptr(agg_out), agg_out.stride(0), ptr(out), out.stride(0), int(bool(relu)),
                             _stream(X)))
    return out


def linear_dw_workspace(n, K, H, device):
    nbytes = int(lib().gs_sage_linear_bwd_weight_ws(n, K, H))
    return torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=device), nbytes


def sage_linear_bwd_weight(A, dout, out, dW, *, Xs=None, sidx=None, relu=True, ws=None):
    """dW = (dOut ⊙ relu')ᵀ · [Xs[sidx] | A]."""
    _dev(A, dout, out, dW, Xs)
    n, F = A.shape
    H = dW.shape[0]
    K = 2 * F if Xs is not None else F
    if dW.shape[1] != K or dW.dtype != torch.float32:
        raise ValueError("dW must be fp32 [H, K]")
    if ws is None:
        ws, nbytes = linear_dw_workspace(n, K, H, A.device)
    else:
        ws, nbytes = ws
    check(lib().gs_sage_linear_bwd_weight(_DT[A.dtype], n, F, H, ptr(Xs),
                                          Xs.stride(0) if Xs is not None else 0, ptr(_i32(sidx)),
                                          ptr(A), A.stride(0), ptr(dout), ptr(out), out.stride(0),
                                          int(bool(relu)), ptr(dW), ptr(ws), nbytes, _stream(A)))
    return dW


def sage_linear_bwd_input(dout, out, W, dA, *, dSelf=None, relu=True):
    """[dSelf | dA] = (dOut ⊙ relu') · W."""
    _dev(dout, out, W, dA, dSelf)
    n, H = dout.shape
    F = dA.shape[1]
    if dSelf is not None and dSelf.stride(0) != dA.stride(0):
        raise ValueError("dSelf and dA must share a leading dimension")
    check(lib().gs_sage_linear_bwd_input(n, F, H, ptr(dout), ptr(out), out.stride(0), int(bool(relu)),
                                         ptr(W), ptr(dSelf), ptr(dA), dA.stride(0), _stream(dout)))


def agg_bwd(agg_func, tptr, tidx, ptr_, dA, dH, *, dSelf=None, argmax=None, Hprev=None):
    """Transposed gather of the aggregate / self-row gradients (+ relu mask)."""
    _dev(tptr, tidx, ptr_, dA, dH, dSelf, argmax, Hprev)
    n_src = tptr.numel() - 1
    F = dA.shape[1]
    ldh = dH.stride(0)
    if Hprev is not None and Hprev.stride(0) != ldh:
        raise ValueError("Hprev and dH must share a leading dimension")
    check(lib().gs_agg_bwd(agg_op(agg_func), n_src, F, ptr(_i32(tptr)), ptr(_i32(tidx)),
                           ptr(_i32(ptr_)), ptr(dA), ptr(dSelf), dA.stride(0), ptr(_i32(argmax)),
                           ptr(Hprev), ldh, ptr(dH), _stream(dA)))
    return dH


def cls_nll_workspace(B, D, C, device):
    return torch.empty(int(lib().gs_cls_nll_ws_floats(B, D, C)), dtype=torch.float32, device=device)


def cls_nll_fwd_bwd(E, Wc, bc, labels, loss, dE, dWc, dbc, ws, roots=None, mask_relu=False):
    """Classification + NLL forward/backward; labels[roots[i]] is row i's label
    (labels[i] without roots).  mask_relu zeroes dE where E <= 0."""
    _dev(E, Wc, bc, labels, loss, dE, dWc, dbc, ws, roots)
    B, D = E.shape
    C = Wc.shape[0]
    check(lib().gs_cls_nll_fwd_bwd(B, D, C, ptr(E), ptr(Wc), ptr(bc), ptr(_i32(labels)), ptr(_i32(roots)),
                                   int(bool(mask_relu)), ptr(loss),
                                   ptr(dE), ptr(dWc), ptr(dbc), ptr(ws), _stream(E)))


def clip_sgd(goff, params, grads, grad_scale, max_norm, lr, ws):
    import numpy as np
    _dev(params, grads, ws)
    go = np.ascontiguousarray(goff, dtype=np.int64)
    check(lib().gs_clip_sgd(len(go) - 1, ptr(go), ptr(params), ptr(grads), float(grad_scale),
                            float(max_norm), float(lr), ptr(ws), _stream(params)))


def fill_uniform(X, seed):
    _dev(X)
    check(lib().gs_fill_uniform(ptr(X), _DT[X.dtype], X.shape[0], X.shape[1], X.stride(0),
                                int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(X)))
    return X


def cast_bf16(src, dst):
    _dev(src, dst)
    if src.numel() != dst.numel() or dst.dtype != torch.bfloat16 or src.dtype != torch.float32:
        raise ValueError("cast_bf16: fp32 -> bf16 of equal size")
    check(lib().gs_cast_f32_bf16(ptr(src), ptr(dst), src.numel(), _stream(src)))
    return dst
