"""Fused factorization-machine loss/gradient passes (``csrc/hip/fm.hip``) + torch CPU path.

forward:  fx = X w + 1/2 sum_f [(X V)^2 - (X∘X)(V∘V)]_f ,  S = X V
backward: g_w = X^T c,  g_V = X^T (c∘S) - V ∘ ((X∘X)^T c)
Reference: ``J/optimizer/FMHoagOptimizer.java:60-160``.
"""
from __future__ import annotations

import torch

from ._ext import check_cuda, hip, ptr, stream
from .sparse import chunk_reduce


def fm_forward(X, w_lin: torch.Tensor, V: torch.Tensor):
    """(fx float64 [n], S float32 [n, k]) for the rows of SparseMatrix X; V: [F, k] view,
    float32 or bfloat16 (bf16 working copy of the SGD path: half the gathered bytes)."""
    k = V.shape[1]
    if X.device.type == "cuda" and 0 <= k <= 64:
        check_cuda(w_lin, V)
        assert V.dtype in (torch.float32, torch.bfloat16)
        V = V.contiguous()
        fx = torch.empty(X.n, dtype=torch.float64, device=X.device)
        S = torch.empty((X.n, k), dtype=torch.float32, device=X.device)
        hip().fm_forward(ptr(X.indptr), ptr(X.indices), ptr(X.values), X.n, ptr(w_lin),
                         ptr(V) if k > 0 else 0, k, ptr(fx), ptr(S) if k > 0 else 0,
                         1 if V.dtype == torch.bfloat16 else 0, stream(w_lin))
        return fx, S
    V = V.float()
    fx = X.matmul(w_lin).double()
    S = X.matmul(V.contiguous())
    Q = X.matmul((V * V).contiguous(), square=True)
    return fx + 0.5 * (S.double() ** 2 - Q.double()).sum(1), S


def fm_backward(X, c: torch.Tensor, S: torch.Tensor, V: torch.Tensor, g_lin: torch.Tensor, gV: torch.Tensor):
    """g_lin[F] = X^T c and gV[F, k] = X^T (c∘S) - V ∘ ((X∘X)^T c) (both overwritten)."""
    k = V.shape[1]
    c = c.float().contiguous()
    if X.device.type == "cuda" and 1 <= k <= 64:
        if X._csc is None:
            X._build_csc()
        check_cuda(c, S, V, g_lin, gV)
        part = torch.empty((max(X.n_chunks, 1), k + 2), dtype=torch.float32, device=X.device)
        tot = torch.empty((X.ncols, k + 2), dtype=torch.float32, device=X.device)
        h, s = hip(), stream(c)
        h.fm_backward(ptr(X.chunk_bounds), ptr(X.chunk_end_b), X.n_chunks, ptr(X.csc_rows), ptr(X.csc_vals), ptr(c),
                      ptr(S.contiguous()), k, ptr(part), s)
        chunk_reduce(X.chunk_ptr, X.ncols, part, k + 2, tot, k + 2, 1.0, 0, ptr(X.chunk_ids), s, X.heavy_cols)
        g_lin.copy_(tot[:, k])
        gV.copy_(tot[:, :k])
        gV.addcmul_(V, tot[:, k + 1:k + 2], value=-1.0)
        return g_lin, gV
    X.t_matmul(c, out=g_lin)
    X.t_matmul((c[:, None] * S).contiguous(), out=gV)
    sq = X.t_matmul(c, square=True)
    gV.sub_(V * sq[:, None])
    return g_lin, gV


def sgd_count(indptr, indices, cnt: torch.Tensor, clear: bool = False, nnz_hint: int = 0):
    """Rows per feature of an SGD batch: cnt[i] += 1 for every entry of the rows of ``indptr``
    (absolute offsets into ``indices``), or cnt[i] = 0 for them (``clear``). GPU: one kernel
    over the device row pointers (no host read); CPU: index ops."""
    n = int(indptr.shape[0] - 1)
    if cnt.is_cuda:
        check_cuda(indptr, indices, cnt)
        hip().sgd_count(ptr(indptr), ptr(indices), n, int(nnz_hint), ptr(cnt), 1 if clear else 0, stream(cnt))
        return cnt
    idx = indices[int(indptr[0]):int(indptr[-1])].long()
    if clear:
        cnt[idx] = 0
    else:
        cnt.index_add_(0, idx, torch.ones_like(idx, dtype=cnt.dtype))
    return cnt


def fm_sgd_update(indptr, indices, values, w_lin, V, S, c, lr: float, l2w: float, l2v: float,
                  reg_skip: int = -1, upd_w: bool = True, bias_latent: bool = False, Vb=None, cnt=None):
    """One Hogwild!-style SGD step over the rows of ``indptr`` (absolute offsets into
    ``indices`` / ``values``): w_i -= lr (c_r x_i + l2w w_i), V_if -= lr (c_r x_i (S_rf - V_if x_i)
    + l2v V_if) for every entry of every row. ``V`` [F, k] / ``S`` [n, k] are None for the
    linear model. ``reg_skip``: the bias index (no regularisation; latent row frozen unless
    ``bias_latent``); ``upd_w = False`` updates only the bias among the linear weights.
    GPU: lock-free float atomics, concurrent rows race as in Hogwild!. CPU: the same
    per-sample gradients applied as one synchronous mini-batch step.
    ``Vb`` (bf16 [F, k], optional): working copy the forward read (S); the gradient's V terms
    use the fp32 master ``V``, and ``Vb`` is re-rounded from it after the step.
    ``cnt`` (int32 [F], optional, :func:`sgd_count`): every weight's step is divided by the
    batch's rows containing its feature (per-feature mean of the per-sample gradients)."""
    n = int(indptr.shape[0] - 1)
    k = 0 if V is None else int(V.shape[1])
    c = c.float().contiguous()
    if w_lin.is_cuda:
        check_cuda(indptr, indices, values, w_lin, V, S, c, Vb, cnt)
        assert Vb is None or (Vb.dtype == torch.bfloat16 and Vb.shape == V.shape and Vb.is_contiguous())
        hip().fm_sgd_update(ptr(indptr), ptr(indices), ptr(values), n, ptr(w_lin), ptr(V), k, ptr(S), ptr(c),
                            float(lr), float(l2w), float(l2v), int(reg_skip), 1 if upd_w else 0,
                            1 if bias_latent else 0, ptr(Vb), ptr(cnt) if cnt is not None else 0, stream(w_lin))
        return
    # bf16 path: S came from the forward over the working copy; the V terms of the gradient
    # use the fp32 master (as sgd_apply_kernel), and the copy is re-rounded after the step
    V_use = V
    b0, e0 = int(indptr[0]), int(indptr[-1])
    rows = torch.repeat_interleave(torch.arange(n), (indptr[1:] - indptr[:-1]).long())
    idx = indices[b0:e0].long()
    x = values[b0:e0]
    cr = c[rows]
    is_bias = idx == reg_skip
    zero = torch.zeros((), dtype=torch.float32)
    gw = cr * x + torch.where(is_bias, zero, l2w * w_lin[idx])
    if not upd_w:
        gw = torch.where(is_bias, gw, zero)
    lri = lr / cnt[idx].clamp(min=1).float() if cnt is not None else torch.full_like(x, lr)
    if k > 0:
        v = V_use[idx]
        gv = (cr * x)[:, None] * (S[rows] - v * x[:, None]) + torch.where(is_bias[:, None], zero, l2v * v)
        if not bias_latent:
            gv[is_bias] = 0.0
        V.index_add_(0, idx, -lri[:, None] * gv)
        if Vb is not None:
            Vb.copy_(V)
    w_lin.index_add_(0, idx, -lri * gw)
