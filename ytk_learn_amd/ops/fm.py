"""Fused factorization-machine loss/gradient passes (``csrc/hip/fm.hip``) + torch CPU path.

forward:  fx = X w + 1/2 sum_f [(X V)^2 - (X∘X)(V∘V)]_f ,  S = X V
backward: g_w = X^T c,  g_V = X^T (c∘S) - V ∘ ((X∘X)^T c)
Reference: ``J/optimizer/FMHoagOptimizer.java:60-160``.
"""
from __future__ import annotations

import torch

from ._ext import check_cuda, hip, ptr, stream


def fm_forward(X, w_lin: torch.Tensor, V: torch.Tensor):
    """(fx float64 [n], S float32 [n, k]) for the rows of SparseMatrix X; V: [F, k] view."""
    k = V.shape[1]
    if X.device.type == "cuda" and 1 <= k <= 64:
        check_cuda(w_lin, V)
        V = V.contiguous()
        fx = torch.empty(X.n, dtype=torch.float64, device=X.device)
        S = torch.empty((X.n, k), dtype=torch.float32, device=X.device)
        hip().fm_forward(ptr(X.indptr), ptr(X.indices), ptr(X.values), X.n, ptr(w_lin), ptr(V), k, ptr(fx), ptr(S),
                         stream(V))
        return fx, S
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
        h.fm_backward(ptr(X.chunk_beg), ptr(X.chunk_end), X.n_chunks, ptr(X.csc_rows), ptr(X.csc_vals), ptr(c),
                      ptr(S.contiguous()), k, ptr(part), s)
        h.chunk_reduce(ptr(X.chunk_ptr), X.ncols, ptr(part), k + 2, ptr(tot), k + 2, 1.0, 0, s)
        g_lin.copy_(tot[:, k])
        gV.copy_(tot[:, :k])
        gV.addcmul_(V, tot[:, k + 1:k + 2], value=-1.0)
        return g_lin, gV
    X.t_matmul(c, out=g_lin)
    X.t_matmul((c[:, None] * S).contiguous(), out=gV)
    sq = X.t_matmul(c, square=True)
    gV.sub_(V * sq[:, None])
    return g_lin, gV
