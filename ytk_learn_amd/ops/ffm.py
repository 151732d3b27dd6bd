"""FFM pair interactions: device kernel (``csrc/hip/ffm.hip``) + torch CPU reference.

fx[r] = sum_{p<q in row r} <V[i_p, f_q], V[i_q, f_p]> x_p x_q        (forward)
gV[i_p, f_q] += c_r x_p x_q V[i_q, f_p];  gV[i_q, f_p] += c_r x_p x_q V[i_p, f_q]   (backward)
Reference: ``J/optimizer/FFMHoagOptimizer.java:90-210``.
"""
from __future__ import annotations

import torch

from ._ext import check_cuda, hip, ptr, stream


def _pairs_cpu(indptr: torch.Tensor):
    """(row, p_pos, q_pos) for every p<q pair, grouped by row length (vectorised)."""
    lens = (indptr[1:] - indptr[:-1]).long()
    rows_all, ps, qs = [], [], []
    for m in torch.unique(lens).tolist():
        if m < 2:
            continue
        rows = torch.nonzero(lens == m).flatten()
        tp, tq = torch.triu_indices(m, m, offset=1)
        base = indptr[:-1][rows].long()
        rows_all.append(rows.repeat_interleave(tp.numel()))
        ps.append((base[:, None] + tp[None, :]).reshape(-1))
        qs.append((base[:, None] + tq[None, :]).reshape(-1))
    if not rows_all:
        z = torch.zeros(0, dtype=torch.long)
        return z, z, z
    return torch.cat(rows_all), torch.cat(ps), torch.cat(qs)


def ffm_forward(indptr, idx, val, fld, V, nfield: int, k: int, out=None, cache=None):
    """Pair-interaction sum per row (float32 [n])."""
    n = indptr.shape[0] - 1
    if out is None:
        out = torch.zeros(n, dtype=torch.float32, device=V.device)
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, out)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, ptr(out), 0, 0, 0,
                        stream(V))
        return out
    r, p, q = cache if cache is not None else _pairs_cpu(indptr)
    V3 = V.view(-1, nfield, k)
    ip, iq = idx[p].long(), idx[q].long()
    fp, fq = fld[p].long(), fld[q].long()
    dots = (V3[ip, fq] * V3[iq, fp]).sum(1) * val[p] * val[q]
    out.zero_()
    out.index_add_(0, r, dots)
    return out


def ffm_backward(indptr, idx, val, fld, V, nfield: int, k: int, coef, gV, cache=None):
    """gV += pair gradients (gV, V: [F * nfield * k] flat)."""
    n = indptr.shape[0] - 1
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, coef, gV)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, 0, ptr(coef), ptr(gV), 1,
                        stream(V))
        return gV
    r, p, q = cache if cache is not None else _pairs_cpu(indptr)
    V3 = V.view(-1, nfield, k)
    G3 = gV.view(-1, nfield, k)
    ip, iq = idx[p].long(), idx[q].long()
    fp, fq = fld[p].long(), fld[q].long()
    s = (coef[r] * val[p] * val[q])[:, None]
    flat = lambda i, f: i * nfield + f
    G2 = G3.view(-1, k)
    G2.index_add_(0, flat(ip, fq), s * V3[iq, fp])
    G2.index_add_(0, flat(iq, fp), s * V3[ip, fq])
    return gV
