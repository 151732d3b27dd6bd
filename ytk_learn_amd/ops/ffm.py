"""FFM pair interactions: device kernel (``csrc/hip/ffm.hip``) + torch CPU reference.

fx[r] = sum_{p<q in row r} <V[i_p, f_q], V[i_q, f_p]> x_p x_q        (forward)
gV[i_p, f_q] += c_r x_p x_q V[i_q, f_p];  gV[i_q, f_p] += c_r x_p x_q V[i_p, f_q]   (backward)
Reference: ``J/optimizer/FFMHoagOptimizer.java:90-210``.
"""
from __future__ import annotations

import os

import torch

from . import sparse as sparse_mod
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


def ffm_pairs_cpu(indptr, idx, val, skip_feat: int = -1):
    """CPU pair list without the pairs that contribute nothing: a zero value on either side
    (dense-style rows such as agaricus carry many explicit ``name:0`` entries) or the
    ``skip_feat`` feature (all-zero latent block). Cache it per dataset and pass as ``cache``."""
    r, p, q = _pairs_cpu(indptr)
    keep = (val[p] != 0) & (val[q] != 0)
    if skip_feat >= 0:
        keep &= (idx[p] != skip_feat) & (idx[q] != skip_feat)
    return r[keep], p[keep], q[keep]


def ffm_forward(indptr, idx, val, fld, V, nfield: int, k: int, out=None, cache=None, skip_feat: int = -1):
    """Pair-interaction sum per row (float32 [n]). CPU: ``cache`` = :func:`ffm_pairs_cpu` output."""
    n = indptr.shape[0] - 1
    if out is None:
        out = torch.zeros(n, dtype=torch.float32, device=V.device)
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, out)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, ptr(out), 0, 0, 0,
                        int(skip_feat), stream(V))
        return out
    r, p, q = cache if cache is not None else ffm_pairs_cpu(indptr, idx, val, skip_feat)
    V3 = V.view(-1, nfield, k)
    ip, iq = idx[p].long(), idx[q].long()
    fp, fq = fld[p].long(), fld[q].long()
    dots = (V3[ip, fq] * V3[iq, fp]).sum(1) * val[p] * val[q]
    out.zero_()
    out.index_add_(0, r, dots)
    return out


def ffm_backward(indptr, idx, val, fld, V, nfield: int, k: int, coef, gV, cache=None, skip_feat: int = -1):
    """gV += pair gradients (gV, V: [F * nfield * k] flat)."""
    n = indptr.shape[0] - 1
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, coef, gV)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, 0, ptr(coef), ptr(gV), 1,
                        int(skip_feat), stream(V))
        return gV
    r, p, q = cache if cache is not None else ffm_pairs_cpu(indptr, idx, val, skip_feat)
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


def _csc_layout(X, fld, nfield: int):
    """Per-dataset inputs of the column-ordered backward, cached on X: whether rows have
    distinct fields (then the LDS accumulator needs no atomics), the packed entry codes
    ``feature | field << sh`` (one 4-B load per entry instead of two) and the values (None
    when all are 1, e.g. one-hot data). Returns None when the codes do not fit 32 bits."""
    key = (fld.data_ptr(), int(nfield))
    cached = getattr(X, "_ffm_layout", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    sh = max(1, int(X.ncols - 1).bit_length())
    if sh + max(1, int(nfield - 1).bit_length()) > 32:
        X._ffm_layout = (key, None)
        return None
    f64 = fld.to(torch.int64)
    ks = torch.sort(X.rows_of_nnz.to(torch.int64) * nfield + f64).values
    distinct = bool(ks.numel() < 2 or not bool((ks[1:] == ks[:-1]).any()))
    del ks
    code = X.indices.to(torch.int64) | (f64 << sh)
    code = torch.where(code >= 2 ** 31, code - 2 ** 32, code).to(torch.int32).contiguous()  # uint32 bits
    vals = None if bool((X.values == 1).all()) else X.values
    # chunk processing order: (row tile, field of the chunk's column), stable -- the gathers
    # of concurrently running chunks then stay inside one field's latent slice
    # (YTK_FFM_FIELD_ORDER=0: CSC order)
    order = None
    if X._csc is None:
        X._build_csc()
    if os.environ.get("YTK_FFM_FIELD_ORDER", "1") != "0" and X.n_chunks > 0:
        e0 = X.csc_perm[X.chunk_beg]                                 # first entry of each chunk (CSR pos)
        tile = X.rows_of_nnz[e0].to(torch.int64) // max(1, sparse_mod.ROW_TILE if X.n > sparse_mod.ROW_TILE else X.n + 1)
        key = tile * nfield + f64[e0]
        order = torch.sort(key, stable=True).indices.to(torch.int32).contiguous()
    lay = (distinct, code, sh, vals, order)
    X._ffm_layout = (key, lay)
    return lay


def ffm_backward_csc(X, fld, V, nfield: int, k: int, coef, gV, skip_feat: int = -1, cache=None):
    """gV += pair gradients, column-ordered (no global atomics; deterministic for rows with
    distinct fields). ``X`` is the :class:`~ytk_learn_amd.ops.sparse.SparseMatrix` of the same
    rows (its CSC chunks define the work split). Falls back to :func:`ffm_backward` on CPU."""
    lay = _csc_layout(X, fld, nfield) if V.is_cuda and nfield * k <= 2048 else None
    if lay is None:
        return ffm_backward(X.indptr, X.indices, X.values, fld, V, nfield, k, coef, gV, cache=cache,
                            skip_feat=skip_feat)
    if X._csc is None:
        X._build_csc()
    distinct, code, sh, vals, order = lay
    J = nfield * k
    check_cuda(fld, V, coef, gV)
    Vt = V.view(X.ncols, nfield, k).transpose(0, 1).contiguous()  # [nfield][F][k]
    part = torch.empty((max(X.n_chunks, 1), J), dtype=torch.float32, device=V.device)
    h, s = hip(), stream(V)
    # (a register-accumulating variant for rows with a fixed field layout measured the same
    # 75 ms on the Criteo shape: this kernel is bound by the L2 misses of its random 16-B
    # latent-row gathers -- 274 GB fetched vs 46 GB for the row-oriented forward, which
    # reuses a row's latent blocks across its pairs -- not by the LDS accumulator)
    h.ffm_grad_csc(ptr(X.chunk_beg), ptr(X.chunk_end), X.n_chunks, ptr(X.csc_rows), ptr(X.csc_vals),
                   ptr(X.csc_perm), ptr(X.indptr), ptr(code), sh, ptr(vals) if vals is not None else 0, ptr(Vt),
                   X.ncols, nfield, k, ptr(coef), ptr(part), int(skip_feat), int(distinct), ptr(order), s)
    h.chunk_reduce(ptr(X.chunk_ptr), X.ncols, ptr(part), J, ptr(gV), J, 1.0, 1, ptr(X.chunk_ids), s)
    return gV
