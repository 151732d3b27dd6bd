"""FFM pair interactions: device kernel (``csrc/hip/ffm.hip``) + torch CPU reference.

fx[r] = sum_{p<q in row r} <V[i_p, f_q], V[i_q, f_p]> x_p x_q        (forward)
gV[i_p, f_q] += c_r x_p x_q V[i_q, f_p];  gV[i_q, f_p] += c_r x_p x_q V[i_p, f_q]   (backward)
Reference: ``J/optimizer/FFMHoagOptimizer.java:90-210``.
"""
from __future__ import annotations

import os

import torch

from ._ext import check_cuda, hip, ptr, stream
from .sparse import chunk_reduce, heavy_columns


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


LDS_FWD = os.environ.get("YTK_FFM_LDS", "1") != "0"  # ffm_pairs_lds_kernel where it applies
# ... and over a whole data set (the L-BFGS forward, 4M Criteo-shape rows): off by default,
# the gather kernel measured faster there (22.9 vs 25.5 ms: every latent row misses to HBM and
# LDS capacity caps the rows in flight at ~6 per CU), while SGD batches gain (0.70 vs 1.05 ms
# per 65536-row pair-term forward; profiles/r5/ffm_lds/)
LDS_FWD_FULL = os.environ.get("YTK_FFM_LDS_FULL", "0") == "1"


def lds_forward_ok(max_m: int, nfield: int, k: int, V) -> bool:
    """The LDS-staged forward applies: k == 4, V 16-B aligned, rows of <= 64 entries whose
    latent rows (max_m x (nfield + 1) x 16 B, padded) fit 64 KiB of LDS."""
    return (LDS_FWD and k == 4 and V.is_cuda and V.data_ptr() % 16 == 0 and 1 <= max_m <= 64
            and max_m * (nfield + 1) * 16 <= 64 * 1024)


def ffm_forward(indptr, idx, val, fld, V, nfield: int, k: int, out=None, cache=None, skip_feat: int = -1,
                max_m: int = 0):
    """Pair-interaction sum per row (float32 [n]). CPU: ``cache`` = :func:`ffm_pairs_cpu` output.
    ``max_m`` (GPU, optional): the longest row's entries -- enables the LDS-staged kernel."""
    n = indptr.shape[0] - 1
    if out is None:
        out = torch.zeros(n, dtype=torch.float32, device=V.device)
    if V.is_cuda and max_m and lds_forward_ok(max_m, nfield, k, V):
        check_cuda(indptr, idx, val, fld, V, out)
        hip().ffm_pairs_lds(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, ptr(out), int(skip_feat),
                            int(max_m), 0, 0, 0, stream(V))
        return out
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, out)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, ptr(out), 0, 0, 0,
                        int(skip_feat), stream(V), 0)
        return out
    r, p, q = cache if cache is not None else ffm_pairs_cpu(indptr, idx, val, skip_feat)
    V3 = V.view(-1, nfield, k)
    ip, iq = idx[p].long(), idx[q].long()
    fp, fq = fld[p].long(), fld[q].long()
    dots = (V3[ip, fq] * V3[iq, fp]).sum(1) * val[p] * val[q]
    out.zero_()
    out.index_add_(0, r, dots)
    return out


def ffm_backward(indptr, idx, val, fld, V, nfield: int, k: int, coef, gV, cache=None, skip_feat: int = -1,
                 cnt=None):
    """gV += pair gradients (gV, V: [F * nfield * k] flat). ``cnt`` (int32 [F], optional: the
    SGD batch's rows per feature): the steps into V[i] are divided by cnt[i]."""
    n = indptr.shape[0] - 1
    if V.is_cuda:
        check_cuda(indptr, idx, val, fld, V, coef, gV)
        if cnt is not None:
            check_cuda(cnt)
        hip().ffm_pairs(ptr(indptr), ptr(idx), ptr(val), ptr(fld), n, ptr(V), nfield, k, 0, ptr(coef), ptr(gV), 1,
                        int(skip_feat), stream(V), ptr(cnt) if cnt is not None else 0)
        return gV
    r, p, q = cache if cache is not None else ffm_pairs_cpu(indptr, idx, val, skip_feat)
    V3 = V.view(-1, nfield, k)
    G3 = gV.view(-1, nfield, k)
    ip, iq = idx[p].long(), idx[q].long()
    fp, fq = fld[p].long(), fld[q].long()
    s = (coef[r] * val[p] * val[q])[:, None]
    flat = lambda i, f: i * nfield + f
    G2 = G3.view(-1, k)
    sp = sq = s
    if cnt is not None:
        sp = s / cnt[ip].clamp(min=1).to(s.dtype)[:, None]
        sq = s / cnt[iq].clamp(min=1).to(s.dtype)[:, None]
    G2.index_add_(0, flat(ip, fq), sp * V3[iq, fp])
    G2.index_add_(0, flat(iq, fp), sq * V3[ip, fq])
    return gV


WAVE_NNZ = int(os.environ.get("YTK_FFM_WAVE_NNZ", 512))  # entries per wave of the streamed kernel
STREAM_GB = float(os.environ.get("YTK_FFM_STREAM_GB", 96))  # cap on the streamed expansion's memory


def _fixed_layout(X, fld, nfield: int):
    """(lay_field int32 [m], m) when every row holds the same m == nfield fields in the same
    order (one entry per field, e.g. Criteo rows with the bias in front), else None."""
    n = X.n
    if n == 0 or X.nnz % n:
        return None
    m = X.nnz // n
    if m != nfield or m < 8 or m > 512:
        return None
    if not bool(torch.equal(X.indptr, torch.arange(n + 1, device=X.indptr.device, dtype=X.indptr.dtype) * m)):
        return None
    lay = fld[:m].to(torch.int32).contiguous()
    if not bool(torch.equal(torch.sort(lay).values.long(), torch.arange(m, device=lay.device))):
        return None
    if not bool((fld.view(n, m) == lay[None, :]).all()):
        return None
    return lay, m


def _column_chunks(X, chunk: int):
    """An untiled column order of X's entries for the streamed kernel: (perm, rows, chunk_beg,
    chunk_end, chunk_ptr). X's own CSC is row-tiled so that the per-row data its kernels gather
    stays cache resident; the streamed kernel reads no row data, and the tiles would only
    multiply its chunks (one per (tile, column): 8M instead of 1M on the Criteo shape), each
    paying an accumulator reduction and a partial-block write."""
    cols = X.indices.to(torch.int64)
    perm = torch.sort(cols, stable=True).indices      # CSR order is row-major: rows stay ascending
    scol = cols[perm]
    del cols
    colptr = torch.searchsorted(scol, torch.arange(X.ncols + 1, dtype=torch.int64, device=scol.device))
    del scol
    counts = colptr[1:] - colptr[:-1]
    nch = (counts + chunk - 1) // chunk
    cptr = torch.zeros(X.ncols + 1, dtype=torch.int64, device=counts.device)
    cptr[1:] = torch.cumsum(nch, 0)
    total = int(cptr[-1])
    chunk_col = torch.repeat_interleave(torch.arange(X.ncols, device=counts.device), nch)
    within = torch.arange(total, device=counts.device) - cptr[:-1][chunk_col]
    beg = (colptr[:-1][chunk_col] + within * chunk).contiguous()
    end = torch.minimum(beg + chunk, colptr[1:][chunk_col]).contiguous()
    rows = X.rows_of_nnz[perm].to(torch.int32).contiguous()
    return perm, rows, beg, end, cptr


def _wave_chunks(beg, end, target: int):
    """Chunk ranges of ~``target`` entries per wave (chunks are never split)."""
    nnz = (end - beg).to(torch.int64)
    start = torch.cumsum(nnz, 0) - nnz
    wid = start // max(1, target)
    _, counts = torch.unique_consecutive(wid, return_counts=True)
    wc = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=nnz.device)
    wc[1:] = torch.cumsum(counts, 0)
    return wc


def _stream_layout(X, fld, nfield: int, skip_feat: int, unit_values: bool):
    """Setup of the streamed XCD-split backward (``ffm_grad_stream_kernel``), cached on X:
    fixed-layout rows whose columns each sit in one position only. The expansion
    ``exp_idx[g][e][0..G)`` holds, for CSC entry e, its row's feature ids at position group
    g's positions (-1 for the entry itself and for ``skip_feat``); ``exp_val`` the matching
    values (None for unit values). None when the layout does not qualify or the expansion
    would not fit (``YTK_FFM_STREAM_GB``, free device memory)."""
    key = (fld.data_ptr(), int(nfield), int(skip_feat))
    cached = getattr(X, "_ffm_stream", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    X._ffm_stream = (key, None)
    if os.environ.get("YTK_FFM_STREAM", "1") == "0" or X.n_chunks == 0:
        return None
    fl = _fixed_layout(X, fld, nfield)
    if fl is None:
        return None
    lay_field, m = fl
    G = (m + 7) // 8
    nnz, n = X.nnz, X.n
    need = 8 * nnz * G * 4 * (1 if unit_values else 2)
    free = torch.cuda.mem_get_info(X.indices.device)[0]
    if need > STREAM_GB * 2 ** 30 or need * 1.25 + 2 * 2 ** 30 > free:
        return None
    dev = X.indices.device
    from . import sparse as sparse_mod
    perm, rows32, cbeg, cend, cptr = _column_chunks(X, sparse_mod.CHUNK)
    rows = rows32.to(torch.int64)
    pa = perm - rows * m                             # position of each column-ordered entry in its row
    cols = X.indices[perm].to(torch.int64)
    colpos = torch.full((X.ncols,), -1, dtype=torch.int64, device=dev)
    colpos[cols] = pa
    if not bool((colpos[cols] == pa).all()):      # a column in several positions
        return None
    del cols
    chunk_fa = lay_field[pa[cbeg]].to(torch.int32)
    if skip_feat >= 0:
        chunk_fa = torch.where(X.indices[perm[cbeg]] == skip_feat, torch.full_like(chunk_fa, -1), chunk_fa)
    idx2 = X.indices.view(n, m)
    val2 = None if unit_values else X.values.view(n, m)
    exp_idx = torch.empty((8, nnz, G), dtype=torch.int32, device=dev)
    exp_val = None if unit_values else torch.empty((8, nnz, G), dtype=torch.float32, device=dev)
    step = 1 << 23
    for b0 in range(0, nnz, step):
        b1 = min(nnz, b0 + step)
        r = rows[b0:b1]
        blk = torch.full((b1 - b0, 8 * G), -1, dtype=torch.int32, device=dev)
        blk[:, :m] = idx2[r]
        blk[torch.arange(b1 - b0, device=dev), pa[b0:b1]] = -1
        if skip_feat >= 0:
            blk[blk == skip_feat] = -1
        exp_idx[:, b0:b1, :] = blk.view(b1 - b0, 8, G).permute(1, 0, 2)
        if val2 is not None:
            bv = torch.zeros((b1 - b0, 8 * G), dtype=torch.float32, device=dev)
            bv[:, :m] = val2[r]
            exp_val[:, b0:b1, :] = bv.view(b1 - b0, 8, G).permute(1, 0, 2)
        del blk
    del rows, pa
    st = dict(lay_field=lay_field, m=m, wc=_wave_chunks(cbeg, cend, WAVE_NNZ), chunk_fa=chunk_fa.contiguous(),
              exp_idx=exp_idx, exp_val=exp_val, rows=rows32, vals=None if unit_values else X.values[perm].contiguous(),
              beg=cbeg, end=cend, cptr=cptr)
    X._ffm_stream = (key, st)
    return st


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
    lay = (distinct, code, sh, vals)
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
    distinct, code, sh, vals = lay
    J = nfield * k
    check_cuda(fld, V, coef, gV)
    Vt = V.view(X.ncols, nfield, k).transpose(0, 1).contiguous()  # [nfield][F][k]
    h, s = hip(), stream(V)
    st = _stream_layout(X, fld, nfield, skip_feat, vals is None) if k in (4, 8, 16) else None
    if st is not None:
        # fixed-layout rows: the streamed XCD-split kernel (each XCD gathers only its own
        # fields' latent rows -- an L2-sized working set -- and streams the row entries)
        se = coef.index_select(0, st["rows"])
        if st["vals"] is not None:
            se.mul_(st["vals"])
        wc, nch = st["wc"], st["beg"].numel()
        part = torch.empty((max(nch, 1), J), dtype=torch.float32, device=V.device)
        h.ffm_grad_stream(ptr(wc), wc.numel() - 1, ptr(st["beg"]), ptr(st["end"]), ptr(st["chunk_fa"]),
                          ptr(st["exp_idx"]), ptr(st["exp_val"]), ptr(se), X.nnz, ptr(st["lay_field"]), st["m"],
                          ptr(Vt), X.ncols, nfield, k, ptr(part), s)
        if "heavy" not in st:
            st["heavy"] = heavy_columns(st["cptr"])
        chunk_reduce(st["cptr"], X.ncols, part, J, gV, J, 1.0, 1, 0, s, st["heavy"])
        return gV
    part = torch.empty((max(X.n_chunks, 1), J), dtype=torch.float32, device=V.device)
    # general rows: one wave per chunk, the row entries read per column (L2-miss bound on its
    # random 16-B latent gathers: 274 GB fetched per Criteo-shape pass vs 46 GB for the
    # row-oriented forward, which reuses a row's latent blocks across its pairs)
    h.ffm_grad_csc(ptr(X.chunk_bounds), ptr(X.chunk_end_b), X.n_chunks, ptr(X.csc_rows), ptr(X.csc_vals),
                   ptr(X.csc_perm), ptr(X.indptr), ptr(code), sh, ptr(vals) if vals is not None else 0,
                   ptr(Vt), X.ncols, nfield, k, ptr(coef), ptr(part), int(skip_feat), int(distinct), s)
    chunk_reduce(X.chunk_ptr, X.ncols, part, J, gV, J, 1.0, 1, ptr(X.chunk_ids), s, X.heavy_cols)
    return gV
