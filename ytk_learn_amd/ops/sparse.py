"""Device sparse matrix for the L-BFGS model family (linear, multiclass, FM, GBMLR...).

Holds CSR (rows) and CSC (columns, split into fixed-size chunks) of the same matrix so
that both ``X @ W`` and ``X^T @ D`` run as the deterministic segmented kernel of
``csrc/hip/sparse.hip`` (no float atomics). On CPU the same products use torch
index ops (reference path for tests).

Reference hot loops: ``J/optimizer/LinearHoagOptimizer.java:76-106`` (Xv / XTv) and the
per-model loops listed in SURVEY.md §2.A K16-K21.
"""
from __future__ import annotations

import os

from typing import Optional

import torch

from ._ext import check_cuda, hip, ptr, stream

CHUNK = 4096  # nnz per CSC chunk: balances the bias column (all rows) against short columns
# rows per CSC row tile (GPU, see SparseMatrix._build_csc); 0 disables the tiling
ROW_TILE = int(os.environ.get("YTK_CSC_ROW_TILE", 524288))
TILE_ON = os.environ.get("YTK_SPMV_TILE", "1") != "0"
TILE_ROWS = os.environ.get("YTK_SPMV_TILE_ROWS", "0") == "1"
FIXED_ON = os.environ.get("YTK_SPMV_FIXED", "1") != "0"
FIX_SPAN = 32768      # == kFixSpan (sparse.hip): columns per position slice staged in LDS
FIX_MIN_ROWS = 1 << 18  # below this the per-row kernel is as fast (one block per 16384 rows)


TILE_CAP = 4096   # == kTileCap (sparse.hip): entries per pass of the tiled SpMV
TILE_SEGS = 256   # == kTileSegs: segments per tiled-SpMV block at most
REDUCE_LIGHT = 16  # == kReduceLight: columns with more chunks are reduced one block each


def tile_blocks(beg: torch.Tensor, end: torch.Tensor) -> Optional[torch.Tensor]:
    """Block table of the entry-tiled SpMV (seg_tile_spmv_kernel) for segments that tile their
    entries contiguously: block b covers segments [bseg[b], bseg[b + 1]) -- at most TILE_SEGS
    of them, all starting inside one (TILE_CAP - 256)-entry window, so a block is one pass of
    the kernel unless its last segment is longer than 256 entries. None when the segments
    are not contiguous (the per-segment kernel is used then)."""
    n = int(beg.numel())
    if n == 0 or not bool((end[:-1] == beg[1:]).all()):
        return None
    ar = torch.arange(n, device=beg.device, dtype=torch.int64)
    key = (beg - beg[0]) // (TILE_CAP - 256) + ar // TILE_SEGS  # nondecreasing: equal keys are runs
    change = torch.nonzero(key[1:] != key[:-1]).flatten() + 1
    return torch.cat([torch.zeros(1, dtype=torch.int64, device=beg.device), change,
                      torch.full((1,), n, dtype=torch.int64, device=beg.device)]).to(torch.int32).contiguous()


def heavy_columns(cptr: torch.Tensor) -> torch.Tensor:
    """Columns with more than REDUCE_LIGHT chunks (int32): chunk_reduce gives each a block."""
    return torch.nonzero((cptr[1:] - cptr[:-1]) > REDUCE_LIGHT).flatten().to(torch.int32).contiguous()


def chunk_reduce(cptr, ncol, part, J, out, ldo, alpha, accumulate, ids, s, heavy=None):
    """out[col, :] (+)= alpha * the column's chunk partials summed in chunk order; ``heavy``
    (heavy_columns(cptr)) routes the long columns to one block each."""
    hv = heavy if heavy is not None else heavy_columns(cptr)
    hip().chunk_reduce(ptr(cptr), ncol, ptr(part), J, ptr(out), ldo, alpha, accumulate, ids, s,
                       ptr(hv) if hv.numel() else 0, int(hv.numel()))


def _lanes(avg_nnz: float) -> int:
    """Lanes per segment for the J == 1 kernel: each lane takes ~4 entries per pass (its four
    loads are issued together), so L = pow2 >= avg / 4, in [4, 64]."""
    L = 1
    while L * 4 < avg_nnz and L < 64:
        L <<= 1
    return max(L, 4)


class SparseMatrix:
    """Immutable CSR/CSC pair. ``indptr`` int64 [n+1], ``indices`` int32, ``values`` float32."""

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, ncols: int,
                 build_csc: bool = True, row_tile: bool = True, chunk: int = 0):
        self.device = indices.device
        self.row_tile = row_tile  # False: one column order over all rows (SGD batches, ops/sgd.py)
        self.chunk = int(chunk) if chunk > 0 else CHUNK  # entries per CSC chunk
        self.n = int(indptr.shape[0] - 1)
        self.ncols = int(ncols)
        self.indptr = indptr.to(torch.int64).contiguous()
        self.indices = indices.to(torch.int32).contiguous()
        self.values = values.to(torch.float32).contiguous()
        self.nnz = int(self.indices.shape[0])
        self.row_beg = self.indptr[:-1].contiguous()
        self.row_end = self.indptr[1:].contiguous()
        self.row_lanes = _lanes(self.nnz / max(self.n, 1))
        # one-hot matrix (e.g. Criteo categorical fields): the products skip the value loads
        self.one_hot = bool(self.nnz > 0 and bool((self.values == 1.0).all()))
        self.rows_of_nnz = torch.repeat_interleave(torch.arange(self.n, device=self.device),
                                                   self.indptr[1:] - self.indptr[:-1])
        # entry-tiled SpMV over the rows: measured slower than the per-row lane groups for
        # Criteo-shaped rows (918 vs 846 us per 164M-entry product: both bound by the random
        # x gathers, tools/microbench/spmv_gather.py), so rows keep seg_spmv_kernel
        # (YTK_SPMV_TILE_ROWS=1: tiled rows too)
        self.row_tiles = (tile_blocks(self.row_beg, self.row_end)
                          if self.device.type == "cuda" and TILE_ON and TILE_ROWS else None)
        self._csc = None
        self._fixed = None  # fixed-layout row product tables (lazy, see _fixed_layout)
        if build_csc:
            self._build_csc()

    def _fixed_layout(self):
        """Tables of fixed_spmv_kernel when every row holds the same number m of entries and
        position j's columns span at most FIX_SPAN (the Criteo shape: bias + one entry per
        field): uint16 position-major local offsets idxT[j][r] = idx[r][j] - lo[j], the values
        likewise (None when one-hot), lo / span per position. False when the layout does not
        qualify (the per-row kernels run then). Built once, on the first product."""
        if self._fixed is not None:
            return self._fixed
        self._fixed = False
        n, nnz = self.n, self.nnz
        if not (FIXED_ON and self.device.type == "cuda" and n >= FIX_MIN_ROWS and nnz % n == 0):
            return False
        m = nnz // n
        if not (1 <= m <= 1024):
            return False
        if not bool(torch.equal(self.indptr, torch.arange(n + 1, device=self.device, dtype=torch.int64) * m)):
            return False
        ix = self.indices.view(n, m)
        lo = ix.amin(0)
        span = ix.amax(0) - lo + 1
        if int(span.max()) > FIX_SPAN:
            return False
        idxT = (ix - lo[None, :]).t().contiguous().to(torch.int32).to(torch.uint16)
        valT = None if self.one_hot else self.values.view(n, m).t().contiguous()
        self._fixed = {"m": m, "idxT": idxT, "valT": valT, "lo": lo.to(torch.int32).contiguous(),
                       "span": span.to(torch.int32).contiguous(), "max_span": int(span.max())}
        return self._fixed

    def _build_csc(self):
        """Column-ordered (CSC) copy in CHUNK-entry chunks for the transposed products.

        On the GPU with more than ROW_TILE rows the entries are ordered (row tile, column,
        row): the chunks of one row tile run together, so the per-row data the column
        kernels gather (FM's S rows, FFM's row entries, the row coefficients) is a
        tile-sized, cache-resident working set (MALL / L2) instead of the whole matrix.
        A column's chunks then come from several tiles; ``chunk_ids`` lists them column
        by column for the ordered chunk reduce (deterministic sum order)."""
        cols = self.indices.to(torch.int64)
        rows = self.rows_of_nnz.to(torch.int64)
        tiled = self.device.type == "cuda" and ROW_TILE > 0 and self.n > ROW_TILE and self.row_tile
        T = -(-self.n // ROW_TILE) if tiled else 1
        seg = (rows // ROW_TILE) * self.ncols + cols if tiled else cols  # (tile, column) segments
        order = torch.sort(seg * (self.n + 1) + rows, stable=True).indices
        del rows
        self.csc_perm = order
        self.csc_rows = self.rows_of_nnz[order].to(torch.int32).contiguous()
        self.csc_vals = self.values[order].contiguous()
        # segment boundaries from the SORTED segment keys (binary searches; no histogram
        # kernel -- torch's bincount ran 23-50 ms per call on 160M entries)
        seg_sorted = seg[order]
        del seg
        S = T * self.ncols
        segptr = torch.searchsorted(seg_sorted, torch.arange(S + 1, dtype=seg_sorted.dtype, device=self.device))
        del seg_sorted
        scounts = segptr[1:] - segptr[:-1]
        counts = scounts.view(T, self.ncols).sum(0) if tiled else scounts
        colptr = torch.zeros(self.ncols + 1, dtype=torch.int64, device=self.device)
        colptr[1:] = torch.cumsum(counts, 0)
        self.colptr = colptr
        # chunks: segment s is split into ceil(len/CHUNK) pieces (none when empty)
        C = self.chunk
        nch = (scounts + C - 1) // C
        cbeg = torch.zeros(scounts.numel() + 1, dtype=torch.int64, device=self.device)
        cbeg[1:] = torch.cumsum(nch, 0)
        total = int(cbeg[-1])
        chunk_seg = torch.repeat_interleave(torch.arange(scounts.numel(), device=self.device), nch)
        within = torch.arange(total, device=self.device) - cbeg[:-1][chunk_seg]
        self.chunk_beg = (segptr[:-1][chunk_seg] + within * C).contiguous()
        self.chunk_end = torch.minimum(self.chunk_beg + C, segptr[1:][chunk_seg]).contiguous()
        self.chunk_col = chunk_seg % self.ncols  # column of each chunk
        if tiled:
            chunk_col = chunk_seg % self.ncols
            self.chunk_ids = torch.sort(chunk_col, stable=True).indices.contiguous()  # column-major, tiles in order
            per_col = nch.view(T, self.ncols).sum(0)  # chunks per column over the row tiles
            cptr = torch.zeros(self.ncols + 1, dtype=torch.int64, device=self.device)
            cptr[1:] = torch.cumsum(per_col, 0)
            self.chunk_ptr = cptr.contiguous()
        else:
            self.chunk_ids = None
            self.chunk_ptr = cbeg.contiguous()
        self.n_chunks = total
        self.chunk_lanes = _lanes(self.nnz / max(total, 1))
        # power-law columns (Criteo: a few hot features, a long tail of short columns): one
        # lane count for all chunks idles most lanes on the tail, so J == 1 products launch
        # three length buckets (<= 16, <= 64, longer: 4 / 16 / 64 lanes per chunk)
        clen = (self.chunk_end - self.chunk_beg)
        self.chunk_tiles = tile_blocks(self.chunk_beg, self.chunk_end) if TILE_ON else None
        # the chunks tile the entries contiguously (chunk_end[i] == chunk_beg[i + 1] by
        # construction): one bounds array serves as both beg ([:-1]) and end ([1:]), so the
        # kernels' begin / end loads share cache lines (half the bounds traffic of two arrays)
        self.chunk_bounds = torch.cat([self.chunk_beg, self.chunk_end[-1:]]).contiguous()
        self.chunk_end_b = self.chunk_bounds[1:]
        self.heavy_cols = heavy_columns(self.chunk_ptr)
        self.chunk_buckets = []
        for lo, hi, lanes in ((0, 16, 4), (16, 64, 16), (64, 1 << 62, 64)):
            ids = torch.nonzero((clen > lo) & (clen <= hi)).flatten().to(torch.int32).contiguous()
            if lo == 0:  # empty chunks never exist, but keep them in the first bucket if they did
                ids = torch.nonzero(clen <= hi).flatten().to(torch.int32).contiguous()
            if ids.numel():
                self.chunk_buckets.append((lanes, ids))
        self._csc = True

    # ------------------------------------------------------------------ products
    def matmul(self, W: torch.Tensor, out: Optional[torch.Tensor] = None, square: bool = False,
               alpha: float = 1.0, accumulate: bool = False, values: Optional[torch.Tensor] = None) -> torch.Tensor:
        """out[n, J] = alpha * X @ W  (W: [ncols] or [ncols, J]); ``square`` uses X∘X.
        ``values`` overrides the stored values (e.g. FFM/FM variants)."""
        W2 = W.reshape(W.shape[0], -1)
        J = W2.shape[1]
        vals = self.values if values is None else values
        if out is None:
            # the GPU kernels write every output row when not accumulating (no zero fill)
            alloc = torch.empty if self.device.type == "cuda" else torch.zeros
            out = alloc((self.n,) if W.dim() == 1 else (self.n, J), dtype=torch.float32, device=self.device)
            accumulate = False
        o2 = out.reshape(self.n, -1)
        if self.device.type == "cuda":
            check_cuda(W2, o2, vals, rows_ok=(W2, o2))  # the kernels take row strides
            vp = 0 if (values is None and self.one_hot) else ptr(vals)
            fx = self._fixed_layout() if (J == 1 and values is None) else False
            if fx and W2.stride(0) == 1 and o2.stride(0) == 1:
                hip().fixed_spmv(ptr(fx["idxT"]), ptr(fx["valT"]) if fx["valT"] is not None else 0, self.n, fx["m"],
                                 ptr(fx["lo"]), ptr(fx["span"]), fx["max_span"], ptr(W2), ptr(o2), float(alpha),
                                 int(accumulate), int(square), stream(W2))
                return out
            if J == 1 and self.row_tiles is not None and W2.stride(0) == 1 and o2.stride(0) == 1:
                hip().seg_tile_spmv(ptr(self.row_beg), ptr(self.row_end), ptr(self.row_tiles),
                                    self.row_tiles.numel() - 1, ptr(self.indices), vp, ptr(W2), ptr(o2),
                                    float(alpha), int(accumulate), int(square), stream(W2))
                return out
            hip().seg_spmm(ptr(self.row_beg), ptr(self.row_end), self.n, ptr(self.indices), vp, ptr(W2),
                           W2.stride(0), J, ptr(o2), o2.stride(0), float(alpha), int(accumulate), int(square),
                           self.row_lanes if J == 1 else min(64, J), 0, stream(W2))
        else:
            v = vals * vals if square else vals
            prod = W2.index_select(0, self.indices.long()) * v[:, None]
            res = torch.zeros((self.n, J), dtype=torch.float32)
            res.index_add_(0, self.rows_of_nnz, prod)
            if accumulate:
                o2 += alpha * res
            else:
                o2.copy_(alpha * res)
        return out

    def t_matmul(self, D: torch.Tensor, out: Optional[torch.Tensor] = None, square: bool = False,
                 alpha: float = 1.0, accumulate: bool = False, values: Optional[torch.Tensor] = None) -> torch.Tensor:
        """out[ncols, J] = alpha * X^T @ D  (D: [n] or [n, J])."""
        if self._csc is None:
            self._build_csc()
        D2 = D.reshape(self.n, -1)
        J = D2.shape[1]
        if out is None:
            # chunk_reduce writes every column (0 for empty ones) when not accumulating
            alloc = torch.empty if self.device.type == "cuda" else torch.zeros
            out = alloc((self.ncols,) if D.dim() == 1 else (self.ncols, J), dtype=torch.float32, device=self.device)
            accumulate = False
        o2 = out.reshape(self.ncols, -1)
        if self.device.type == "cuda":
            csc_vals = self.csc_vals if values is None else values
            check_cuda(D2, o2, csc_vals, rows_ok=(D2, o2))  # the kernels take row strides
            part = torch.empty((max(self.n_chunks, 1), J), dtype=torch.float32, device=self.device)
            h = hip()
            s = stream(D2)
            vp = 0 if (values is None and self.one_hot) else ptr(csc_vals)
            if J == 1 and self.chunk_tiles is not None and D2.stride(0) == 1:
                h.seg_tile_spmv(ptr(self.chunk_bounds), ptr(self.chunk_bounds[1:]), ptr(self.chunk_tiles),
                                self.chunk_tiles.numel() - 1, ptr(self.csc_rows), vp, ptr(D2), ptr(part), 1.0, 0,
                                int(square), s)
            elif J == 1:  # chunks bucketed by length, each bucket with its own lane count
                for lanes, perm in self.chunk_buckets:
                    h.seg_spmm(ptr(self.chunk_bounds), ptr(self.chunk_end_b), perm.numel(), ptr(self.csc_rows), vp,
                               ptr(D2), D2.stride(0), 1, ptr(part), 1, 1.0, 0, int(square), lanes, ptr(perm), s)
            else:
                h.seg_spmm(ptr(self.chunk_bounds), ptr(self.chunk_end_b), self.n_chunks, ptr(self.csc_rows), vp,
                           ptr(D2), D2.stride(0), J, ptr(part), J, 1.0, 0, int(square), min(64, J), 0, s)
            chunk_reduce(self.chunk_ptr, self.ncols, part, J, o2, o2.stride(0), float(alpha), int(accumulate),
                         ptr(self.chunk_ids), s, self.heavy_cols)
        else:
            vals = self.csc_vals if values is None else values
            v = vals * vals if square else vals
            prod = D2.index_select(0, self.csc_rows.long()) * v[:, None]
            # column-ordered segment sums (deterministic, same chunk order as the GPU path)
            res = torch.zeros((self.ncols, J), dtype=torch.float32)
            cols = torch.repeat_interleave(torch.arange(self.ncols), self.colptr[1:] - self.colptr[:-1])
            res.index_add_(0, cols, prod)
            if accumulate:
                o2 += alpha * res
            else:
                o2.copy_(alpha * res)
        return out

    def csc_values_of(self, nnz_values: torch.Tensor) -> torch.Tensor:
        """Permute a per-nnz CSR-ordered tensor into CSC order (for custom-valued products)."""
        if self._csc is None:
            self._build_csc()
        return nnz_values[self.csc_perm].contiguous()
