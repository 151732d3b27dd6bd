"""GBDT device ops.

Each op takes torch tensors. Tensors on the GPU go to the hand-written HIP
kernels in ``csrc/hip/gbdt_kernels.hip`` (no fallback: a missing extension
raises). CPU tensors use a plain PyTorch/NumPy implementation of the same
semantics; that path is the numerics reference for the kernel tests and the
engine for CPU-only (gloo) runs.

Reference semantics are cited in the kernel file header.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._ext import check_cuda, hip, hist_cols, ptr, stream

SPLIT_DTYPE = np.dtype(
    [("loss_chg", "<f4"), ("feat", "<i4"), ("bin_a", "<i4"), ("bin_b", "<i4"),
     ("gl", "<f8"), ("hl", "<f8"), ("g", "<f8"), ("h", "<f8")]
)
assert SPLIT_DTYPE.itemsize == 48

LOSS_IDS = {"sigmoid": 0, "l2": 1, "l1": 2, "poisson": 3, "huber": 4, "softmax": 5}


def _bin_bytes(bins: torch.Tensor) -> int:
    if bins.dtype == torch.uint8:
        return 1
    if bins.dtype == torch.int16:
        return 2
    raise ValueError(f"bins must be uint8 or int16, got {bins.dtype}")


# ---------------------------------------------------------------------------
# histogram build
# ---------------------------------------------------------------------------
def fixed_point_scales(max_abs_g: float, max_h: float, n_rows: int):
    """Per-tree power-of-two scales so |sum over all rows| < 2^62 (exact int64 sums).

    Returns (sg, sh) as float32-representable powers of two."""
    out = []
    for m in (max_abs_g, max_h):
        m = float(m)
        if not np.isfinite(m):
            raise ValueError("non-finite gradient/hessian")
        if m <= 0.0:
            out.append(1.0)
            continue
        k = int(np.floor(np.log2((2.0 ** 62) / (m * max(1, int(n_rows))))))
        out.append(float(2.0 ** min(max(k, -120), 120)))
    return out[0], out[1]


def quantize_gh(gh: torch.Tensor, sg: float, sh: float) -> torch.Tensor:
    """Reference of the kernels' rounding: __float2ll_rn(x * 2^k) per component."""
    q = torch.empty(gh.shape, dtype=torch.int64, device=gh.device)
    q[..., 0] = torch.round(gh[..., 0].float() * np.float32(sg)).to(torch.int64)
    q[..., 1] = torch.round(gh[..., 1].float() * np.float32(sh)).to(torch.int64)
    return q


WIDE_LDS_BYTES = 160 * 1024  # == kWideLdsBytes in csrc/hip/gbdt_hist.hip


def wide_group(B: int, F: int) -> int:
    """Features per block (a power of two <= 32) of the wide-bin (uint16, B > 256) LDS
    histogram kernel; 0 when
    one feature's B x 16-byte (g, h) planes exceed the LDS budget (mirrors
    ytk_hist_wide_group)."""
    per = B * 16
    if B <= 0 or per > WIDE_LDS_BYTES:
        return 0
    fit = min(32, WIDE_LDS_BYTES // per)
    g = 1
    while 2 * g <= fit:
        g *= 2
    return g


def hist_build(bins, F, ghp, rows, work, hist, B, sg, sh, staging=None, slot_base=0, nslots=0, slot_ids=None,
               binsT=None):
    """Accumulate exact int64 fixed-point (g, h) histograms.

    bins: [N, S] uint8/int16 row-major (S >= F, S % 32 == 0 for the LDS path)
    ghp:  [M, 2] float32 (g, h) in POSITION order (ghp[pos] belongs to rows[pos])
    rows: int32 row permutation or None (identity positions)
    work: int32 [nwork, 4] = (slot, begin, end, 0); positions index ``rows``
    hist: int64 [slots, B, F, 2], target slots must be zeroed by the caller
    sg, sh: power-of-two fixed-point scales (``fixed_point_scales``)
    staging: optional int64 scratch (>= nwork * hist_cols(F) * B * 2 elements): block
      partials are stored, then reduced into the work's slots, which must be the
      contiguous range [slot_base, slot_base + nslots) (two-stage flush, no per-block
      global atomics -- see csrc/hip/gbdt_hist.hip); ``slot_ids`` (int32 device tensor of
      nslots ids) replaces the contiguous range when given
    binsT: optional column-major [F, N] copy of the bins; with uint16 bins and B > 256 it
      feeds the wide-bin LDS kernel (feature groups per block) instead of global atomics
    """
    nwork = work.shape[0]
    if nwork == 0:
        return
    assert hist.dtype == torch.int64
    if bins.is_cuda:
        check_cuda(bins, ghp, rows, work, hist)
        assert hist.shape[1] == B and hist.shape[2] == F and hist.shape[3] == 2
        assert ghp.shape[1] == 2 and ghp.dtype == torch.float32
        if rows is None:
            assert ghp.shape[0] >= bins.shape[0]
        stride = bins.shape[1]
        h = hip()
        if bins.dtype == torch.uint8 and B <= 256 and stride % 32 == 0 and stride >= ((F + 31) // 32) * 32:
            if staging is not None and nslots > 0:
                assert staging.numel() >= nwork * hist_cols(F) * B * 2
                h.hist_fx_staged(ptr(bins), stride, F, ptr(ghp), ptr(rows), ptr(work), nwork, ptr(hist), B,
                                 float(sg), float(sh), 0, 0, ptr(staging), slot_base, nslots, ptr(slot_ids),
                                 0, stream(bins))
            else:
                h.hist_fx(ptr(bins), stride, F, ptr(ghp), ptr(rows), ptr(work), nwork, ptr(hist), B,
                          float(sg), float(sh), 0, 0, stream(bins))
        elif (bins.dtype == torch.int16 and wide_group(B, F) > 0 and stride % wide_group(B, F) == 0
              and bins.is_contiguous()):
            # row-major wide-bin LDS kernel (feature groups per block, one vector load per row)
            use_st = staging is not None and nslots > 0 and slot_ids is None
            if use_st:
                assert staging.numel() >= nwork * hist_cols(F) * B * 2
            h.hist_wide_rm(ptr(bins), stride, F, ptr(ghp), ptr(rows), ptr(work), nwork, ptr(hist), B,
                           float(sg), float(sh), 0, 0, 0, ptr(staging) if use_st else 0, slot_base,
                           nslots if use_st else 0,
                           ptr(binsT) if (binsT is not None and binsT.dtype == torch.int16 and binsT.is_contiguous()
                                          and binsT.shape[0] == F) else 0,
                           binsT.shape[1] if binsT is not None else 0, stream(bins))
        else:
            h.hist_fx_global(ptr(bins), _bin_bytes(bins), stride, F, ptr(ghp), ptr(rows), ptr(work),
                             nwork, ptr(hist), B, float(sg), float(sh), stream(bins))
        return
    # CPU reference (bitwise identical: integer sums)
    w = work.numpy()
    hv = hist.view(-1, 2)
    mask = 0xFFFF if bins.dtype == torch.int16 else 0xFF
    for slot, b, e, _ in w:
        if e <= b:
            continue
        r = rows[b:e].long() if rows is not None else torch.arange(b, e, dtype=torch.long)
        bb = bins[r, :F].long() & mask
        idx = (int(slot) * B + bb) * F + torch.arange(F, dtype=torch.long)[None, :]
        v = quantize_gh(ghp[b:e], sg, sh)[:, None, :].expand(-1, F, 2)
        hv.index_add_(0, idx.reshape(-1), v.reshape(-1, 2))


# ---------------------------------------------------------------------------
# split finding
# ---------------------------------------------------------------------------
def split_node_fits(B: int, F: int) -> bool:
    """Whether split_find runs the node-resident LDS kernel (same test as ytk_split_find
    in csrc/hip/gbdt_split.hip): then it needs no per-feature scratch."""
    return (B <= 256 and F * (B + 1) * 16 <= 144 * 1024 and B * F <= 8 * 1024 and F <= 256
            and os.environ.get("YTK_SPLIT_NODE") != "0")


def split_groups(B: int, F: int) -> int:
    """Feature groups per node for the node-resident split search (split_node_grouped:
    one block per (node, group), the planner keeps each node's best record). YTK_SPLIT_GROUPS
    (default 4, profiles/r2_split_groups.md); 1 when the node-resident kernel does not apply.
    Every group must hold at least one feature."""
    if not split_node_fits(B, F):
        return 1
    g = max(1, min(F, int(os.environ.get("YTK_SPLIT_GROUPS", "4"))))
    while g > 1 and (g - 1) * (-(-F // g)) >= F:
        g -= 1
    return g


def split_find(hist, B, F, nbins_f, fmask, f0, items, params):
    """Best split per item. items int32 [n, 4] = (slot, parent, sibling, derived).

    Returns a uint8 tensor [n, 48] (view with SPLIT_DTYPE after moving to host).
    Derived items also write their (parent - sibling) histogram into ``slot``.
    """
    n = items.shape[0]
    mcw, l1, l2, mal = (float(params[k]) for k in ("mcw", "l1", "l2", "max_abs_leaf"))
    inv_sg, inv_sh = 1.0 / float(params["sg"]), 1.0 / float(params["sh"])
    assert hist.dtype == torch.int64
    if hist.is_cuda:
        out = torch.empty((n, 48), dtype=torch.uint8, device=hist.device)
        if n == 0:
            return out
        check_cuda(hist, nbins_f, fmask, items)
        part = counters = None
        if not split_node_fits(B, F):  # the (node, feature) kernel combines through scratch
            part = torch.empty((n * F, 48), dtype=torch.uint8, device=hist.device)
            counters = torch.zeros(n, dtype=torch.int32, device=hist.device)
        hip().split_find(ptr(hist), B, F, ptr(nbins_f), ptr(fmask), int(f0), ptr(items), n,
                         ptr(out), mcw, l1, l2, mal, inv_sg, inv_sh, 0, 0, ptr(part), ptr(counters),
                         stream(hist))
        return out
    res = np.zeros(n, dtype=SPLIT_DTYPE)
    it = items.numpy()
    nb = nbins_f.numpy()
    fm = fmask.numpy().astype(bool)
    for i, (slot, par, sib, der) in enumerate(it):
        if der:
            hist[slot] = hist[par] - hist[sib]
        hn = hist[slot].numpy()  # [B, F, 2] int64
        res[i] = _split_one_cpu(hn, nb, fm, int(f0), mcw, l1, l2, mal, inv_sg, inv_sh)
    return torch.from_numpy(res.view(np.uint8).reshape(n, 48).copy())


def _thr_l1(w, lam):
    return np.where(w > lam, w - lam, np.where(w < -lam, w + lam, 0.0))


def node_value_np(g, h, mcw, l1, l2, mal):
    g = np.asarray(g, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    v = (-g / (h + l2)) if l1 == 0.0 else (-_thr_l1(g, l1) / (h + l2))
    if mal > 0:
        v = np.clip(v, -mal, mal)
    return np.where(h < mcw, 0.0, v)


def node_value_py(g: float, h: float, mcw: float, l1: float, l2: float, mal: float) -> float:
    """Scalar ``node_value_np`` in plain Python floats (IEEE double, same results)."""
    if h < mcw:
        return 0.0
    if l1 == 0.0:
        v = -g / (h + l2)
    else:
        t = g - l1 if g > l1 else (g + l1 if g < -l1 else 0.0)
        v = -t / (h + l2)
    if mal > 0:
        v = min(max(v, -mal), mal)
    return v


def calc_gain_np(g, h, mcw, l1, l2, mal):
    g = np.asarray(g, dtype=np.float64)
    h = np.asarray(h, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        if mal <= 0:
            t = g if l1 == 0.0 else _thr_l1(g, l1)
            gain = t * t / (h + l2)
        else:
            v = node_value_np(g, h, mcw, l1, l2, mal)
            gain = -2.0 * (g * v + 0.5 * (h + l2) * v * v + l1 * np.abs(v))
    return np.where(h < mcw, 0.0, gain)


def _split_one_cpu(hn, nb, fm, f0, mcw, l1, l2, mal, inv_sg, inv_sh):
    Bn, Fn, _ = hn.shape
    Gq = int(hn[: nb[f0], f0, 0].sum())
    Hq = int(hn[: nb[f0], f0, 1].sum())
    G, H = float(np.float64(Gq) * inv_sg), float(np.float64(Hq) * inv_sh)
    root_gain = np.float32(calc_gain_np(G, H, mcw, l1, l2, mal))
    best = (-np.inf, 1 << 30, 1 << 30)
    rec = (np.float32(-np.inf), -1, -1, -1, 0.0, 0.0)
    for f in range(Fn):
        if not fm[f]:
            continue
        m = min(nb[f], Bn)
        gq = hn[:m, f, 0]
        hq = hn[:m, f, 1]
        ne = (gq != 0) | (hq != 0)
        pgq = np.concatenate([[0], np.cumsum(gq)[:-1]]).astype(np.int64)  # exclusive prefix
        phq = np.concatenate([[0], np.cumsum(hq)[:-1]]).astype(np.int64)
        pg, ph = pgq.astype(np.float64) * inv_sg, phq.astype(np.float64) * inv_sh
        idx = np.where(ne, np.arange(m), -1)
        lastne = np.maximum.accumulate(idx) if m else idx
        prev = np.concatenate([[-1], lastne[:-1]])
        ok = ne & (prev >= 0) & (phq != 0) & (ph >= mcw)
        rg, rh = (Gq - pgq).astype(np.float64) * inv_sg, (Hq - phq).astype(np.float64) * inv_sh
        ok &= rh >= mcw
        if not ok.any():
            continue
        chg = (calc_gain_np(pg, ph, mcw, l1, l2, mal) + calc_gain_np(rg, rh, mcw, l1, l2, mal)
               - np.float64(root_gain)).astype(np.float32)
        chg = np.where(ok, chg, np.float32(-np.inf))
        j = int(np.argmax(chg))  # first max -> lowest bin
        c = chg[j]
        if (c > best[0]) or (c == best[0] and f < best[1]):
            best = (c, f, j)
            rec = (np.float32(c), f, int(prev[j]), j, float(pg[j]), float(ph[j]))
    out = np.zeros((), dtype=SPLIT_DTYPE)
    out["loss_chg"], out["feat"], out["bin_a"], out["bin_b"], out["gl"], out["hl"] = rec
    out["g"], out["h"] = G, H
    return out


# ---------------------------------------------------------------------------
# partition
# ---------------------------------------------------------------------------
def partition(binsT, rows, rows_out, ghp, gh_out, flags, items, feat, thr, node_begin, first_blk,
              nblk, n_split):
    """Stable partition of node segments; moves row ids AND position-ordered (g, h).

    binsT: column-major bins [F, N]; items int32 [nblk_total, 4] = (split_idx, begin, end,
    blk_in_node); go left iff binsT[feat, row] <= thr. Returns left counts int32 [n_split].
    """
    if binsT.is_cuda:
        left = torch.zeros(n_split, dtype=torch.int32, device=binsT.device)
        nitems = items.shape[0]
        if nitems == 0:
            return left
        check_cuda(binsT, rows, rows_out, ghp, gh_out, flags, items, feat, thr, node_begin,
                   first_blk, nblk)
        counts = torch.empty(nitems, dtype=torch.int32, device=binsT.device)
        hip().partition(ptr(binsT), _bin_bytes(binsT), binsT.shape[1], ptr(rows), ptr(rows_out),
                        ptr(ghp), ptr(gh_out), ptr(flags), ptr(items), nitems, ptr(feat), ptr(thr),
                        ptr(node_begin), ptr(first_blk), ptr(nblk), ptr(counts), ptr(left), 0, 0,
                        stream(binsT))
        return left
    left = torch.zeros(n_split, dtype=torch.int32)
    nbv, fv, tv, nb_ = node_begin.numpy(), feat.numpy(), thr.numpy(), nblk.numpy()
    fb = first_blk.numpy()
    it = items.numpy()
    mask = 0xFFFF if binsT.dtype == torch.int16 else 0xFF
    for i in range(n_split):
        if nb_[i] == 0:
            continue
        b = int(it[fb[i], 1])
        e = int(it[fb[i] + nb_[i] - 1, 2])
        assert b == nbv[i]
        r = rows[b:e] if rows is not None else torch.arange(b, e, dtype=torch.int32)
        g = ghp[b:e]
        go = (binsT[int(fv[i])][r.long()].long() & mask) <= int(tv[i])
        nl = int(go.sum())
        rows_out[b:b + nl] = r[go]
        rows_out[b + nl:e] = r[~go]
        gh_out[b:b + nl] = g[go]
        gh_out[b + nl:e] = g[~go]
        left[i] = nl
    return left


PART_CHUNK = 2048  # rows per block of the single-pass partition kernel


def partition_atomic(binsT, rows, rows_out, ghp, gh_out, first_blk, hdr, nblocks, feat, thr,
                     node_begin, node_count, cursor=None):
    """Single-pass partition (GPU): each 2048-row chunk reserves its left run at the front
    and its right run at the back of its node segment with one atomic; chunks land in
    any order (rows inside a chunk keep theirs). hdr int32 [2] = (n_split, n_blocks) on the
    device; first_blk = exclusive scan of ceil(count / 2048). Returns left counts (int64).
    ``cursor`` (optional int64 device buffer >= n_split): zeroed here with one async
    memset and returned RAW -- (right rows << 32) | left rows; mask on the host."""
    n = feat.shape[0]
    if cursor is None:
        cursor = torch.zeros(max(n, 1), dtype=torch.int64, device=binsT.device)[:n]
        raw = False
    else:
        cursor = cursor[:n]
        raw = True
        if n:
            hip().memset_async(ptr(cursor), 0, n * 8, stream(binsT))
    if nblocks == 0 or n == 0:
        return cursor
    check_cuda(binsT, rows, rows_out, ghp, gh_out, first_blk, hdr, feat, thr, node_begin, node_count)
    hip().partition_atomic(ptr(binsT), _bin_bytes(binsT), binsT.shape[1], ptr(rows), ptr(rows_out),
                           ptr(ghp), ptr(gh_out), ptr(first_blk), ptr(hdr), ptr(hdr) + 4, nblocks,
                           ptr(feat), ptr(thr), ptr(node_begin), ptr(node_count), ptr(cursor), 0, 0,
                           stream(binsT))
    return cursor if raw else cursor & 0xFFFFFFFF


def segment_copy(items, src_rows, dst_rows, src_gh, dst_gh):
    """dst[p] = src[p] (row ids and (g, h)) for every chunk [b, e) of ``items`` [n, 4]."""
    n = items.shape[0]
    if n == 0:
        return
    if dst_rows.is_cuda:
        check_cuda(items, src_rows, dst_rows, src_gh, dst_gh)
        hip().segment_copy(ptr(items), n, ptr(src_rows), ptr(dst_rows), ptr(src_gh), ptr(dst_gh),
                           stream(dst_rows))
        return
    for _, b, e, _ in items.numpy():
        dst_rows[b:e] = src_rows[b:e]
        dst_gh[b:e] = src_gh[b:e]


def partition_count(binsT, rows, flags, items, feat, thr):
    """Per-block left counts only (no scatter). Returns int32 [nblk_total]."""
    nitems = items.shape[0]
    if binsT.is_cuda:
        counts = torch.zeros(max(nitems, 1), dtype=torch.int32, device=binsT.device)[:nitems]
        if nitems == 0:
            return counts
        check_cuda(binsT, rows, flags, items, feat, thr)
        hip().partition_count(ptr(binsT), _bin_bytes(binsT), binsT.shape[1], ptr(rows), ptr(flags),
                              ptr(items), nitems, ptr(feat), ptr(thr), ptr(counts), 0, 0, stream(binsT))
        return counts
    counts = torch.zeros(nitems, dtype=torch.int32)
    it = items.numpy()
    mask = 0xFFFF if binsT.dtype == torch.int16 else 0xFF
    for j, (si, b, e, _) in enumerate(it):
        r = rows[b:e].long() if rows is not None else torch.arange(b, e)
        counts[j] = int(((binsT[int(feat[si])][r].long() & mask) <= int(thr[si])).sum())
    return counts


# ---------------------------------------------------------------------------
# scoring
# ---------------------------------------------------------------------------
def _walk_bins(binsT, tree_arrays):
    tfeat, tthr, tleft, tright, tval = tree_arrays
    N = binsT.shape[1]
    node = torch.zeros(N, dtype=torch.long)
    tf, tt, tl, tr = (t.long() for t in (tfeat, tthr, tleft, tright))
    mask = 0xFFFF if binsT.dtype == torch.int16 else 0xFF
    ar = torch.arange(N)
    for _ in range(1 << 12):
        f = tf[node]
        active = f >= 0
        if not bool(active.any()):
            break
        b = binsT[f.clamp(min=0), ar].long() & mask
        nxt = torch.where(b <= tt[node], tl[node], tr[node])
        node = torch.where(active, nxt, node)
    return tval[node]


def tree_add_bins(binsT, tree_arrays, score, col):
    """score[:, col] += value(leaf(row)) traversing a bin-threshold tree (binsT column-major)."""
    tfeat, tthr, tleft, tright, tval = tree_arrays
    N = binsT.shape[1]
    if binsT.is_cuda:
        check_cuda(binsT, tfeat, tthr, tleft, tright, tval, score)
        hip().tree_add_bins(ptr(binsT), _bin_bytes(binsT), N, ptr(tfeat), ptr(tthr), ptr(tleft),
                            ptr(tright), ptr(tval), tfeat.shape[0], ptr(score), score.shape[1], col,
                            stream(binsT))
        return
    score[:, col] += _walk_bins(binsT, tree_arrays)


def forest_predict(X, forest, out, scale=1.0, leaf_out=None):
    """out[:, tout[t]] += scale * leaf_value(tree t, row) over raw float features.

    forest: dict of tensors nfeat, nthr, nleft, nright, ndefl (uint8), nval, troot, tout.
    With ``leaf_out`` (int32 [N, T]) writes per-tree leaf indices instead.
    """
    T = forest["troot"].shape[0]
    N = X.shape[0]
    if X.is_cuda:
        check_cuda(X, out, leaf_out, *forest.values())
        # narrow contiguous rows: whole row in registers, nodes in LDS (one launch either way)
        if X.is_contiguous() and hip().forest_predict_regs(
                ptr(X), X.shape[1], N, ptr(forest["nfeat"]), ptr(forest["nthr"]), ptr(forest["nleft"]),
                ptr(forest["nright"]), ptr(forest["ndefl"]), ptr(forest["nval"]), ptr(forest["troot"]),
                ptr(forest["tout"]), T, forest["nfeat"].numel(), ptr(out), out.shape[1] if out is not None else 0,
                float(scale), ptr(leaf_out), stream(X)):
            return
        hip().forest_predict(ptr(X), X.shape[1], N, ptr(forest["nfeat"]), ptr(forest["nthr"]),
                             ptr(forest["nleft"]), ptr(forest["nright"]), ptr(forest["ndefl"]),
                             ptr(forest["nval"]), ptr(forest["troot"]), ptr(forest["tout"]), T,
                             ptr(out), out.shape[1] if out is not None else 0, float(scale),
                             ptr(leaf_out), stream(X))
        return
    nf = forest["nfeat"].long()
    nt = forest["nthr"]
    nl = forest["nleft"].long()
    nr = forest["nright"].long()
    nd = forest["ndefl"].bool()
    nv = forest["nval"]
    ar = torch.arange(N)
    for t in range(T):
        root = int(forest["troot"][t])
        node = torch.full((N,), root, dtype=torch.long)
        for _ in range(1 << 12):
            f = nf[node]
            active = f >= 0
            if not bool(active.any()):
                break
            v = X[ar, f.clamp(min=0)]
            left = torch.where(torch.isnan(v), nd[node], v <= nt[node])
            node = torch.where(active, torch.where(left, nl[node], nr[node]), node)
        if leaf_out is not None:
            leaf_out[:, t] = (node - root).int()
        else:
            out[:, int(forest["tout"][t])] += scale * nv[node]


# ---------------------------------------------------------------------------
# binning
# ---------------------------------------------------------------------------
def bin_assign(X, cand, coff, out, outT=None):
    """Nearest-candidate bin id per element (FeatureApprData semantics).
    out: row-major [N, S]; outT (optional): column-major copy [F, N]."""
    N, F = X.shape
    if X.is_cuda:
        check_cuda(X, cand, coff, out, outT)
        hip().bin_assign(ptr(X), X.shape[1], N, F, ptr(cand), ptr(coff), ptr(out),
                         _bin_bytes(out), out.shape[1], ptr(outT), stream(X))
        return
    co = coff.numpy()
    for f in range(F):
        c = cand[co[f]:co[f + 1]]
        n = c.numel()
        if n <= 1:
            out[:, f] = 0
        else:
            x = X[:, f].contiguous()
            lo = torch.searchsorted(c, x, right=True)  # first candidate > x
            u = (lo - 1).clamp(min=0)
            eq = c[u] == x
            idx = torch.where(eq, u, lo.clamp(max=n - 1))
            prevv = c[(idx - 1).clamp(min=0)]
            down = (idx >= 1) & (x < (c[idx] + prevv) * 0.5)
            idx = torch.where(down, idx - 1, idx)
            idx = torch.where(x > c[n - 1], torch.full_like(idx, n - 1), idx)
            out[:, f] = idx.to(out.dtype)
        if outT is not None:
            outT[f] = out[:, f]


# ---------------------------------------------------------------------------
# gradients
# ---------------------------------------------------------------------------
ACC_LEN = 4 + 2 * 256 * 8  # == kAccLen (gbdt_score.hip): (loss, weight), counter, block partials


_LGY = {}  # id(label) -> (weakref to label, lgamma(label + 1) float64 on its device)


def label_term(label, loss) -> int:
    """Device address of lgamma(label + 1) (float64, one per label entry) for the Poisson loss,
    else 0: the kernels add this label term to the point loss instead of evaluating lgamma
    themselves (that inlined lgamma cost the fused gradient + histogram kernel 238 VGPR
    spills). Computed once per label tensor (cached while the tensor lives)."""
    if LOSS_IDS[loss] != 3:
        return 0
    import weakref
    hit = _LGY.get(id(label))
    if hit is None or hit[0]() is not label:
        if len(_LGY) > 16:
            for k in [k for k, (r, _) in _LGY.items() if r() is None]:
                del _LGY[k]
        hit = (weakref.ref(label), torch.lgamma(label.double() + 1.0).contiguous())
        _LGY[id(label)] = hit
    return ptr(hit[1])


def forest_predict_loss(X, tree, score, init, label, weight, loss, param, score_div, pred, finish=True):
    """Test-set round tail in one GPU pass (K == 1, ONE raw tree ``tree`` rooted at node 0, as
    forest_predict's dict; its troot / tout are not read): score += tree(row), then the loss sums and prediction -- exactly
    forest_predict + grad_hess(want_grad=False) (same values, same fp64 summation order).
    Returns the float64 [2] (loss sum, weight sum) device tensor, or None when the fused
    kernel does not apply (the caller then runs the two steps). ``finish=False``: returns
    (partials [ACC_LEN], number of partials) unfinished -- the caller finishes them with the
    train-side pass (tree_grad(te_acc=...)), one launch less per round."""
    loss_id = LOSS_IDS[loss]
    if not (X.is_cuda and X.is_contiguous() and score.shape[1] == 1 and loss_id != 5
            and tree["troot"].numel() == 1):
        return None
    check_cuda(X, score, init, label, weight, pred, *tree.values())
    acc = torch.empty(ACC_LEN, dtype=torch.float64, device=X.device)
    ok = hip().forest_loss_regs(ptr(X), X.shape[1], X.shape[0], ptr(tree["nfeat"]), ptr(tree["nthr"]),
                                ptr(tree["nleft"]), ptr(tree["nright"]), ptr(tree["ndefl"]), ptr(tree["nval"]),
                                0, tree["nfeat"].numel(), ptr(score),
                                ptr(init), ptr(label), label_term(label, loss), ptr(weight), loss_id, float(param),
                                float(score_div),
                                ptr(pred), ptr(acc), 1 if finish else 0, stream(X))
    if not ok:
        return None
    return acc[:2] if finish else (acc, int(ok))


def grad_hess(score, init, label, weight, loss, param, score_div, pred, gh, want_grad=True,
              ghmax=None):
    """Fill pred [N,K] (optional) and gh [K,N,2]; return (weighted loss sum, weight sum) as a
    float64 tensor of shape [2] on the data device (no host sync).

    ``ghmax`` (float32 [K,2], optional) is max-accumulated with max|g|, max|h| per class —
    the next trees' fixed-point histogram scales (see DeviceLevelBuilder)."""
    N, K = score.shape
    loss_id = LOSS_IDS[loss]
    if score.is_cuda:
        check_cuda(score, init, label, weight, pred, gh, ghmax)
        acc = torch.empty(ACC_LEN, dtype=torch.float64, device=score.device)  # fully written by the kernels
        hip().grad_hess(ptr(score), ptr(init), ptr(label), label_term(label, loss), ptr(weight), N, K, loss_id,
                        float(param), float(score_div), ptr(pred), ptr(gh), ptr(acc),
                        1 if want_grad else 0, ptr(ghmax), stream(score))
        return acc[:2]
    z = score.double() / score_div + init.double()
    y = label.double()
    w = weight.double() if weight is not None else torch.ones(N, dtype=torch.float64)
    if loss_id == 5:
        lse = torch.logsumexp(z, dim=1, keepdim=True)
        p = torch.exp(z - lse)
        lv = -(y * (z - lse)).sum(1)
        g = p - y
        h = 2.0 * p * (1.0 - p)
    else:
        z1, y1 = z[:, 0], y[:, 0]
        if loss_id == 0:
            lv = torch.where(z1 >= 0, torch.log1p(torch.exp(-z1)) + z1 * (1 - y1),
                             torch.log1p(torch.exp(z1)) - z1 * y1)
            p = torch.sigmoid(z1).float().double()
            g = p - y1
            h = p * (1 - p)
            if param != 0:
                zz = torch.where(h != 0, -(g / h), torch.zeros_like(h))
                h = torch.where(zz > param, -(g / param), torch.where(zz < -param, -(g / -param), h))
        elif loss_id == 1:
            lv = 0.5 * (y1 - z1) ** 2
            p = z1.float().double()
            g = p - y1
            h = torch.ones_like(p)
        elif loss_id == 2:
            lv = (y1 - z1).abs()
            p = z1.float().double()
            g = torch.sign(p - y1)
            h = torch.ones_like(p)
        elif loss_id == 3:
            zc = torch.clamp(z1, max=30.0)
            lv = -y1 * z1 + torch.exp(zc) + torch.lgamma(y1 + 1)
            p = torch.exp(zc).float().double()
            g = p - y1
            h = p
        else:
            a = z1 - y1
            d = float(param)
            lv = torch.where(a.abs() <= d, 0.5 * a * a, d * (a.abs() - 0.5 * d))
            p = z1.float().double()
            aa = p - y1
            g = torch.where(aa.abs() <= d, aa, torch.sign(aa) * d)
            h = torch.zeros_like(p)
        p, g, h = p[:, None], g[:, None], h[:, None]
    if pred is not None:
        pred.copy_(p.float())
    if want_grad:
        gh[:, :, 0] = (g * w[:, None]).float().t()
        gh[:, :, 1] = (h * w[:, None]).float().t()
        if ghmax is not None:
            m = gh.abs().amax(dim=1).reshape(ghmax.shape)
            ghmax.copy_(torch.maximum(ghmax, m))
    return torch.tensor([float((w * lv).sum()), float(w.sum())], dtype=torch.float64)


# (work item, feature group) blocks per level of the wide-bin (B > 256) histograms: one
# 160-KiB block per CU, so this many blocks is ~4 rounds over the 256 CUs
WIDE_HIST_BLOCKS = int(os.environ.get("YTK_WIDE_HIST_BLOCKS", 1024))
LDS_BUDGET = 160 * 1024 - 1024  # == kLdsBudget (csrc/hip/common.h)


def leaf_counts_fit(max_nodes: int) -> bool:
    """Whether tree_grad can count rows per node for trees of ``max_nodes`` nodes: the
    per-block counters sit in LDS next to the five node arrays (6 ints per node)."""
    return max_nodes * 6 * 4 <= LDS_BUDGET


def acc_finish(acc, nblocks, out):
    """Ordered finish of a pass's loss partials (forest_predict_loss(finish=False)) into out[0:2]."""
    hip().acc_finish(ptr(acc), int(nblocks), ptr(out), 0, 0, 0, stream(acc))


def tree_grad(bins, tree_arrays, score, init, label, weight, loss, param, score_div, pred, gh,
              want_grad=True, ghmax=None, leaf_counts=None, root=None, acc_out=None, te_acc=None):
    """Fused K==1 round tail: score += tree(row) (bin space, ROW-MAJOR bins [N, S]), then
    pred (optional) / (g, h) / loss sums / max|g|,|h| (optional ``ghmax`` [1,2]).
    ``tree_arrays`` may be None (no tree). Returns float64 [2] (loss sum, weight sum).
    ``leaf_counts`` (optional, float64 [nodes], GPU): rows per tree node from the same walk
    (the level engine's last-level leaf counts without a counting partition pass).
    ``root`` (optional dict, GPU): also accumulate the NEXT tree's root histogram in the same
    pass (tree_grad_hist_kernel) into the zeroed slot ``root["slot"]`` with the fixed-point
    scales ``root["scales"]``; ``root["done"]`` reports whether the fused pass ran (layouts it
    does not cover fall back to the plain pass).
    ``acc_out`` (optional, float64 [2], GPU): where the loss sums go (the returned tensor is
    then ``acc_out``); ``te_acc`` (optional): (partials, count, out [2]) of the test-set pass
    to finish in the same launch (falls back to its own finish launch)."""
    loss_id = LOSS_IDS[loss]
    assert loss_id != 5 and score.shape[1] == 1
    if score.is_cuda:
        N = score.shape[0]
        acc = torch.empty(ACC_LEN, dtype=torch.float64, device=score.device)  # fully written by the kernels
        if tree_arrays is None:
            tf = tt = tl = tr = tv = None
            nn = 0
        else:
            tf, tt, tl, tr, tv = tree_arrays
            nn = tf.shape[0]
            assert bins is not None and bins.shape[0] == N and bins.stride(1) == 1
        check_cuda(bins, score, init, label, weight, pred, gh, ghmax, tf, tt, tl, tr, tv, leaf_counts)
        part = None
        if leaf_counts is not None:
            assert nn > 0 and leaf_counts.dtype == torch.float64 and leaf_counts.numel() >= nn
            # rows per (virtual block, node): the fused pass may run more virtual blocks
            # (YTK_TGH_VBLOCKS) than the plain gradient kernel
            nvb = max(hip().tree_grad_grid(N), 4 * hip().tree_grad_hist_grid(N))
            part = torch.empty(nvb * nn, dtype=torch.int32, device=score.device)
        if root is not None:
            root["done"] = False
            if (tree_arrays is not None and want_grad and bins.dtype == torch.uint8 and bins.stride(0) == 32
                    and nn > 0):
                root["done"] = bool(hip().tree_grad_hist(
                    ptr(bins), bins.stride(0), ptr(tf), ptr(tt), ptr(tl), ptr(tr), ptr(tv), nn, ptr(score), ptr(init),
                    ptr(label), label_term(label, loss), ptr(weight), N, loss_id, float(param), float(score_div),
                    ptr(pred), ptr(gh), ptr(acc),
                    ptr(ghmax), ptr(part), ptr(leaf_counts), root["scales"], root["staging"], root["work"],
                    root["slot"], root["B"], root["F"], ptr(acc_out),
                    ptr(te_acc[0]) if te_acc is not None else 0, int(te_acc[1]) if te_acc is not None else 0,
                    ptr(te_acc[2]) if te_acc is not None else 0, root.get("zero", 0), root.get("zero_n", 0),
                    stream(score)))
            if root["done"]:
                return acc_out if acc_out is not None else acc[:2]
        ok = hip().tree_grad(ptr(bins), _bin_bytes(bins) if bins is not None else 1,
                        bins.stride(0) if bins is not None else 0, ptr(tf), ptr(tt), ptr(tl),
                        ptr(tr), ptr(tv), nn, ptr(score), ptr(init), ptr(label), label_term(label, loss),
                        ptr(weight), N,
                        loss_id, float(param), float(score_div), ptr(pred), ptr(gh), ptr(acc),
                        1 if want_grad else 0, ptr(ghmax), ptr(part), ptr(leaf_counts), stream(score))
        if not ok:
            raise ValueError(f"tree_grad: per-node leaf counts of a {nn}-node tree exceed the LDS budget "
                             "(see leaf_counts_fit)")
        if te_acc is not None:
            acc_finish(te_acc[0], te_acc[1], te_acc[2])
        if acc_out is not None:
            acc_out.copy_(acc[:2])
            return acc_out
        return acc[:2]
    assert leaf_counts is None, "leaf_counts: GPU only"
    if tree_arrays is not None:
        score[:, 0] += _walk_bins(bins.t(), tree_arrays)
    return grad_hess(score, init, label, weight, loss, param, score_div, pred, gh.unsqueeze(0),
                     want_grad, ghmax)
