"""L1 (least-absolute-deviation) leaf refinement, on the device.

Reference: ``J/optimizer/gbdt/TreeRefiner.java:72-254`` -- for ``l1`` loss every
leaf value is replaced by learning_rate x weighted median of the residuals
(label - current score) of the rows in that leaf. ``lad_refine_appr`` selects the
mergeable-summary (approximate) or the exact distributed quantile.

Device-native, no row ever goes to the host:
  * leaf ids come from the bin-threshold walk (tree_add_bins with node ids as values);
  * rows are sorted by (leaf, residual) on the device and equal residuals of a leaf merge
    into summary entries (value, weight, leaf-local rank interval) -- per leaf exactly
    ``WQSummary::from_sorted`` (csrc/native/wquantile.cpp);
  * ``csrc/hip/gbdt_refine.hip`` answers per leaf: the exact sorted weighted median
    (lad_refine_appr = false; TreeRefiner getLeafRefineValForLADPrecise) or the query at
    W / 2 of the leaf's summary pruned to 100,000 entries (lad_refine_appr = true, the
    reference default, eps 1e-5 = Constants.java:55-56) -- one value per leaf reaches the
    host.
  * multi-GPU: exact mode runs the bucketed distributed median
    (``utils.quantile.distributed_weighted_median``: fixed-size tensor collectives, no row
    gather); approximate mode exchanges the per-leaf pruned summaries (two ragged tensor
    all-gathers) and merges them in rank order (the reference's allreduceMap of summaries).

The same code refines trees of the host-driven builder (its leaf values are patched on the
host tree) and of the GPU engines (their node tables and scoring arrays are patched in
place on the device, before the round's score update and test scoring).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ...ops import gbdt as gops
from ...ops._ext import hip, ptr, stream
from ...parallel.comm import Comm

SUMMARY_POINTS = 100_000  # 1 / QUNANTILE_APPROXIMATE_EPS and QUNANTILE_PRECISION_MAX_SAMPLE_CNT


def _weighted_median_sorted(v: np.ndarray, w: np.ndarray) -> float:
    c = np.cumsum(w)
    i = int(np.searchsorted(c, 0.5 * c[-1], side="left"))
    return float(v[min(i, len(v) - 1)])


def leaf_entries(leaf: torch.Tensor, resid: torch.Tensor, w: torch.Tensor, n_nodes: int):
    """Per-leaf weighted summaries of the residuals, all leaves in one set of arrays.

    Returns (v, rmin, rmax, mid, seg): entries sorted by (leaf, value), equal values of a
    leaf merged; rmin / rmax the entry's rank interval inside its leaf (rmax = rmin + its
    weight), mid = (rmin + rmax) / 2; leaf s owns entries [seg[s], seg[s + 1])."""
    dev = resid.device
    if resid.numel() == 0:
        z = torch.zeros(0, dtype=torch.float64, device=dev)
        return z, z, z, z, torch.zeros(n_nodes + 1, dtype=torch.int64, device=dev)
    o = torch.argsort(resid)
    o = o[torch.argsort(leaf[o], stable=True)]
    lv, rv, wv = leaf[o], resid[o], w[o]
    new = torch.ones_like(lv, dtype=torch.bool)
    new[1:] = (lv[1:] != lv[:-1]) | (rv[1:] != rv[:-1])
    eid = torch.cumsum(new.to(torch.int64), 0) - 1
    first = torch.nonzero(new).flatten()
    E = first.numel()
    v = rv[first]
    le = lv[first]
    if resid.is_cuda:
        # sorted runs: segmented sums (ties -- e.g. integer labels -- would pile fp64 atomics
        # onto one entry, ~100x slower at 10M rows; see metrics/evaluators.py:slot_sums)
        lens = torch.diff(first, append=torch.tensor([lv.numel()], dtype=first.dtype, device=dev))
        wx = torch.segment_reduce(wv.double(), "sum", lengths=lens)
    else:
        wx = torch.zeros(E, dtype=torch.float64, device=dev).index_add_(0, eid, wv)
    seg = torch.searchsorted(le, torch.arange(n_nodes + 1, dtype=le.dtype, device=dev))
    cw = torch.cumsum(wx, 0)
    excl = cw - wx
    base = excl[seg[:-1].clamp(max=max(E - 1, 0))]  # leaf-start offset of every leaf
    rmin = excl - base[le]
    rmax = rmin + wx
    return v, rmin, rmax, (rmin + rmax) * 0.5, seg


def _np_prune_picks(mid: np.ndarray, b: int, n: int, W: float, size: int) -> np.ndarray:
    """Entry offsets WQSummary::prune keeps for the targets k = 1 .. size - 2."""
    k = np.arange(1, size - 1, dtype=np.float64)
    d = W * k / float(size - 1)
    m = mid[b:b + n]
    i = np.minimum(1 + np.searchsorted(m[1:], d, side="left"), n - 1)
    a = np.abs(m[np.maximum(i - 1, 0)] - d)
    c = np.abs(m[i] - d)
    return np.where((i > 1) & (a < c), i - 1, i)


def seg_median(v, rmin, rmax, mid, seg, exact: bool, size: int = SUMMARY_POINTS) -> torch.Tensor:
    """Per leaf: exact weighted median (first entry with rmax >= W / 2) or the
    WQSummary query at W / 2 of the (pruned) summary. float64 [n_leaves], NaN if empty."""
    nseg = seg.numel() - 1
    out = torch.empty(nseg, dtype=torch.float64, device=v.device)
    if v.is_cuda:
        hip().seg_median(ptr(v), ptr(rmin), ptr(rmax), ptr(mid), ptr(seg), nseg, 0 if exact else 1, size,
                         ptr(out), stream(v))
        return out
    vv, r0, r1, mm, sg = (t.numpy() for t in (v, rmin, rmax, mid, seg))
    res = np.full(nseg, np.nan)
    for s in range(nseg):  # host fallback (CPU tensors): the kernel's rule, leaf by leaf
        b, e = int(sg[s]), int(sg[s + 1])
        n = e - b
        if n <= 0:
            continue
        W = r1[e - 1]
        if exact:
            i = min(b + int(np.searchsorted(r1[b:e], 0.5 * W, side="left")), e - 1)
            res[s] = vv[i]
            continue
        m2 = r0[b:e] + r1[b:e]
        if W <= m2[0]:
            res[s] = vv[b]
            continue
        if W >= m2[-1]:
            res[s] = vv[e - 1]
            continue
        idx = np.arange(n) if (n <= size or size < 3) else np.unique(
            np.concatenate([[0], _np_prune_picks(mm, b, n, W, size), [n - 1]]))
        lo = int(np.searchsorted(m2[idx], W, side="left"))
        a, c = W - m2[idx[lo - 1]], m2[idx[lo]] - W
        res[s] = vv[b + (idx[lo - 1] if a < c else idx[lo])]
    return torch.from_numpy(res)


def leaf_summaries(v, rmin, rmax, mid, seg, leaves, size: int = SUMMARY_POINTS):
    """WQSummary arrays [m, 4] = (value, rmin, rmax, wmin) of the given leaves, each pruned
    to ``size`` entries when larger (multi-GPU approximate mode exchanges these)."""
    sg = seg.cpu().numpy()
    out = []
    big = [s for s in leaves if sg[s + 1] - sg[s] > size >= 3]
    picks = {}
    if big and v.is_cuda:
        lv = torch.tensor(big, dtype=torch.int32, device=v.device)
        pick = torch.empty((len(big), size - 2), dtype=torch.int64, device=v.device)
        hip().seg_prune(ptr(mid), ptr(rmax), ptr(seg), ptr(lv), len(big), size, ptr(pick), stream(v))
        for i, s in enumerate(big):
            picks[s] = pick[i]
    for s in leaves:
        b, e = int(sg[s]), int(sg[s + 1])
        if e <= b:
            out.append(torch.zeros((0, 4), dtype=torch.float64, device=v.device))
            continue
        if s in picks or (e - b > size >= 3):
            p = picks[s] if s in picks else torch.from_numpy(
                b + _np_prune_picks(mid.numpy(), b, e - b, float(rmax[e - 1]), size))
            idx = torch.unique_consecutive(torch.cat([p.new_tensor([b]), p, p.new_tensor([e - 1])]))
        else:
            idx = torch.arange(b, e, device=v.device)
        out.append(torch.stack([v[idx], rmin[idx], rmax[idx], rmax[idx] - rmin[idx]], 1))
    return out


class TreeRefiner:
    def __init__(self, comm: Comm, approximate: bool = True):
        self.comm = comm
        self.approximate = approximate

    @staticmethod
    def leaf_ids(arrays, binsT: torch.Tensor) -> torch.Tensor:
        """Leaf node id of every row for a bin-threshold tree (feat, thr, left, right, ...)."""
        feat, thr, left, right = arrays[:4]
        n = feat.shape[0]
        ids = torch.arange(n, dtype=torch.float32, device=binsT.device)  # exact below 2^24
        out = torch.zeros((binsT.shape[1], 1), dtype=torch.float32, device=binsT.device)
        gops.tree_add_bins(binsT, (feat, thr, left, right, ids), out, 0)
        return out[:, 0].to(torch.int64)

    def medians(self, leaf, y, cur_score, w, keep, n_nodes: int, leaves) -> torch.Tensor:
        """float64 [n_nodes] weighted residual median per node (NaN: no rows), on the
        device of ``y``; ``leaves``: the leaf node ids (host ints)."""
        resid = y.double() - cur_score.double()
        ww = w.double() if w is not None else torch.ones_like(resid)
        if keep is not None:
            leaf, resid, ww = leaf[keep], resid[keep], ww[keep]
        if not self.approximate and self.comm.is_dist:
            from ...utils.quantile import distributed_weighted_median
            gmax = int(os.environ.get("YTK_MEDIAN_GATHER_MAX", 8192))  # tests force bucket rounds
            med = distributed_weighted_median(resid, ww, leaf, n_nodes, self.comm, gather_max=gmax)
            return torch.from_numpy(np.asarray(med, np.float64)).to(y.device)
        ent = leaf_entries(leaf, resid, ww, n_nodes)
        if not self.comm.is_dist:
            return seg_median(*ent, exact=not self.approximate)
        # approximate, multi-GPU: per-leaf pruned summaries -> rank-order merge -> query
        from ...utils import quantile as wq
        summ = leaf_summaries(*ent, leaves)
        parts = wq.allgather_summaries(summ, self.comm)  # two tensor all-gathers
        med = np.full(n_nodes, np.nan)
        for li, nid in enumerate(leaves):
            sm = wq.merge([p[li] for p in parts], SUMMARY_POINTS)
            if len(sm):
                med[nid] = float(wq.query(sm, [0.5])[0])
        return torch.from_numpy(med).to(y.device)

    def refine(self, tree, builder, y: torch.Tensor, cur_score: torch.Tensor, w: torch.Tensor, lr: float):
        """Host-built tree: leaf values patched on the host tree (one value per leaf read)."""
        dev = y.device
        if hasattr(builder, "leaf_ids_of"):  # raw-threshold (exact-greedy) trees
            leaf = builder.leaf_ids_of(tree)
        else:
            arrs = tuple(torch.from_numpy(a).to(dev) for a in tree.bin_arrays())
            leaf = self.leaf_ids(arrs, builder.binsT)
        leaves = tree.leaf_nodes()
        med = self.medians(leaf, y, cur_score, w, getattr(builder, "last_keep", None), tree.num_nodes,
                           leaves).cpu().numpy()
        for nid in leaves:
            if not np.isnan(med[nid]):
                tree.leaf[nid] = float(np.float32(med[nid]) * np.float32(lr))

    def refine_device(self, dt, builder, y: torch.Tensor, cur_score: torch.Tensor, w: torch.Tensor, lr: float):
        """GPU-engine tree (DeviceTree): the leaf values of its scoring arrays and node table
        -- and of the engine's live copies, which test-set scoring reads -- are replaced on
        the device; only the leaf list (one small copy) visits the host."""
        tf, tt, tl, tr, tv = dt.bin_arrays
        n = tf.shape[0]
        leaf = self.leaf_ids((tf, tt, tl, tr), builder.binsT)
        is_leaf = tf < 0
        leaves = torch.nonzero(is_leaf).flatten().cpu().tolist() if (self.comm.is_dist and self.approximate) else []
        med = self.medians(leaf, y, cur_score, w, getattr(builder, "last_keep", None), n, leaves)
        upd = is_leaf & ~torch.isnan(med)
        newv = torch.where(upd, med.float() * torch.tensor(np.float32(lr), device=tv.device), tv)
        targets = [(dt.nodes, tv)]
        live = builder.live_tree_views()
        if live[1].data_ptr() != tv.data_ptr():
            targets.append(live)
        for nodes, vals in targets:
            vals.copy_(newv)
            recs = nodes.view(torch.float32).view(-1, 22)[:n, 20]  # DNODE_DTYPE "value"
            recs.copy_(torch.where(upd, newv, recs))
