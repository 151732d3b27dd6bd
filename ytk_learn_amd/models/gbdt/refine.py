"""L1 (least-absolute-deviation) leaf refinement.

Reference: ``J/optimizer/gbdt/TreeRefiner.java:72-254`` -- for ``l1`` loss every
leaf value is replaced by learning_rate x weighted median of the residuals
(label - current score) of the rows in that leaf. ``lad_refine_appr`` selects the
mergeable-summary (approximate) or the exact distributed quantile.

Device-native: leaf ids come from the bin-threshold traversal kernel, the
per-leaf weighted medians from one segmented sort on the device (sort by
(leaf, residual), segmented cumulative weights).
  * approximate (lad_refine_appr = true, the reference default, TreeRefiner.java
    getLeafRefineValForLADAppr): weighted mergeable summaries per leaf on EVERY world
    size, sized like the reference's (eps 1e-5, exact up to 1e5 samples,
    Constants.java:55-56), merged in rank order;
  * exact (false, getLeafRefineValForLADPrecise + PreciseQuantile.java:237-320): one
    process sorts; across GPUs the bucketed distributed median of
    ``utils.quantile.distributed_weighted_median`` (fixed-size tensor collectives, no
    pickled residual lists).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ...ops import gbdt as gops
from ...parallel.comm import Comm

SUMMARY_POINTS = 100_000  # 1 / QUNANTILE_APPROXIMATE_EPS and QUNANTILE_PRECISION_MAX_SAMPLE_CNT


def _weighted_median_sorted(v: np.ndarray, w: np.ndarray) -> float:
    c = np.cumsum(w)
    i = int(np.searchsorted(c, 0.5 * c[-1], side="left"))
    return float(v[min(i, len(v) - 1)])


class TreeRefiner:
    def __init__(self, comm: Comm, approximate: bool = True):
        self.comm = comm
        self.approximate = approximate

    def leaf_ids(self, tree, binsT: torch.Tensor) -> torch.Tensor:
        n = tree.num_nodes
        # score column trick: value = node id, so tree_add_bins writes the leaf id
        feat, thr, left, right, _ = tree.bin_arrays()
        ids = np.arange(n, dtype=np.float32)
        out = torch.zeros((binsT.shape[1], 1), dtype=torch.float32, device=binsT.device)
        arrs = tuple(torch.from_numpy(a).to(binsT.device) for a in (feat, thr, left, right, ids))
        gops.tree_add_bins(binsT, arrs, out, 0)
        return out[:, 0].round().to(torch.int64)

    def refine(self, tree, builder, y: torch.Tensor, cur_score: torch.Tensor,
               w: torch.Tensor, lr: float):
        leaf = self.leaf_ids(tree, builder.binsT)
        keep = getattr(builder, "last_keep", None)
        resid = (y.double() - cur_score.double())
        ww = w.double() if w is not None else torch.ones_like(resid)
        if keep is not None:
            leaf, resid, ww = leaf[keep], resid[keep], ww[keep]
        leaves = tree.leaf_nodes()
        if not self.approximate and self.comm.is_dist:
            from ...utils.quantile import distributed_weighted_median
            gmax = int(os.environ.get("YTK_MEDIAN_GATHER_MAX", 8192))  # tests force bucket rounds
            med = distributed_weighted_median(resid, ww, leaf, tree.num_nodes, self.comm, gather_max=gmax)
            for nid in leaves:
                if not np.isnan(med[nid]):
                    tree.leaf[nid] = float(np.float32(med[nid]) * np.float32(lr))
            return
        # segmented sort on device: key = leaf * big + rank(resid)
        o = torch.argsort(resid)
        leaf_o = leaf[o]
        o2 = torch.argsort(leaf_o, stable=True)
        idx = o[o2]
        lv = leaf[idx].cpu().numpy()
        rv = resid[idx].cpu().numpy()
        wv = ww[idx].cpu().numpy()
        bounds = {}
        if lv.size:
            starts = np.flatnonzero(np.r_[True, lv[1:] != lv[:-1]])
            ends = np.r_[starts[1:], lv.size]
            for s, e in zip(starts, ends):
                bounds[int(lv[s])] = (s, e)
        local = {}
        for nid in leaves:
            if nid not in bounds:
                local[nid] = (np.zeros(0), np.zeros(0))
                continue
            s, e = bounds[nid]
            local[nid] = (rv[s:e], wv[s:e])
        if self.approximate:
            # weighted mergeable summaries (WeightApproximateQuantile), on every world size
            from ...utils import quantile as wq
            summ = [wq.build(*local[nid], SUMMARY_POINTS) for nid in leaves]
            parts = wq.allgather_summaries(summ, self.comm)  # two tensor all-gathers
            for li, nid in enumerate(leaves):
                sm = wq.merge([p[li] for p in parts], SUMMARY_POINTS)
                if len(sm) == 0:
                    continue
                med = float(wq.query(sm, [0.5])[0])
                tree.leaf[nid] = float(np.float32(med) * np.float32(lr))
            return
        for nid in leaves:  # exact, one process
            vs, ws = local[nid]
            if vs.size == 0:
                continue
            med = _weighted_median_sorted(vs, ws)
            tree.leaf[nid] = float(np.float32(med) * np.float32(lr))
