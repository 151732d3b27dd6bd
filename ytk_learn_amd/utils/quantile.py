"""Weighted mergeable quantile summaries (native ``WQSummary``, csrc/native/wquantile.cpp).

Reference: ``J/utils/WeightApproximateQuantile.java`` -- per-worker summaries are built
locally, exchanged with an object collective, merged in a fixed order and queried. Used by
sample_by_quantile binning, the quantile missing-value fill and the l1 leaf refine.
A summary is a float64 array [n, 4] = (value, rmin, rmax, wmin).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ..ops._ext import native


def build(values, weights=None, size: int = 0) -> np.ndarray:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(-1))
    w = (np.ones_like(v) if weights is None
         else np.ascontiguousarray(np.asarray(weights, dtype=np.float64).reshape(-1)))
    return native().wq_build(v, w, int(size))


def merge(summaries: Sequence[np.ndarray], size: int = 0) -> np.ndarray:
    out = np.zeros((0, 4), np.float64)
    nat = native()
    for s in summaries:
        out = nat.wq_combine(out, np.asarray(s, np.float64).reshape(-1, 4), int(size))
    return out


def total(summary: np.ndarray) -> float:
    return float(summary[-1, 2]) if len(summary) else 0.0


def query(summary: np.ndarray, fractions) -> np.ndarray:
    """Values at rank fraction q * W for every q in ``fractions``."""
    q = np.asarray(fractions, dtype=np.float64).reshape(-1)
    return native().wq_query(summary, q * total(summary))


def distributed_quantiles(values, weights, fractions, comm, size: int) -> np.ndarray:
    """Quantiles of the union of every rank's (values, weights): local summary of ``size``
    entries, object all-gather, merge in rank order (identical on every rank), query."""
    local = build(values, weights, size)
    parts = [p[0] for p in allgather_summaries([local], comm)]
    return query(merge(parts, size), fractions)


def device_summary(vals, w, size: int):
    """``WQSummary::from_sorted`` + ``prune(size)`` (csrc/native/wquantile.cpp:22-61) on the
    device, vectorised: ``vals`` sorted DISTINCT float64, ``w`` their float64 weights.
    Returns float64 [m, 4] (value, rmin, rmax, wmin) on the same device.

    The prune walk is monotone, so each target rank d_k = W k / (size - 1) maps to
    i_k = first index >= 1 with mid >= d_k (clamped to n - 1) by one searchsorted; the
    nearer of i_k - 1 / i_k is kept, duplicates dropped, first and last always kept --
    the same entries as the sequential loop (bit-identical when the weight prefix sums
    are exact, e.g. counts)."""
    import torch

    n = vals.numel()
    if n == 0:
        return torch.zeros((0, 4), dtype=torch.float64, device=vals.device)
    cum = torch.cumsum(w, 0)
    rmin = torch.cat([cum.new_zeros(1), cum[:-1]])
    ent = torch.stack([vals, rmin, cum, w], 1)
    if n <= size or size < 3:
        return ent
    mid = (rmin + cum) * 0.5
    W = cum[-1]
    k = torch.arange(1, size - 1, dtype=torch.float64, device=vals.device)
    d = W * k / float(size - 1)
    i = (1 + torch.searchsorted(mid[1:].contiguous(), d, right=False)).clamp_(max=n - 1)
    a = (mid[i - 1] - d).abs()
    b = (mid[i] - d).abs()
    j = torch.where((i > 1) & (a < b), i - 1, i)
    j = j[(j >= 1) & (j + 1 < n)]
    j = torch.unique_consecutive(j)
    idx = torch.cat([j.new_zeros(1), j, j.new_full((1,), n - 1)])
    return ent[idx]


def allgather_summaries(local, comm) -> List[List[np.ndarray]]:
    """All ranks' summary lists ([rank][i] -> float64 [m_i, 4]) with two fixed-shape
    tensor all-gathers (lengths, then the padded concatenation) instead of a pickled
    object collective. ``local``: list of float64 [m_i, 4] numpy arrays or tensors."""
    import torch

    ts = [torch.as_tensor(np.asarray(x, np.float64).reshape(-1, 4)) if not torch.is_tensor(x) else x.double()
          for x in local]
    dev = ts[0].device if ts else torch.device("cpu")
    lens = torch.tensor([t.shape[0] for t in ts], dtype=torch.int64, device=dev)
    flat = torch.cat(ts) if ts else torch.zeros((0, 4), dtype=torch.float64, device=dev)
    if comm is None or not comm.is_dist:
        all_lens, all_flat = [lens], [flat]
    else:
        all_lens = comm.allgather(lens).view(comm.world, -1)
        all_flat = comm.allgather_ragged(flat)
    out = []
    for r in range(len(all_flat)):
        L = all_lens[r].cpu().numpy()
        F = all_flat[r].cpu().numpy()
        offs = np.concatenate([[0], np.cumsum(L)])
        out.append([F[offs[i]:offs[i + 1]] for i in range(len(L))])
    return out


def _first_reaching(cum: "np.ndarray", target: "np.ndarray") -> "np.ndarray":
    """Per row of cum [G, K]: first column whose value >= target[g] (K if none)."""
    ok = cum >= target[:, None]
    return np.where(ok.any(axis=1), ok.argmax(axis=1), cum.shape[1])


MEDIAN_STATS = {"gathered_local": 0}  # rows this rank put into the last survivor gather


def distributed_weighted_median(values, weights, groups, n_groups: int, comm, buckets: int = 1024,
                                gather_max: int = 8192, max_rounds: int = 8):
    """EXACT weighted median per group of the union of every rank's rows, with fixed-size
    tensor collectives only (reference: J/utils/PreciseQuantile.java:237-320 -- count,
    bucket, per-bucket weight sums, locate the bucket holding the median, gather that
    bucket's values).

    Each round histograms the surviving rows of every group into ``buckets`` equal-width
    value buckets over the group's global [min, max] (one all-reduce of G x K weights and
    counts), keeps only the bucket where the cumulative weight reaches half the group's
    weight (adding the weight below it to an offset), until every group has at most
    ``gather_max`` survivors; those are all-gathered (padded tensors) and the median is the
    first sorted survivor whose offset + cumulative weight >= W / 2 -- the same rule as a
    single-process sort (``_weighted_median_sorted``). Returns float64 [G] (NaN for empty
    groups). values / weights: float64 tensors, groups: int64 tensor in [0, G)."""
    import torch

    from .segsum import slot_sums
    v = values.double().reshape(-1)
    w = weights.double().reshape(-1)
    g = groups.long().reshape(-1)
    G, K = int(n_groups), int(buckets)
    dev = v.device
    W = slot_sums(g, w, G)[0]
    lo = torch.full((G,), float("inf"), dtype=torch.float64, device=dev).scatter_reduce(0, g, v, "amin")
    hi = torch.full((G,), float("-inf"), dtype=torch.float64, device=dev).scatter_reduce(0, g, v, "amax")
    comm.allreduce_(W)
    comm.allreduce_(lo, op="min")
    comm.allreduce_(hi, op="max")
    target = 0.5 * W.cpu().numpy()
    below = np.zeros(G, np.float64)
    alive = torch.ones_like(g, dtype=torch.bool)
    lo_np, hi_np = lo.cpu().numpy(), hi.cpu().numpy()
    # groups whose surviving rows all hold ONE value are resolved on the spot (median = that
    # value) and leave the gather: heavy ties (e.g. integer residuals) would otherwise keep
    # landing in one bucket and ship every tied row to every rank
    resolved = np.full(G, np.nan)
    for _ in range(max_rounds):
        ga = g[alive]
        cnt = slot_sums(ga, torch.ones_like(ga, dtype=torch.float64), G)[1].to(torch.int64)
        comm.allreduce_(cnt)
        cnt_np = cnt.cpu().numpy()
        flat = (cnt_np > 0) & (hi_np <= lo_np) & np.isnan(resolved)
        if flat.any():
            resolved[flat] = lo_np[flat]
            fl_t = torch.from_numpy(flat).to(dev)
            alive &= ~fl_t[g]
            cnt_np = np.where(flat, 0, cnt_np)
        if cnt_np.max(initial=0) <= gather_max:
            break
        width = (hi_np - lo_np) / K
        width = np.where(width > 0, width, 1.0)
        gi = g[alive]
        vi = v[alive]
        lo_t = torch.from_numpy(lo_np).to(dev)
        wd_t = torch.from_numpy(width).to(dev)
        b = torch.floor((vi - lo_t[gi]) / wd_t[gi]).clamp_(0, K - 1).long()
        hw = slot_sums(gi * K + b, w[alive], G * K)[0]
        comm.allreduce_(hw)
        cum = below[:, None] + np.cumsum(hw.view(G, K).cpu().numpy(), axis=1)
        kstar = np.minimum(_first_reaching(cum, target), K - 1)
        prev = np.where(kstar > 0, cum[np.arange(G), np.maximum(kstar - 1, 0)], below)
        # groups already small (or degenerate: one distinct value) keep all survivors
        small = (cnt_np <= gather_max) | (hi_np <= lo_np)
        kk = torch.from_numpy(np.where(small, -1, kstar)).to(dev)
        keep = (kk[gi] < 0) | (b == kk[gi])
        below = np.where(small, below, prev)
        new_lo = np.where(small, lo_np, lo_np + kstar * width)
        new_hi = np.where(small, hi_np, np.minimum(hi_np, lo_np + (kstar + 1) * width))
        alive_idx = torch.nonzero(alive).flatten()
        alive[alive_idx[~keep]] = False
        # the survivors' actual range (one MIN all-reduce of (min, -max)): a bucket holding a
        # single distinct value collapses to hi == lo and is resolved next round
        gi2, vi2 = g[alive], v[alive]
        mm = torch.full((2 * G,), float("inf"), dtype=torch.float64, device=dev)
        mm[:G].scatter_reduce_(0, gi2, vi2, "amin")
        mm[G:].scatter_reduce_(0, gi2, -vi2, "amin")
        comm.allreduce_(mm, op="min")
        mm_np = mm.cpu().numpy()
        act_lo, act_hi = mm_np[:G], -mm_np[G:]
        lo_np = np.where(small, new_lo, np.where(np.isfinite(act_lo), act_lo, new_lo))
        hi_np = np.where(small, new_hi, np.where(np.isfinite(act_hi), act_hi, new_hi))
    # gather the survivors (padded all-gather of (group, value, weight))
    idx = torch.nonzero(alive).flatten()
    MEDIAN_STATS["gathered_local"] = int(idx.numel())
    n_loc = torch.tensor([idx.numel()], dtype=torch.int64, device=dev)
    if comm.is_dist:
        ns = comm.allgather(n_loc).cpu().numpy()
        m = int(ns.max())
        pad = torch.zeros((m, 3), dtype=torch.float64, device=dev)
        pad[:idx.numel(), 0] = g[idx].double()
        pad[:idx.numel(), 1] = v[idx]
        pad[:idx.numel(), 2] = w[idx]
        allr = comm.allgather(pad).cpu().numpy().reshape(comm.world, m, 3)
        rows = np.concatenate([allr[r, :ns[r]] for r in range(comm.world)])
    else:
        rows = torch.stack([g[idx].double(), v[idx], w[idx]], 1).cpu().numpy()
    out = resolved.copy()
    if rows.size:
        o = np.lexsort((rows[:, 1], rows[:, 0]))
        rows = rows[o]
        gs = rows[:, 0].astype(np.int64)
        starts = np.flatnonzero(np.r_[True, gs[1:] != gs[:-1]])
        ends = np.r_[starts[1:], len(gs)]
        for s, e in zip(starts, ends):
            k = gs[s]
            c = below[k] + np.cumsum(rows[s:e, 2])
            i = int(np.searchsorted(c, target[k], side="left"))
            out[k] = rows[s + min(i, e - s - 1), 1]
    return out
