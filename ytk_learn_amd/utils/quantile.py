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
    parts: List[np.ndarray] = comm.allgather_object(local) if comm is not None and comm.is_dist else [local]
    return query(merge(parts, size), fractions)
