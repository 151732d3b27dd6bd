"""Per-slot sums of row values without hot-slot atomics (evaluators, quantile sketches).

torch.bincount / index_add_ on the GPU add with fp64 atomics; when many rows share a slot
(clustered predictions, few groups, tied values) those serialise on a few addresses:
10.5M rows into 4 cells took 131 ms on MI355X against 1.2 ms for one sort + segmented sums
(``profiles/r3s4_slot_sums_microbench.txt``), whose summation order is also the same every
run."""
from __future__ import annotations

import torch


def slot_sums(slot: torch.Tensor, w: torch.Tensor, n: int) -> torch.Tensor:
    """float64 [2, n]: per-slot weight sums and row counts of int64 ``slot`` in [0, n).

    On the GPU: one sort of the slot ids, then segmented sums over the runs of equal ids
    (torch.segment_reduce) scattered to their slots. torch.bincount's fp64 atomics pile onto
    the few slots clustered predictions fall into (and their order varies run to run); the
    sorted sums take the same order every run."""
    if not slot.is_cuda:
        return torch.stack([torch.bincount(slot, weights=w, minlength=n), torch.bincount(slot, minlength=n).double()])
    h = torch.zeros((2, n), dtype=torch.float64, device=slot.device)
    if slot.numel() == 0:
        return h
    key = slot.to(torch.int32) if n < 2 ** 31 else slot
    s, order = torch.sort(key, stable=True)
    ids, counts = torch.unique_consecutive(s, return_counts=True)
    ids = ids.long()
    h[0, ids] = torch.segment_reduce(w[order], "sum", lengths=counts)
    h[1, ids] = counts.double()
    return h


def run_sums(w_sorted: torch.Tensor, inv: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """float64 sums of ``w_sorted`` over its runs (run k = ``counts[k]`` consecutive rows;
    ``inv`` the run id of every row): segmented sums on the GPU, index_add_ on the CPU."""
    w = w_sorted.double()
    if w.is_cuda:
        return torch.segment_reduce(w, "sum", lengths=counts)
    return torch.zeros(counts.numel(), dtype=torch.float64).index_add_(0, inv, w)
