"""One-shot peer-memory all-reduce for the tree engines' histogram messages (xGMI).

mp4j's histogram collectives were latency-optimised recursive-halving / Rabenseifner
algorithms (docs/gbdt_features.md:36,142-143, HistogramBuilder.java:95); at a 1/8 shard a
level's build takes 10-20 us, so the collective's latency sets the multi-GPU tree time.
This path replaces the RCCL call of a level with five stream-ordered launches and no host
involvement (``csrc/hip/gbdt_comm.hip``): every rank exports ONE uncached device block
[signal | send | recv] with hipIpcGetMemHandle, the handles travel once over the host
group, and each all-reduce is pack -> device barrier -> two-shot reduce (rank r sums chunk r
of every send slab and writes it into every recv slab) -> device barrier -> unpack.
Integer (int64) sums: the result is bitwise the RCCL result.

Opt-in (``YTK_PEER_REDUCE=1``) until measured on an 8-GPU node; RCCL stays the default.
Barrier waits are bounded (``YTK_PEER_MAX_SPINS``); a timed-out wait sets an error word
that :meth:`check` turns into an exception.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..ops._ext import hip, ptr, stream
from .comm import Comm


def enabled(comm: Comm) -> bool:
    return comm.is_dist and comm.device.type == "cuda" and os.environ.get("YTK_PEER_REDUCE", "0") == "1"


class PeerReduce:
    MAX_SPINS = int(os.environ.get("YTK_PEER_MAX_SPINS", 20_000_000))

    def __init__(self, comm: Comm, cap_elems: int):
        self.comm = comm
        self.cap = int(cap_elems)
        h = hip()
        handle = np.zeros(64, np.uint8)
        self.hnd = h.peer_create(comm.world, comm.rank, self.cap, handle.ctypes.data)
        parts = comm.allgather_bytes(handle.tobytes())  # rank order, host group
        allh = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
        h.peer_open(self.hnd, allh.ctypes.data)
        comm.barrier()
        self.calls = 0

    def allreduce_(self, t: torch.Tensor):
        """In-place sum over the ranks of a contiguous int64 device tensor (stream-ordered)."""
        assert t.dtype == torch.int64 and t.is_contiguous() and t.is_cuda
        n = t.numel()
        if n > self.cap:
            raise ValueError(f"peer all-reduce of {n} int64 exceeds the {self.cap}-element slab")
        hip().peer_allreduce(self.hnd, ptr(t), n, self.MAX_SPINS, stream(t))
        self.calls += 1
        self.comm.stats["calls"] += 1
        self.comm.stats["bytes"] += n * 8
        if self.comm.log is not None:
            self.comm.log.append(("peer_allreduce", "torch.int64", int(n)))

    def check(self):
        if hip().peer_check(self.hnd):
            raise RuntimeError("peer all-reduce: a device barrier wait timed out (a rank stopped issuing)")

    def close(self):
        if self.hnd is not None:
            hip().peer_destroy(self.hnd)
            self.hnd = None
