"""Peer-memory exchange for the tree engines' level / batch messages (xGMI), one kernel each.

mp4j's histogram collectives were latency-optimised recursive-halving / Rabenseifner
algorithms (docs/gbdt_features.md:36,142-143, HistogramBuilder.java:95); at a 1/8 shard a
level's build takes 10-20 us, so the collective's latency sets the multi-GPU tree time.
Here every rank exports ONE uncached device block [flag words | send slab 0 | send slab 1]
with hipIpcGetMemHandle, the handles travel once over the host group, and each all-reduce is
ONE stream-ordered kernel (``csrc/hip/gbdt_comm.hip`` ``peer_xchg_kernel``): every block
copies its chunk into the send slab, stamps a flag into every peer, waits for the peers'
flags of that chunk, and sums the chunk of all P slabs in rank order back into place. No
pack, unpack or barrier launches, no host involvement, and a message may be counted on the
device (the leaf-wise batch). int64 sums are exact (bitwise the RCCL result); fp64 sums
(the round's loss vector) are taken in rank order, identical on every rank.

Default for single-node multi-GPU jobs (every rank on this host: LOCAL_WORLD_SIZE ==
WORLD_SIZE); every rank must create and open every handle, else an all-rank vote falls back
to RCCL. ``YTK_PEER_REDUCE=0`` forces RCCL, ``=1`` forces the peer path (e.g. several ranks
sharing one GPU over gloo). Flag waits are bounded (``YTK_PEER_TIMEOUT_S``, default the
process-group timeout ``YTK_COMM_TIMEOUT``, 1800 s -- a rank may legitimately trail its peers by
rank-0-only host work such as a model dump; the start-up self-test waits at most 10 s); a timed-out
wait sets a host-mapped error word that :meth:`PeerReduce.check` (called where the trainer
lands its rounds) turns into an exception.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..ops._ext import hip, ptr, stream
from ..utils.fault import fault_point
from .comm import Comm


# outcome of the last peer-group creation on this process (bench / diagnostics):
# {"state": "off" | "ok" | "rccl", "reason": why the ranks voted for RCCL}
LAST_STATUS = {"state": "off", "reason": ""}


def enabled(comm: Comm) -> bool:
    mode = os.environ.get("YTK_PEER_REDUCE", "auto")
    if mode == "0" or not (comm.is_dist and comm.device.type == "cuda") or comm.world > 16:
        return False
    if mode == "1":
        return True
    # auto: one node, one process per GPU (torchrun sets LOCAL_WORLD_SIZE)
    return int(os.environ.get("LOCAL_WORLD_SIZE", comm.world)) == comm.world


def make(comm: Comm, cap_elems: int) -> Optional["PeerReduce"]:
    """A peer group for messages of up to ``cap_elems`` words, or None (RCCL) when the peer
    path is off or any rank failed to create / open its handles (all-rank vote)."""
    if not enabled(comm):
        LAST_STATUS.update(state="off", reason="YTK_PEER_REDUCE=0, not one node, or not a GPU job")
        return None
    return PeerReduce.create(comm, cap_elems)


class PeerReduce:
    _TYPES = {torch.int64: 0, torch.float64: 1, torch.float32: 2}

    def __init__(self, comm: Comm, hnd: int, cap: int):
        self.comm = comm
        # per flag wait (device wall clock): as long as the RCCL path it replaces would wait
        self.TIMEOUT_S = float(os.environ.get("YTK_PEER_TIMEOUT_S", os.environ.get("YTK_COMM_TIMEOUT", 1800.0)))
        self.hnd = hnd
        self.cap = int(cap)  # 8-byte words
        self.cap_bytes = 8 * self.cap
        self.calls = 0
        self.shared_gpu = False  # several ranks of the group on one GPU (a rehearsal)

    @classmethod
    def create(cls, comm: Comm, cap_elems: int) -> Optional["PeerReduce"]:
        h = hip()
        cap = int(cap_elems)
        handle = np.zeros(64, np.uint8)
        hnd, ok, err, shared = None, 1.0, None, False
        try:
            hnd = h.peer_create(comm.world, comm.rank, 8 * cap, handle.ctypes.data)
        except Exception as e:  # noqa: BLE001 -- any failure votes for RCCL
            ok = 0.0
            err = e
        # the device's identity travels with the handle: ranks sharing one GPU (a rehearsal of
        # the multi-GPU paths) run every exchange as ONE block. An exchange's blocks spin on
        # their peers' blocks; with several processes on one GPU the blocks of one rank's
        # exchange need not all be scheduled while the other ranks' spin (measured: 4 ranks x
        # 2.6M rows of leaf-wise growth deadlocked until the wait timeout with 32 blocks per
        # exchange, ran clean with 1 -- profiles/r4/s32_*, s33_*). One process per GPU has no
        # such coupling: a stream-ordered exchange owns the whole GPU (<= 256 blocks, one per CU).
        props = torch.cuda.get_device_properties(comm.device)
        ident = str(tuple(getattr(props, a, None) for a in ("uuid", "pci_domain_id", "pci_bus_id", "pci_device_id")))
        uuid = np.frombuffer(ident.encode()[:96].ljust(96), dtype=np.uint8)
        parts = comm.allgather_bytes(handle.tobytes() + uuid.tobytes())  # rank order, host group
        if ok:
            try:
                allh = np.frombuffer(b"".join(p[:64] for p in parts), dtype=np.uint8).copy()
                h.peer_open(hnd, allh.ctypes.data)
                shared = len({p[64:] for p in parts}) < comm.world
                if shared:  # several ranks on one GPU
                    h.peer_set_grid_cap(hnd, 1)
                if os.environ.get("YTK_PEER_GRID_CAP"):  # (diagnostics) blocks per exchange
                    h.peer_set_grid_cap(hnd, int(os.environ["YTK_PEER_GRID_CAP"]))
            except Exception as e:  # noqa: BLE001
                ok = 0.0
                err = e
        agreed = comm.allreduce_scalars([ok], op="min")[0] > 0.5
        if agreed:
            # self-test before any engine relies on the path: two exchanges of known int64 and
            # fp64 data under a short flag timeout (a path that cannot deliver -- e.g. peer
            # memory that is not coherent across these devices -- votes for RCCL instead of
            # producing wrong histograms or hanging the job)
            pr = cls(comm, hnd, cap)
            pr.shared_gpu = shared
            try:
                ok = 1.0 if pr._self_test() else 0.0
                if not ok:
                    err = RuntimeError("self-test exchange returned wrong sums")
            except Exception as e:  # noqa: BLE001
                ok, err = 0.0, e
            agreed = comm.allreduce_scalars([ok], op="min")[0] > 0.5
            if agreed:
                LAST_STATUS.update(state="ok", reason="")
                return pr
        if hnd is not None:
            torch.cuda.synchronize(comm.device)
            comm.barrier()
            h.peer_destroy(hnd)
        why = f"{type(err).__name__}: {err}" if err is not None else "another rank could not use its peers"
        LAST_STATUS.update(state="rccl", reason=why[:300])
        if comm.is_master:
            print(f"[ytk] peer-memory exchange unavailable ({why}); histogram messages use RCCL", flush=True)
        return None

    def _self_test(self) -> bool:
        P, r = self.comm.world, self.comm.rank
        saved = self.TIMEOUT_S
        self.TIMEOUT_S = min(saved, 10.0)
        stats = dict(self.comm.stats)  # the probe exchanges are not the job's traffic
        nlog = len(self.comm.log) if self.comm.log is not None else 0
        try:
            n = min(self.cap, 4099)  # odd: the single-element tail too (probes sized to the slab)
            t = torch.arange(n, dtype=torch.int64, device=self.comm.device) * P + r + 1
            f = torch.full((min(5, self.cap),), 0.5 * (r + 1), dtype=torch.float64, device=self.comm.device)
            g = torch.full((min(1025, 2 * self.cap),), 0.25 * (r + 1), dtype=torch.float32, device=self.comm.device)
            self.allreduce_(t)
            self.allreduce_(f)
            self.allreduce_(g)
            # reduce-scatter + all-gather of 2P int64 (one unit per segment) == the all-reduce
            rs = torch.arange(2 * P, dtype=torch.int64, device=self.comm.device) + 10 * r
            seg = self.fits_segments(rs)  # a slab smaller than 2P words: no segment probe
            if seg:
                self.reduce_scatter_(rs)
                self.allgather_(rs)
            torch.cuda.synchronize(self.comm.device)
            self.check()
            want = torch.arange(n, dtype=torch.int64, device=self.comm.device) * P * P + P * (P + 1) // 2
            want_rs = P * torch.arange(2 * P, dtype=torch.int64, device=self.comm.device) + 10 * P * (P - 1) // 2
            return (bool(torch.equal(t, want)) and bool(torch.all(f == 0.25 * P * (P + 1)))
                    and bool(torch.all(g == 0.125 * P * (P + 1))) and (not seg or bool(torch.equal(rs, want_rs))))
        finally:
            self.TIMEOUT_S = saved
            self.calls = 0
            self.comm.stats = stats
            if self.comm.log is not None:
                del self.comm.log[nlog:]

    def _account(self, t: torch.Tensor, n: int, skippable: bool = False):
        """Count an exchange. ``skippable`` ones (device skip word: leaf-wise batches a host
        queued past the tree's end are no-ops on the device) are not logged in the collective
        sequence -- hosts queue different numbers of them, and they pair up on the device."""
        self.calls += 1
        self.comm.last_op = ("peer_allreduce", str(t.dtype), int(n))
        if skippable:
            return
        self.comm.stats["calls"] += 1
        self.comm.stats["bytes"] += n * 8
        if self.comm.log is not None:
            self.comm.log.append(self.comm.last_op)

    def fits(self, t: torch.Tensor) -> bool:
        return (t.dtype in self._TYPES and t.is_contiguous() and t.is_cuda and t.data_ptr() % 16 == 0
                and t.numel() * t.element_size() <= self.cap_bytes)

    def allreduce_(self, t: torch.Tensor):
        """In-place sum over the ranks of a contiguous, 16-B aligned int64 / float64 / float32
        device tensor (one stream-ordered kernel; one-shot below YTK_PEER_TWO_SHOT_BYTES,
        two-shot reduce-scatter + all-gather above)."""
        assert self.fits(t), (t.dtype, t.numel(), t.data_ptr() % 16)
        n = t.numel()
        if fault_point("peer", self.calls, self.comm.rank):  # tests: an exchange this rank drops
            self.calls += 1
            return
        hip().peer_allreduce(self.hnd, ptr(t), n, self._TYPES[t.dtype], self.TIMEOUT_S, stream(t))
        self._account(t, n * t.element_size() // 8)

    def fits_segments(self, t: torch.Tensor) -> bool:
        """``t`` splits into P equal segments of whole 16-byte units (owner-computes sync)."""
        return self.fits(t) and (t.numel() * t.element_size()) % (16 * self.comm.world) == 0

    def reduce_scatter_(self, t: torch.Tensor) -> torch.Tensor:
        """Segment ``rank`` of ``t`` (P equal segments) <- its sum over the ranks, in place; the
        other segments keep this rank's values. Returns the reduced segment (a view). One
        kernel: the first half of the two-shot exchange."""
        assert self.fits_segments(t), (t.dtype, t.numel(), t.data_ptr() % 16)
        n = t.numel()
        hip().peer_reduce_scatter(self.hnd, ptr(t), n, self._TYPES[t.dtype], self.TIMEOUT_S, stream(t))
        self._account(t, n * t.element_size() // 8)
        seg = n // self.comm.world
        return t.view(-1)[self.comm.rank * seg:(self.comm.rank + 1) * seg]

    def allgather_(self, t: torch.Tensor, skip_dev: int = 0):
        """Every segment q of ``t`` (P equal segments) <- rank q's segment q, in place (each rank
        fills its own segment first). One kernel: the second half of the two-shot exchange.
        ``skip_dev`` (optional device word address): no exchange while it is non-zero."""
        assert self.fits_segments(t), (t.dtype, t.numel(), t.data_ptr() % 16)
        n = t.numel()
        hip().peer_allgather(self.hnd, ptr(t), n, self._TYPES[t.dtype], self.TIMEOUT_S, stream(t), skip_dev)
        self._account(t, n * t.element_size() // 8, skippable=skip_dev != 0)

    def reduce_scatter_dev_(self, x: torch.Tensor, seg_slot: int, nb_dev: int, k_dev: int, cur_stride: int,
                            skip_dev: int):
        """Reduce-scatter of the int64 message at ``x``: P equal segments of *nb_dev * seg_slot +
        *k_dev * cur_stride words, sized on the device (leaf-wise owner-computes batch); segment
        ``rank`` ends up reduced in place. Skipped while *skip_dev != 0. Counted with 0 bytes."""
        assert x.dtype == torch.int64 and x.is_cuda and x.data_ptr() % 16 == 0
        hip().peer_reduce_scatter_dev(self.hnd, ptr(x), seg_slot, nb_dev, k_dev, cur_stride, skip_dev, self.TIMEOUT_S,
                                      stream(x))
        self._account(x, 0, skippable=True)

    def allreduce_slots_(self, hist: torch.Tensor, slot_elems: int, ids: int, nb_dev: int, cursor: torch.Tensor,
                         k_dev: int, cur_stride: int, skip_dev: int):
        """Leaf-wise batch message counted on the device: the *nb_dev slots listed at ``ids``
        plus *k_dev x cur_stride cursor words (skipped while *skip_dev != 0). Its size is
        known only on the device: counted as a call with 0 bytes in ``comm.stats``."""
        hip().peer_allreduce_slots(self.hnd, ptr(hist), slot_elems, ids, nb_dev, ptr(cursor), k_dev, cur_stride,
                                   skip_dev, self.TIMEOUT_S, stream(hist))
        self._account(hist, 0, skippable=True)

    def timing(self):
        """(exchanges that ran, their summed device wall time in us) since the group was made
        (the self-test's five included; synchronous read -- diagnostics)."""
        out = np.zeros(2, np.float64)
        if self.hnd is not None:
            hip().peer_timing(self.hnd, out.ctypes.data)
        return int(out[0]), float(out[1])

    def check(self):
        v = hip().peer_check(self.hnd) if self.hnd is not None else 0
        if v == 1:
            raise RuntimeError(f"peer exchange: a flag wait timed out (a rank stopped issuing); rank {self.comm.rank}: "
                               f"{self.calls} exchanges issued, last completed epoch {hip().peer_epoch(self.hnd)}")
        if v:
            raise RuntimeError(f"peer exchange: device error {v} (message larger than the slab)")

    def abort(self):
        """Local, for a failing job: release every exchange of this rank that waits now or
        later (their results are void), so the device drains and the process can exit."""
        if self.hnd is not None:
            hip().peer_abort(self.hnd)

    def close(self):
        """Collective: every rank drains its device, then all free their blocks together (a
        peer may still be reading this rank's slab until it has drained)."""
        if self.hnd is None:
            return
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()
        hip().peer_destroy(self.hnd)
        self.hnd = None
