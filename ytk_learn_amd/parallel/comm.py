"""Communicator facade (replaces the reference's external ytk-mp4j ThreadCommSlave).

Reference call surface: allreduce / allreduceArray /
reduceScatterArray / allgatherArray / allreduceMap / allreduceRpc / barrier, plus
``info/error`` log shipping to a master (``J/utils/LogUtils.java:41-65``).

MI355X-native design: one process per GPU, ``torch.distributed`` with the
``nccl`` backend (= RCCL over xGMI on ROCm) for device tensors and ``gloo`` for
CPU tensors / host objects. A "worker" is a rank (the reference's
(process, thread) pairs collapse to GPUs). Map/object collectives go through
``all_gather_object`` and a caller-supplied merge (deterministic rank order).
With ``world_size == 1`` every collective is a no-op, so single-GPU runs pay
nothing.
"""
from __future__ import annotations

import datetime
import os
from typing import Any, Callable, List, Optional

import torch
import torch.distributed as dist

_OPS = {
    "sum": dist.ReduceOp.SUM,
    "max": dist.ReduceOp.MAX,
    "min": dist.ReduceOp.MIN,
}


class Comm:
    """Collective facade. ``Comm.local()`` is the single-worker instance."""

    def __init__(self, rank: int = 0, world: int = 1, device: Optional[torch.device] = None,
                 group=None, cpu_group=None):
        self.rank = rank
        self.world = world
        self.device = device if device is not None else torch.device("cpu")
        self.group = group
        self.cpu_group = cpu_group
        # YTK_FORCE_DIST=1 (set before from_env): a world-1 job still takes every
        # multi-rank code path and issues its collectives -- over RCCL on a GPU this runs the
        # real nccl-backend calls (work handles, reduce-scatter, all-gather) on one-GPU boxes
        self.force_dist = group is not None and world == 1
        # per-collective accounting (calls, payload bytes) for the bench / profile reports
        self.stats = {"calls": 0, "bytes": 0}
        # YTK_COMM_LOG=1: record every collective (op, dtype, numel) -- ranks must issue the
        # identical sequence (a mismatch is a hang under RCCL); checked by the tests
        self.log = [] if os.environ.get("YTK_COMM_LOG") == "1" else None
        self.last_op = None

    def _count(self, t: torch.Tensor, op: str = ""):
        self.stats["calls"] += 1
        self.stats["bytes"] += t.numel() * t.element_size()
        self.last_op = (op, str(t.dtype), int(t.numel()))  # named in timeout / failure reports
        if self.log is not None:
            self.log.append(self.last_op)

    def reset_stats(self):
        self.stats = {"calls": 0, "bytes": 0}

    # -- construction ---------------------------------------------------------
    @classmethod
    def local(cls, device=None) -> "Comm":
        return cls(0, 1, torch.device(device) if device is not None else None)

    @classmethod
    def from_env(cls, device: Optional[str] = None, timeout_s: int = 1800) -> "Comm":
        """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).

        device: "cuda", "cpu" or None (auto: cuda if available).
        """
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        # collective watchdog: a rank stuck longer than this in a collective aborts the job
        timeout_s = int(os.environ.get("YTK_COMM_TIMEOUT", timeout_s))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device == "cuda":
            idx = local_rank % max(1, torch.cuda.device_count())  # >1 rank per GPU only with gloo
            torch.cuda.set_device(idx)
            dev = torch.device("cuda", idx)
        else:
            dev = torch.device("cpu")
        force = os.environ.get("YTK_FORCE_DIST") == "1"
        if world <= 1 and not force:
            return cls(0, 1, dev)
        # YTK_DIST_BACKEND=gloo forces gloo even for GPU tensors: lets several ranks share ONE
        # GPU to rehearse the multi-GPU code paths (RCCL needs one GPU per rank).
        backend = os.environ.get("YTK_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            kw = {}
            if dev.type == "cuda" and backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        group = dist.group.WORLD
        cpu_group = group
        if dev.type == "cuda" and backend == "nccl":
            cpu_group = dist.new_group(backend="gloo")
        return cls(dist.get_rank(), dist.get_world_size(), dev, group, cpu_group)

    @property
    def is_dist(self) -> bool:
        return self.world > 1 or self.force_dist

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    # -- tensor collectives -----------------------------------------------------
    def allreduce_(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        """In-place allreduce (RCCL for device tensors, gloo for host tensors)."""
        if not self.is_dist:
            return None
        self._count(t, "allreduce_" + op)
        g = self.group if t.device.type == "cuda" else self.cpu_group
        return dist.all_reduce(t, op=_OPS[op], group=g, async_op=async_op)

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        t = t.clone()
        self.allreduce_(t, op)
        return t

    def allreduce_scalars(self, values, op: str = "sum", dtype=torch.float64) -> List[float]:
        """Batch several scalars into one collective (reference issues one each)."""
        t = torch.tensor(list(values), dtype=dtype)
        if self.is_dist:
            self._count(t, "allreduce_scalars_" + op)
            dist.all_reduce(t, op=_OPS[op], group=self.cpu_group)
        return t.tolist()

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        """out = this rank's 1/world block (dim 0) of the element-wise reduction of inp."""
        if not self.is_dist:
            out.copy_(inp.view_as(out) if inp.numel() == out.numel() else inp.reshape(-1)[: out.numel()].view_as(out))
            return
        self._count(inp, "reduce_scatter")
        g = self.group if inp.device.type == "cuda" else self.cpu_group
        # rank blocks stacked along dim 0 with out's trailing shape (gloo checks shapes)
        inp = inp.reshape((self.world * out.shape[0],) + tuple(out.shape[1:]))
        dist.reduce_scatter_tensor(out, inp, op=_OPS[op], group=g)

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate equal-size shards along dim 0."""
        if not self.is_dist:
            return t.clone()
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        self._count(t, "allgather")
        g = self.group if t.device.type == "cuda" else self.cpu_group
        dist.all_gather_into_tensor(out, t.contiguous(), group=g)
        return out

    def allgather_ragged(self, t: torch.Tensor) -> List[torch.Tensor]:
        """Every rank's ``t`` (dim 0 may differ per rank; trailing dims equal): one size
        all-gather + one padded all-gather (fixed-shape tensors, RCCL-friendly)."""
        if not self.is_dist:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        ns = self.allgather(n).tolist()
        m = max(ns)
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        allp = self.allgather(pad)
        return [allp[r * m: r * m + ns[r]] for r in range(self.world)]

    def broadcast_(self, t: torch.Tensor, src: int = 0):
        if not self.is_dist:
            return
        self._count(t, "broadcast")
        g = self.group if t.device.type == "cuda" else self.cpu_group
        dist.broadcast(t, src=src, group=g)

    def drain_pending(self):
        """Before a HIP graph capture: wait until the nccl process group's watchdog thread has
        retired every eager work handle. The watchdog keeps each eager collective until its
        next poll (~100 ms) and then queries the work's end event; a query the HIP runtime
        refuses because a capture is open ("operation not permitted when stream is
        capturing") throws in the watchdog thread and aborts the process with SIGABRT from
        ProcessGroupNCCL::Watchdog::run (reproduced in global capture mode by
        tools/probe_capture_watchdog.py; docs/performance.md, round 6). Collectives issued
        inside a capture are never handed to the watchdog, so after this drain it has nothing
        to query until the capture ends, whatever the capture mode."""
        if not self.is_dist or self.group is None:
            return
        try:
            if dist.get_backend(self.group) != "nccl":
                return
        except Exception:  # noqa: BLE001 -- no backend: nothing to drain
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.group._wait_for_pending_works()

    def barrier(self):
        if self.is_dist:
            self.last_op = ("barrier", "", 0)
            dist.barrier(group=self.cpu_group)

    # -- object collectives ---------------------------------------------------
    def allgather_object(self, obj: Any) -> List[Any]:
        if not self.is_dist:
            return [obj]
        out: List[Any] = [None] * self.world
        self.stats["calls"] += 1
        if self.log is not None:
            self.log.append(("allgather_object", "object", 0))
        dist.all_gather_object(out, obj, group=self.cpu_group)
        return out

    def allreduce_object(self, obj: Any, merge: Callable[[Any, Any], Any]) -> Any:
        """allreduceMap / allreduceRpc equivalent: fold objects in rank order."""
        objs = self.allgather_object(obj)
        acc = objs[0]
        for o in objs[1:]:
            acc = merge(acc, o)
        return acc

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.is_dist:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.cpu_group)
        return lst[0]

    # -- keyed merges (allreduceMap / allreduceMapSetUnion) ---------------------
    def _a2a_bytes(self, parts: List[bytes]) -> List[bytes]:
        """All-to-all of per-destination byte strings over the host group (uint8 tensors)."""
        P = self.world
        send_sizes = torch.tensor([len(b) for b in parts], dtype=torch.int64)
        recv_sizes = torch.empty(P, dtype=torch.int64)
        self.stats["calls"] += 2
        dist.all_to_all_single(recv_sizes, send_sizes, group=self.cpu_group)
        payload = b"".join(parts)
        inp = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if payload else torch.empty(0, dtype=torch.uint8)
        out = torch.empty(int(recv_sizes.sum()), dtype=torch.uint8)
        self.stats["bytes"] += len(payload)
        dist.all_to_all_single(out, inp, recv_sizes.tolist(), send_sizes.tolist(), group=self.cpu_group)
        res, off, raw = [], 0, out.numpy().tobytes()
        for n in recv_sizes.tolist():
            res.append(raw[off:off + n])
            off += n
        return res

    def merge_named(self, names: List[str], vals, ops: List[str]):
        """Global merge of per-name value rows -- the reference's allreduceMap over
        Map<String, T> (CoreData.java:628-632) -- with fixed-size tensor traffic instead of
        gathering every rank's whole map: names are hash-partitioned (crc32) to an owner
        rank (all-to-all), each owner reduces its share (column ops: "sum" | "max" |
        "min"), and the reduced rows are all-gathered once. Returns (sorted names,
        float64 [n, m] rows) identical on every rank."""
        import zlib

        import numpy as np

        vals = np.asarray(vals, dtype=np.float64).reshape(len(names), -1)
        m = vals.shape[1]

        def reduce(nm, vv):
            if not len(nm):
                return [], np.zeros((0, m))
            arr = np.asarray(nm, dtype=object)
            order = np.argsort(arr, kind="stable")
            arr, vv = arr[order], vv[order]
            start = np.flatnonzero(np.r_[True, arr[1:] != arr[:-1]])
            out = np.empty((len(start), m))
            for j, op in enumerate(ops):
                f = {"sum": np.add, "max": np.maximum, "min": np.minimum}[op]
                out[:, j] = f.reduceat(vv[:, j], start)
            return arr[start].tolist(), out

        if not self.is_dist:
            return reduce(names, vals)
        P = self.world
        enc = [n.encode("utf-8") for n in names]
        owner = np.fromiter((zlib.crc32(b) % P for b in enc), dtype=np.int64, count=len(enc))
        parts = []
        for o in range(P):
            idx = np.flatnonzero(owner == o)
            blob = b"\n".join(enc[i] for i in idx)
            head = np.array([len(idx), len(blob)], np.int64).tobytes()
            parts.append(head + blob + vals[idx].tobytes())
        got_names, got_vals = [], []
        for raw in self._a2a_bytes(parts):
            k, nb = np.frombuffer(raw[:16], np.int64)
            if k:
                got_names += raw[16:16 + nb].decode("utf-8").split("\n")
                got_vals.append(np.frombuffer(raw[16 + nb:], np.float64).reshape(int(k), m))
        mine_n, mine_v = reduce(got_names, np.concatenate(got_vals) if got_vals else np.zeros((0, m)))
        blob = "\n".join(mine_n).encode("utf-8")
        head = np.array([len(mine_n), len(blob)], np.int64).tobytes()
        allp = self.allgather_bytes(head + blob + np.asarray(mine_v, np.float64).tobytes())
        out_n, out_v = [], []
        for raw in allp:
            k, nb = np.frombuffer(raw[:16], np.int64)
            if k:
                out_n += raw[16:16 + nb].decode("utf-8").split("\n")
                out_v.append(np.frombuffer(raw[16 + nb:], np.float64).reshape(int(k), m))
        if not out_n:
            return [], np.zeros((0, m))
        arr = np.asarray(out_n, dtype=object)
        order = np.argsort(arr, kind="stable")
        return arr[order].tolist(), np.concatenate(out_v)[order]

    def allgather_bytes(self, b: bytes) -> List[bytes]:
        """Variable-size byte strings from every rank (two fixed-shape tensor all-gathers)."""
        if not self.is_dist:
            return [b]
        n = torch.tensor([len(b)], dtype=torch.int64)
        ns = torch.empty(self.world, dtype=torch.int64)
        self.stats["calls"] += 2
        dist.all_gather_into_tensor(ns, n, group=self.cpu_group)
        mx = int(ns.max())
        buf = torch.zeros(mx, dtype=torch.uint8)
        if b:
            buf[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        out = torch.empty(self.world * mx, dtype=torch.uint8)
        self.stats["bytes"] += mx
        dist.all_gather_into_tensor(out, buf, group=self.cpu_group)
        raw = out.numpy().tobytes()
        return [raw[r * mx:r * mx + int(ns[r])] for r in range(self.world)]

    # -- even partition helper (CommUtils.createThreadArrayFroms/Tos) ---------
    def feature_blocks(self, F: int):
        """Owner-computes feature partition: rank r owns [r * Fr, min(F, (r + 1) * Fr)) with
        Fr = ceil(F / world) (GBDTDataFlow.java:252-272 assigns contiguous column ranges)."""
        fr = -(-F // self.world)
        return fr, [(min(F, r * fr), min(F, (r + 1) * fr)) for r in range(self.world)]

    def shard_range(self, dim: int, rank: Optional[int] = None):
        r = self.rank if rank is None else rank
        base, rem = divmod(dim, self.world)
        start = r * base + min(r, rem)
        return start, start + base + (1 if r < rem else 0)

    def close(self):
        if self.is_dist and dist.is_initialized():
            dist.destroy_process_group()
