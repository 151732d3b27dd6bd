"""Data-parallel histogram tree builder (level-wise and loss-guided growth).

Reference behaviour: ``J/optimizer/gbdt/DataParallelTreeMaker.java`` (make() :229-295,
expansion conditions :249-273, smaller-child histogram + subtraction :489-508,
node stats :543-573, split enumeration :598-637, best-split sync :640-653) and
``J/optimizer/gbdt/UpdateStrategy.java``.

MI355X-first structure (not a translation):
  * all per-row state (row-major + column-major bins, position-ordered (g,h), row
    permutation) stays resident in HBM;
  * one batched launch per level for histogram build / split search / partition
    (level-wise); loss-guided growth uses the same kernels with batch size 1;
  * the partition moves (g,h) along with the row ids, so histogram builds read
    (g,h) contiguously and only gather the 32-B bin rows;
  * level-wise histograms are indexed by a per-tree slot counter (even 509 slots x
    28 features x 256 bins is 29 MB of the 288 GB HBM); loss-guided growth recycles
    slots from a free list, bounded like the reference's LRU pool when
    ``histogram_pool_capacity`` is set;
  * per-call metadata (work lists, split items) is built with vectorised numpy and
    shipped in ONE pinned host->device copy per launch group;
  * multi-GPU: rows are sharded; the level's freshly built histograms are one
    contiguous slab -> ONE RCCL all-reduce per level. Every rank then runs the
    same split kernel on identical inputs, so split decisions agree without a
    SplitInfo exchange.
"""
from __future__ import annotations

import heapq
import os
import time
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from ...ops import gbdt as gops
from ...ops._ext import hip, hist_cols, stream
from ...parallel.comm import Comm
from .tree import Tree


@dataclass
class TreeParams:
    max_depth: int = 6
    max_leaf_cnt: int = 64
    min_child_hessian_sum: float = 1e-8
    max_abs_leaf_val: float = -1.0
    min_split_loss: float = 0.0
    min_split_samples: int = -1
    learning_rate: float = 0.1
    l1: float = 0.0
    l2: float = 0.0
    grow_policy: str = "level"  # "level" | "loss"
    instance_sample_rate: float = 1.0
    feature_sample_rate: float = 1.0
    seed: int = 2018
    # multi-GPU histogram synchronisation: "allreduce" (every rank gets every global
    # histogram and searches all features), "owner" (reduce-scatter by feature block,
    # owner-computes split search, allgather of 48-B split records + deterministic argmax:
    # HistogramBuilder.java:95, DataParallelTreeMaker.java:575-653) or "auto" (owner when
    # a level's histogram slab is large, where halving the bytes pays for the extra
    # small collective)
    hist_sync: str = "auto"

    def gain_params(self):
        f = lambda v: float(np.float32(v))  # kernel receives float32 params
        return {"mcw": f(self.min_child_hessian_sum), "l1": f(self.l1), "l2": f(self.l2),
                "max_abs_leaf": f(self.max_abs_leaf_val)}


OWNER_MIN_SLOT_BYTES = 1 << 20  # "auto": owner-computes once one node histogram is >= 1 MiB


def resolve_hist_sync(mode: str, slot_bytes: int) -> str:
    """Effective multi-GPU histogram sync mode (env YTK_HIST_SYNC overrides the config)."""
    mode = os.environ.get("YTK_HIST_SYNC", mode or "auto").lower()
    if mode == "auto":
        return "owner" if slot_bytes >= OWNER_MIN_SLOT_BYTES else "allreduce"
    if mode not in ("allreduce", "owner"):
        raise ValueError(f"hist_sync must be auto, allreduce or owner, got {mode!r}")
    return mode


@dataclass
class TimeStats:
    """Per-phase timers mirroring ``J/data/gbdt/TimeStats.java`` (host wall time;
    with ``profile=True`` each phase synchronises so device time is attributed)."""
    build_hist: float = 0.0
    comm_hist: float = 0.0
    find_split: float = 0.0
    partition: float = 0.0
    plan: float = 0.0  # host-side expansion planning (leaf-wise replay)
    total: float = 0.0
    trees: int = 0

    def add(self, o: "TimeStats"):
        for k in ("build_hist", "comm_hist", "find_split", "partition", "plan", "total"):
            setattr(self, k, getattr(self, k) + getattr(o, k))
        self.trees += o.trees

    def stats(self) -> str:
        return (f"[time stats] trees={self.trees} total={self.total:.4f}s build_hist={self.build_hist:.4f}s "
                f"comm_hist={self.comm_hist:.4f}s find_split={self.find_split:.4f}s "
                f"partition={self.partition:.4f}s plan={self.plan:.4f}s")


@dataclass
class _Node:
    begin: int = 0
    cnt_local: int = 0
    cnt_global: int = 0
    slot: int = -1
    depth: int = 0
    seq: int = 0
    rec: Optional[np.void] = None
    G: float = 0.0
    H: float = 0.0
    children: Optional[tuple] = None  # (left, right) ids once expanded (loss-guided)
    rec_used: bool = True             # False: leafified child -> dump lossChg = -inf


class _Uploader:
    """Packs small int32 host arrays into one pinned buffer -> one H2D copy.

    Safe to reuse after every device->host sync (each tree level has one)."""

    def __init__(self, dev: torch.device, cap: int = 1 << 20):
        self.dev = dev
        self.cuda = dev.type == "cuda"
        self.cap = cap
        if self.cuda:
            self.host = torch.empty(cap, dtype=torch.int32, pin_memory=True)
            self.devbuf = torch.empty(cap, dtype=torch.int32, device=dev)
        self.off = 0

    def reset(self):
        self.off = 0

    def put(self, *arrays: np.ndarray):
        arrays = [np.ascontiguousarray(a, dtype=np.int32) for a in arrays]
        if not self.cuda:
            return [torch.from_numpy(a) for a in arrays]
        n = sum(a.size for a in arrays)
        if self.off + n > self.cap:
            torch.cuda.current_stream(self.dev).synchronize()
            self.off = 0
            if n > self.cap:
                self.cap = 1 << int(np.ceil(np.log2(n)))
                self.host = torch.empty(self.cap, dtype=torch.int32, pin_memory=True)
                self.devbuf = torch.empty(self.cap, dtype=torch.int32, device=self.dev)
        o = self.off
        hv = self.host.numpy()
        outs = []
        p = o
        for a in arrays:
            hv[p:p + a.size] = a.reshape(-1)
            outs.append((p, a.shape))
            p += a.size
        self.devbuf[o:p].copy_(self.host[o:p], non_blocking=True)
        self.off = p
        return [self.devbuf[s:s + int(np.prod(shape))].view(*shape) for s, shape in outs]


def _put_flat(up: "_Uploader", a: np.ndarray) -> int:
    """One int32 array -> the uploader's device buffer; returns its device address."""
    t, = up.put(a)
    return t.data_ptr()


def _chunk_segments(begins: np.ndarray, counts: np.ndarray, ch: int):
    """Vectorised chunking of segments -> (seg_idx, chunk_begin, chunk_end, blk_in_seg)."""
    nb = np.where(counts > 0, (counts + ch - 1) // ch, 0).astype(np.int64)
    total = int(nb.sum())
    seg = np.repeat(np.arange(len(counts)), nb)
    first = np.concatenate([[0], np.cumsum(nb)[:-1]]) if len(nb) else np.zeros(0, np.int64)
    k = np.arange(total) - np.repeat(first, nb)
    s = begins[seg] + k * ch
    e = np.minimum(s + ch, (begins + counts)[seg])
    return seg, s, e, k, first, nb


class TreeBuilder:
    MIN_ROWS_PER_BLOCK = 2048
    TARGET_BLOCKS = 256  # histogram blocks per launch: one 128-KiB-LDS block per CU

    def __init__(self, bins: torch.Tensor, binsT: torch.Tensor, F: int, B: int, nbins_f: np.ndarray,
                 params: TreeParams, comm: Optional[Comm] = None, profile: bool = False,
                 pool_mb: float = -1.0):
        self.bins = bins
        self.binsT = binsT
        self.dev = bins.device
        self.N = bins.shape[0]
        self.F = F
        self.B = B
        self.p = params
        self.comm = comm or Comm.local(self.dev)
        self.nbins_f_np = np.asarray(nbins_f, np.int32)
        self.nbins_f = torch.from_numpy(self.nbins_f_np).to(self.dev)
        self.gp = params.gain_params()
        ml = params.max_leaf_cnt if params.max_leaf_cnt > 0 else (1 << 30)
        if params.max_depth >= 0:
            max_nodes = min((1 << (params.max_depth + 1)) - 1, 2 * ml - 1)
        else:
            max_nodes = 2 * ml - 1
        self.max_nodes = int(max_nodes)
        # Loss-guided growth expands speculative batches (see build()): every real split
        # uses two slots, and up to `spec_waste` further expansions may be discarded.
        n_slots = self.max_nodes
        self.spec_waste = 0
        if params.grow_policy == "loss" and params.max_leaf_cnt > 0:
            slot_bytes = B * F * 16
            self.spec_waste = int(min(params.max_leaf_cnt, max(0, (4 << 30) // max(1, 2 * slot_bytes))))
            n_slots += 2 * self.spec_waste
        # histogram_pool_capacity (MB, <= 0: unlimited; reference HistogramPool.java:36-273,
        # DataParallelTreeMaker.java:192-204,489-508): bounds the live histogram slots of
        # loss-guided growth. When the pool is full the least recently built histogram is
        # evicted; expanding an evicted node then builds BOTH children (a pool miss)
        # instead of deriving the larger one by subtraction.
        self.slot_bytes = B * F * 16
        if pool_mb is not None and pool_mb > 0 and params.grow_policy == "loss":
            n_slots = int(min(n_slots, max(3, (pool_mb * (1 << 20)) // self.slot_bytes)))
        self.n_slots = n_slots
        self.hist_miss = 0
        # YTK_LOSSGUIDE_SPEC=0: expand one leaf per step (the plain sequential schedule;
        # used by the tests to check that speculation does not change the tree)
        self.speculate = os.environ.get("YTK_LOSSGUIDE_SPEC", "1") != "0"
        # YTK_LEAF_NATIVE=0: the Python planner (_grow_loss_guided) instead of the native one
        self.native_leafwise = os.environ.get("YTK_LEAF_NATIVE", "1") != "0"
        # exact int64 fixed-point histograms (see csrc/hip/gbdt_hist.hip)
        self.hist = torch.zeros((self.n_slots, B, F, 2), dtype=torch.int64, device=self.dev)
        self.gp_tree = dict(self.gp, sg=1.0, sh=1.0)
        self.rows = torch.empty(self.N, dtype=torch.int32, device=self.dev)
        self.rows_tmp = torch.empty(self.N, dtype=torch.int32, device=self.dev)
        self.ghp = torch.empty((self.N, 2), dtype=torch.float32, device=self.dev)
        self.gh_tmp = torch.empty((self.N, 2), dtype=torch.float32, device=self.dev)
        self.flags = torch.empty(self.N, dtype=torch.uint8, device=self.dev)
        self.iota = torch.arange(self.N, dtype=torch.int32, device=self.dev)
        self.up = _Uploader(self.dev)
        self.profile = profile
        self.last_stats = TimeStats()
        self.total_stats = TimeStats()
        self.tree_count = 0
        self.last_keep = None
        self._root_gh = None
        self._staging = None
        self._cursor = None
        self._split_out = None
        self.free_slots = None
        self.part_atomic = os.environ.get("YTK_PART_ATOMIC", "1") != "0"
        self.fmask_np = np.ones(F, np.uint8)
        # owner-computes histogram sync (multi-GPU): see TreeParams.hist_sync
        self.owner = self.comm.is_dist and resolve_hist_sync(params.hist_sync, self.slot_bytes) == "owner"
        if self.owner:
            self.fr, self.fblocks = self.comm.feature_blocks(F)
            self.own = self.fblocks[self.comm.rank]
            self._own_masks = {}

    # ------------------------------------------------------------------ utils
    def _sync(self):
        if self.profile and self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def _chunk(self, total: int) -> int:
        return max(self.MIN_ROWS_PER_BLOCK, -(-total // self.TARGET_BLOCKS))

    # ----------------------------------------------------------- primitives
    def _build_and_find(self, nodes: Dict[int, _Node], build: List[int], derived: List[tuple],
                        fmask: torch.Tensor, f0: int, identity_rows: bool = False):
        """Histogram the ``build`` nodes, derive ``derived`` = (node, parent, sibling),
        then find the best split of every one of them."""
        nb = len(build)
        if self.free_slots is not None:  # recycled pool (loss-guided): any free slots
            need = nb + len(derived)
            keep = {p for _, p, _ in derived}
            while len(self.free_slots) < need:
                self._evict(nodes, keep)
            ids = [self.free_slots.pop() for _ in range(need)]
            for nid, sl in zip(list(build) + [n for n, _, _ in derived], ids):
                self.lru[nid] = sl
            s0 = -1
        else:  # one contiguous range per call
            s0 = self.next_slot
            ids = list(range(s0, s0 + nb + len(derived)))
            self.next_slot += nb + len(derived)
        for i, nid in enumerate(build):
            nodes[nid].slot = ids[i]
        for j, (nid, _, _) in enumerate(derived):
            nodes[nid].slot = ids[nb + j]
        items = np.zeros((nb + len(derived), 4), np.int32)
        items[:nb, 0] = ids[:nb]
        for j, (n, p, s) in enumerate(derived):
            items[nb + j] = (nodes[n].slot, nodes[p].slot, nodes[s].slot, 1)
        begins = np.array([nodes[n].begin for n in build], np.int64)
        counts = np.array([nodes[n].cnt_local for n in build], np.int64)
        recs = self._hist_split(begins, counts, np.asarray(ids, np.int32), nb, items, fmask, f0,
                                identity_rows=identity_rows, s0=s0)
        mcw2 = self.p.min_child_hessian_sum * 2.0
        names = gops.SPLIT_DTYPE.names
        order = list(build) + [n for n, _, _ in derived]
        # plain dicts of Python scalars: the host bookkeeping then avoids numpy scalar ops
        for nid, tup in zip(order, recs.tolist()):
            r = dict(zip(names, tup))  # loss_chg: the exact double of the float32 gain
            nd = nodes[nid]
            nd.rec = r
            nd.G = r["g"]
            nd.H = r["h"]
            # canSplit (UpdateStrategy.canSplit): H >= 2*mcw and n >= min_split_samples
            if not (nd.H >= mcw2 and nd.cnt_global >= self.p.min_split_samples):
                r["loss_chg"] = -np.inf
                r["feat"] = -1

    def _hist_split(self, begins: np.ndarray, counts: np.ndarray, ids: np.ndarray, nb: int, items: np.ndarray,
                    fmask: torch.Tensor, f0: int, identity_rows: bool = False, s0: int = -1) -> np.ndarray:
        """Device part of a histogram + split step: build the nb nodes' histograms
        (segments begins/counts -> slots ids[:nb]; s0 >= 0: the contiguous range s0..),
        all-reduce them, run the split search over ``items`` [n, 4]; returns the split
        records (host structured array, SPLIT_DTYPE)."""
        st = self.last_stats
        t0 = time.perf_counter()
        work = np.zeros((0, 4), np.int32)
        if nb:
            seg, s, e, _, _, _ = _chunk_segments(begins, counts, self._chunk(int(counts.sum())))
            work = np.zeros((len(seg), 4), np.int32)
            work[:, 0] = ids[:nb][seg]
            work[:, 1] = s
            work[:, 2] = e
        work_d, items_d, ids_d = self.up.put(work, items, ids[:nb])
        if nb:
            if s0 >= 0:
                self.hist[s0:s0 + nb].zero_()
            elif self.dev.type == "cuda":  # one launch, no id conversion
                hip().zero_slots(self.hist.data_ptr(), self.slot_bytes, ids_d.data_ptr(), nb, stream(self.hist))
            else:
                self.hist.index_fill_(0, ids_d.long(), 0)
            src_gh = self._root_gh if (identity_rows and self._root_gh is not None) else self.ghp
            staging = None
            if (self.dev.type == "cuda" and os.environ.get("YTK_HOST_STAGED", "1") != "0"
                    and self.bins.dtype == torch.uint8 and self.B <= 256):
                need = len(work) * ((self.F + 31) // 32) * self.B * 64
                if self._staging is None or self._staging.numel() < need:
                    self._staging = torch.empty(int(need * 1.25), dtype=torch.int64, device=self.dev)
                staging = self._staging
            gops.hist_build(self.bins, self.F, src_gh, None if identity_rows else self.rows,
                            work_d, self.hist, self.B, self.gp_tree["sg"], self.gp_tree["sh"],
                            staging=staging, slot_base=max(s0, 0), nslots=nb,
                            slot_ids=ids_d if s0 < 0 else None, binsT=self.binsT)
        self._sync()
        t1 = time.perf_counter()
        if nb and self.comm.is_dist:
            if self.owner:
                idx = (torch.arange(s0, s0 + nb, device=self.dev) if s0 >= 0 else ids_d.long())
                self._owner_reduce(idx)
            elif s0 >= 0:
                self.comm.allreduce_(self.hist[s0:s0 + nb])
            else:  # gather the scattered slots into one buffer -> one all-reduce
                idx = ids_d.long()
                buf = self.hist.index_select(0, idx)
                self.comm.allreduce_(buf)
                self.hist.index_copy_(0, idx, buf)
            self._sync()
        t2 = time.perf_counter()
        if self.owner:
            fm_own, f0_own = self._owner_mask(f0)
            out = gops.split_find(self.hist, self.B, self.F, self.nbins_f, fm_own, f0_own, items_d, self.gp_tree)
            recs = self._owner_combine(out)
        else:
            out = gops.split_find(self.hist, self.B, self.F, self.nbins_f, fmask, f0, items_d, self.gp_tree)
            recs = out.cpu().numpy().view(gops.SPLIT_DTYPE).reshape(-1)
        self.up.reset()  # the .cpu() above synchronised the stream
        t3 = time.perf_counter()
        st.build_hist += t1 - t0
        st.comm_hist += t2 - t1
        st.find_split += t3 - t2
        return recs

    # ------------------------------------------------ owner-computes histogram sync
    def _owner_reduce(self, idx: torch.Tensor):
        """Reduce-scatter the built slots ``idx`` by feature block: afterwards this rank
        holds the GLOBAL sums of its own features [lo, hi) (HistogramBuilder.java:95);
        the other feature columns keep local partials and are never read."""
        P, fr = self.comm.world, self.fr
        nb = int(idx.numel())
        buf = self.hist.index_select(0, idx)  # [nb, B, F, 2]
        if P * fr != self.F:
            pad = torch.zeros((nb, self.B, P * fr - self.F, 2), dtype=buf.dtype, device=buf.device)
            x = torch.cat([buf, pad], dim=2)
        else:
            x = buf
        x = x.reshape(nb, self.B, P, fr, 2).permute(2, 0, 1, 3, 4).contiguous()
        out = torch.empty((nb, self.B, fr, 2), dtype=buf.dtype, device=buf.device)
        self.comm.reduce_scatter_(out, x)
        lo, hi = self.own
        if hi > lo:
            buf[:, :, lo:hi] = out[:, :, :hi - lo]
        self.hist.index_copy_(0, idx, buf)

    def _owner_mask(self, f0: int):
        """(device fmask of the sampled features this rank owns, node-total feature).
        A rank owning no sampled feature searches nothing; its totals are ignored."""
        lo, hi = self.own
        fm = self.fmask_np.copy()
        fm[:lo] = 0
        fm[hi:] = 0
        key = fm.tobytes()
        if key not in self._own_masks:
            if len(self._own_masks) > 64:
                self._own_masks.clear()
            self._own_masks[key] = torch.from_numpy(fm).to(self.dev)
        nz = np.flatnonzero(fm)
        return self._own_masks[key], (int(nz[0]) if nz.size else (lo if hi > lo else 0))

    def _owner_combine(self, out: torch.Tensor) -> np.ndarray:
        """Allgather the per-rank best splits (48-B records) and take the global argmax with
        the reference tie-break (SplitInfo.needReplace: larger lossChg, then lower feature,
        then lower bin) -- the same total order the split kernels use, so the result is
        bitwise the all-reduce mode's record. Node totals come from the first rank owning
        a sampled feature (exact int64 sums: every feature's total is the same)."""
        n = out.shape[0]
        allr = self.comm.allgather(out.contiguous().view(n, 48))
        recs = allr.cpu().numpy().view(gops.SPLIT_DTYPE).reshape(self.comm.world, n)
        big = np.int64(0x7fffffff)
        best = recs[0].copy()
        for r in range(1, self.comm.world):
            c = recs[r]
            cf = np.where(c["feat"] < 0, big, c["feat"])
            bf = np.where(best["feat"] < 0, big, best["feat"])
            cb = np.where(c["bin_b"] < 0, big, c["bin_b"])
            bb = np.where(best["bin_b"] < 0, big, best["bin_b"])
            rep = ((c["loss_chg"] > best["loss_chg"])
                   | ((c["loss_chg"] == best["loss_chg"]) & ((cf < bf) | ((cf == bf) & (cb < bb)))))
            best[rep] = c[rep]
        for r, (lo, hi) in enumerate(self.fblocks):
            if hi > lo and self.fmask_np[lo:hi].any():
                best["g"] = recs[r]["g"]
                best["h"] = recs[r]["h"]
                break
        return best

    def _evict(self, nodes: Dict[int, _Node], keep):
        """Drop the least recently built histogram not needed by the current call."""
        for sid in list(self.lru):
            if sid in keep:
                continue
            sl = self.lru.pop(sid)
            nodes[sid].slot = -1
            self.free_slots.append(sl)
            return
        raise RuntimeError("histogram_pool_capacity too small for one expansion")

    def _split_arrays(self, nodes: Dict[int, _Node], splits: List[tuple]):
        begins = np.array([nodes[s[0]].begin for s in splits], np.int64)
        counts = np.array([nodes[s[0]].cnt_local for s in splits], np.int64)
        feat = np.array([int(nodes[x[0]].rec["feat"]) for x in splits], np.int32)
        thr = np.array([(int(nodes[x[0]].rec["bin_a"]) + int(nodes[x[0]].rec["bin_b"])) // 2 for x in splits],
                       np.int32)
        return begins, counts, feat, thr

    def _partition(self, nodes: Dict[int, _Node], splits: List[tuple], copy_back: bool):
        """splits: list of (nid, left_child, right_child). Updates child segments/counts."""
        lloc, lglob = self._partition_arrays(*self._split_arrays(nodes, splits), copy_back)
        lloc, lglob = lloc.tolist(), lglob.tolist()
        for i, (nid, lc, rc) in enumerate(splits):
            nd = nodes[nid]
            nodes[lc] = _Node(begin=nd.begin, cnt_local=lloc[i], cnt_global=lglob[i], depth=nd.depth + 1)
            nodes[rc] = _Node(begin=nd.begin + lloc[i], cnt_local=nd.cnt_local - lloc[i],
                              cnt_global=nd.cnt_global - lglob[i], depth=nd.depth + 1)

    def _partition_arrays(self, begins: np.ndarray, counts: np.ndarray, feat: np.ndarray, thr: np.ndarray,
                          copy_back: bool):
        """Partition the segments (begins, counts) by bin(feat) <= thr; returns the left
        row counts (local, global) as int64 arrays."""
        t0 = time.perf_counter()
        n = len(begins)
        seg, s, e, k, first, nblk = _chunk_segments(begins, counts, self._chunk(int(counts.sum())))
        items = np.stack([seg, s, e, k], axis=1).astype(np.int32).reshape(-1, 4)
        root = self._root_gh is not None  # first partition of an unsampled tree: identity rows
        rows_in, gh_in = (None, self._root_gh) if root else (self.rows, self.ghp)
        if self.dev.type == "cuda" and self.part_atomic:
            # single-pass partition: 2048-row chunks mapped from an exclusive block scan
            nb_a = (counts + gops.PART_CHUNK - 1) // gops.PART_CHUNK
            first_a = np.concatenate([[0], np.cumsum(nb_a)[:-1]]) if n else np.zeros(0, np.int64)
            hdr = np.array([n, int(nb_a.sum())], np.int32)
            items_d, feat_d, thr_d, nbeg_d, cnt_d, first_d, hdr_d = self.up.put(
                items, feat, thr, begins, counts, first_a, hdr)
            if self._cursor is None or self._cursor.numel() < n:
                self._cursor = torch.empty(max(n, 1024), dtype=torch.int64, device=self.dev)
            # raw split cursors (right << 32 | left): masked on the host after the copy
            left = gops.partition_atomic(self.binsT, rows_in, self.rows_tmp, gh_in, self.gh_tmp, first_d,
                                         hdr_d, int(hdr[1]), feat_d, thr_d, nbeg_d, cnt_d, cursor=self._cursor)
        else:
            items_d, feat_d, thr_d, nbeg_d, first_d, nblk_d = self.up.put(
                items, feat, thr, begins, first, nblk)
            left = gops.partition(self.binsT, rows_in, self.rows_tmp, gh_in, self.gh_tmp, self.flags,
                                  items_d, feat_d, thr_d, nbeg_d, first_d, nblk_d, n)
        if root:  # the root segment is every row: take the output buffers whole
            copy_back = False
            self._root_gh = None
        if copy_back:  # only these segments were partitioned: copy them back in one launch
            gops.segment_copy(items_d, self.rows_tmp, self.rows, self.gh_tmp, self.ghp)
        else:
            self.rows, self.rows_tmp = self.rows_tmp, self.rows
            self.ghp, self.gh_tmp = self.gh_tmp, self.ghp
        if self.comm.is_dist:
            both = torch.stack([left, left]).to(torch.int64) & 0xFFFFFFFF
            self.comm.allreduce_(both[1])
            both = both.cpu().numpy()
            lloc, lglob = both[0], both[1]
        else:
            lloc = left.to(torch.int64).cpu().numpy() & 0xFFFFFFFF
            lglob = lloc
        self.up.reset()
        self.last_stats.partition += time.perf_counter() - t0
        return lloc, lglob

    def _count_children(self, nodes: Dict[int, _Node], splits: List[tuple]):
        """Children that become leaves right away: only their sample counts are needed
        (node statistics in the dump), so run the flag/count pass without the scatter."""
        lloc, lglob = self._count_arrays(*self._split_arrays(nodes, splits))
        lloc, lglob = lloc.tolist(), lglob.tolist()
        for i, (nid, lc, rc) in enumerate(splits):
            nd = nodes[nid]
            nodes[lc] = _Node(cnt_local=lloc[i], cnt_global=lglob[i], depth=nd.depth + 1)
            nodes[rc] = _Node(cnt_local=nd.cnt_local - lloc[i],
                              cnt_global=nd.cnt_global - lglob[i], depth=nd.depth + 1)

    def _count_arrays(self, begins: np.ndarray, counts: np.ndarray, feat: np.ndarray, thr: np.ndarray):
        """Left row counts (local, global) of the segments without moving rows."""
        t0 = time.perf_counter()
        seg, s, e, k, first, nblk = _chunk_segments(begins, counts, self._chunk(int(counts.sum())))
        items = np.stack([seg, s, e, k], axis=1).astype(np.int32).reshape(-1, 4)
        items_d, feat_d, thr_d = self.up.put(items, feat, thr)
        bc = gops.partition_count(self.binsT, None if self._root_gh is not None else self.rows, self.flags,
                                  items_d, feat_d, thr_d)
        left = torch.zeros(len(begins), dtype=torch.int64, device=self.dev)
        if len(seg):
            left.index_add_(0, torch.from_numpy(seg).to(self.dev), bc.to(torch.int64))
        if self.comm.is_dist:
            both = torch.stack([left, left])
            self.comm.allreduce_(both[1])
            both = both.cpu().numpy()
            lloc, lglob = both[0], both[1]
        else:
            lloc = left.cpu().numpy()
            lglob = lloc
        self.up.reset()
        self.last_stats.partition += time.perf_counter() - t0
        return lloc, lglob

    # ------------------------------------------------------- loss-guided growth
    def _fast_leafwise_ok(self) -> bool:
        """Lean launch path for the native planner: single-pass partition, staged uint8
        histograms and the node-resident split kernel (what the packs encode)."""
        stride = self.bins.shape[1]
        return (self.dev.type == "cuda" and self.part_atomic
                and self.bins.dtype == torch.uint8 and self.binsT.dtype == torch.uint8 and self.B <= 256
                and stride % 32 == 0 and stride >= ((self.F + 31) // 32) * 32
                and gops.split_node_fits(self.B, self.F)
                and os.environ.get("YTK_HOST_STAGED", "1") != "0"
                and os.environ.get("YTK_LEAF_FAST", "1") != "0")

    def _fast_partition(self, g, splits):
        """Partition of the batch's split segments from one native pack (one upload, raw
        kernel launches); returns the left row counts (local, global)."""
        t0 = time.perf_counter()
        h, s = hip(), stream(self.rows)
        arr, off, nitems, nblocks = g.pack_partition(splits, gops.PART_CHUNK, self.TARGET_BLOCKS,
                                                     self.MIN_ROWS_PER_BLOCK)
        base = _put_flat(self.up, arr)
        a = lambda i: base + 4 * off[i]  # noqa: E731
        n = len(splits)
        if self._cursor is None or self._cursor.numel() < n:
            self._cursor = torch.empty(max(n, 1024), dtype=torch.int64, device=self.dev)
        cur = self._cursor.data_ptr()
        h.memset_async(cur, 0, n * 8, s)
        root = self._root_gh is not None  # first partition of an unsampled tree: identity rows
        rows_in = 0 if root else self.rows.data_ptr()
        gh_in = (self._root_gh if root else self.ghp).data_ptr()
        if nblocks > 0:
            h.partition_atomic(self.binsT.data_ptr(), 1, self.binsT.shape[1], rows_in, self.rows_tmp.data_ptr(),
                               gh_in, self.gh_tmp.data_ptr(), a(5), a(6), a(6) + 4, int(nblocks), a(1), a(2),
                               a(3), a(4), cur, 0, 0, s)
        if root:  # the root segment is every row: take the output buffers whole
            self._root_gh = None
            self.rows, self.rows_tmp = self.rows_tmp, self.rows
            self.ghp, self.gh_tmp = self.gh_tmp, self.ghp
        elif nitems > 0:
            h.segment_copy(a(0), int(nitems), self.rows_tmp.data_ptr(), self.rows.data_ptr(),
                           self.gh_tmp.data_ptr(), self.ghp.data_ptr(), s)
        if self.comm.is_dist:  # global counts: one all-reduce of the masked cursors
            both = (self._cursor[:n] & 0xFFFFFFFF).repeat(2, 1)
            self.comm.allreduce_(both[1])
            both = both.cpu().numpy()
            lloc, lglob = both[0], both[1]
        else:
            lloc = self._cursor[:n].cpu().numpy() & 0xFFFFFFFF
            lglob = lloc
        self.up.reset()
        self.last_stats.partition += time.perf_counter() - t0
        return lloc, lglob

    def _fast_hist_split(self, g, splits, fmask, f0):
        """Histograms + split search of the batch's children from one native pack."""
        t0 = time.perf_counter()
        h, s = hip(), stream(self.hist)
        order, nb, arr, off, nwork = g.plan_hist_packed(splits, self.TARGET_BLOCKS, self.MIN_ROWS_PER_BLOCK)
        base = _put_flat(self.up, arr)
        n = len(order)
        gp = self.gp_tree
        if nb:
            h.zero_slots(self.hist.data_ptr(), self.slot_bytes, base + 4 * off[2], nb, s)
            need = nwork * hist_cols(self.F) * self.B * 2
            if self._staging is None or self._staging.numel() < need:
                self._staging = torch.empty(int(need * 1.25), dtype=torch.int64, device=self.dev)
            h.hist_fx_staged(self.bins.data_ptr(), self.bins.shape[1], self.F, self.ghp.data_ptr(),
                             self.rows.data_ptr(), base, int(nwork), self.hist.data_ptr(), self.B,
                             float(gp["sg"]), float(gp["sh"]), 0, 0, self._staging.data_ptr(), 0, nb,
                             base + 4 * off[2], 0, s)
            if self.comm.is_dist:  # the built slots, gathered -> one all-reduce -> scattered
                idx = torch.from_numpy(arr[off[2]:off[2] + nb].astype(np.int64)).to(self.dev)
                if self.owner:
                    self._owner_reduce(idx)
                else:
                    buf = self.hist.index_select(0, idx)
                    self.comm.allreduce_(buf)
                    self.hist.index_copy_(0, idx, buf)
        t1 = time.perf_counter()
        if self._split_out is None or self._split_out.numel() < n * 48:
            self._split_out = torch.empty(max(n, 512) * 48, dtype=torch.uint8, device=self.dev)
        if self.owner:
            fmask, f0 = self._owner_mask(f0)
        h.split_find(self.hist.data_ptr(), self.B, self.F, self.nbins_f.data_ptr(), fmask.data_ptr(), int(f0),
                     base + 4 * off[1], n, self._split_out.data_ptr(), gp["mcw"], gp["l1"], gp["l2"],
                     gp["max_abs_leaf"], 1.0 / float(gp["sg"]), 1.0 / float(gp["sh"]), 0, 0, 0, 0, s)
        if self.owner:
            recs = self._owner_combine(self._split_out[:n * 48].view(n, 48))
        else:
            recs = self._split_out[:n * 48].cpu().numpy().view(gops.SPLIT_DTYPE).reshape(-1)
        self.up.reset()
        self.last_stats.build_hist += t1 - t0
        self.last_stats.find_split += time.perf_counter() - t1
        return order, recs

    def _grow_native(self, tree: Tree, fmask, f0: int, identity: bool, n_local: int, n_global: int):
        """Loss-guided growth with the native planner (csrc/native/leafwise.cpp): the same
        schedule, trees and statistics as ``_grow_loss_guided`` -- replay, speculative batch
        choice, child bookkeeping, slot recycling/LRU eviction and the tree itself live in
        C++; this loop only runs the device steps of each batch."""
        from ...ops._ext import native

        nat = native()
        p = self.p
        lp = nat.LwParams()
        lp.max_leaf = int(p.max_leaf_cnt)
        lp.max_depth = int(p.max_depth)
        lp.min_split_samples = int(p.min_split_samples)
        lp.min_split_loss = float(np.float32(p.min_split_loss))
        lp.mcw, lp.l1, lp.l2, lp.max_abs_leaf = (self.gp[k] for k in ("mcw", "l1", "l2", "max_abs_leaf"))
        lp.mcw2 = p.min_child_hessian_sum * 2.0
        lp.lr = float(np.float32(p.learning_rate))
        lp.speculate = bool(self.speculate)
        g = nat.LeafGrower(lp, int(self.n_slots))
        slot0 = g.root(int(n_local), int(n_global))
        items = np.array([[slot0, 0, 0, 0]], np.int32)
        recs = self._hist_split(np.array([0], np.int64), np.array([n_local], np.int64),
                                np.array([slot0], np.int32), 1, items, fmask, f0, identity_rows=identity)
        g.apply_recs(np.zeros(1, np.int32), recs)
        fast = self._fast_leafwise_ok()
        while True:
            t_plan = time.perf_counter()
            batch = g.replay()
            if not batch:
                self.last_stats.plan += time.perf_counter() - t_plan
                break
            splits, counts_only = g.expand(batch)
            self.last_stats.plan += time.perf_counter() - t_plan
            if counts_only:
                sg = g.segments(counts_only)
                lloc, lglob = self._count_arrays(sg[0], sg[1], sg[2], sg[3])
                g.set_children(counts_only, lloc, lglob, False)
            if splits:
                if fast:
                    lloc, lglob = self._fast_partition(g, splits)
                    g.set_children(splits, lloc, lglob, True)
                    order, recs = self._fast_hist_split(g, splits, fmask, f0)
                else:
                    sg = g.segments(splits)
                    lloc, lglob = self._partition_arrays(sg[0], sg[1], sg[2], sg[3], copy_back=True)
                    g.set_children(splits, lloc, lglob, True)
                    order, slots, nb, hb, hc, items = g.plan_hist(splits)
                    recs = self._hist_split(hb, hc, np.asarray(slots, np.int32), nb, items, fmask, f0)
                g.apply_recs(np.asarray(order, np.int32), recs)
            g.release_batch(batch)
        t = g.finish()
        n = len(t["left"])
        tree.left, tree.right, tree.parent = t["left"], t["right"], t["parent"]
        tree.feat, tree.slot_a, tree.slot_b, tree.cond = t["feat"], t["slot_a"], t["slot_b"], t["cond"]
        tree.leaf, tree.is_leaf = t["leaf"], t["is_leaf"]
        tree.loss_chg, tree.hess_sum, tree.sample_cnt = t["loss_chg"], t["hess_sum"], t["sample_cnt"]
        tree.feat_name = [None] * n
        tree.default_left = [True] * n
        self.last_batches, self.last_expanded = g.batches, g.expanded
        self.hist_miss += g.hist_miss

    def _grow_loss_guided(self, tree: Tree, nodes: Dict[int, _Node], fmask, f0, pop_is_leaf, make_leaf,
                          children_terminal, leafify_children) -> Dict[int, int]:
        """Exact leaf-wise growth (reference: priority queue ordered by lossChg,
        DataParallelTreeMaker.java:104-115,219-295) without one device round trip per node.

        The reference pops the best leaf, splits it, histograms its children and pushes
        them -- 254 strictly sequential steps for 255 leaves. Splitting a leaf never
        changes another leaf's best split, so the pop ORDER can be replayed on the host
        from the gains alone. Here the replay runs until it reaches a leaf that must be
        split but whose children are not computed yet; then that leaf AND the next
        best candidates (up to the remaining leaf budget) are expanded together in one
        batched partition + histogram + split launch group. Expansions the replay never
        pops are discarded (their rows were only permuted inside their own segment), so
        the tree -- node ids, splits, values, statistics -- is identical to the
        sequential algorithm, in ~log2(leaves) + a few batches instead of leaves - 1.

        ``nodes`` is keyed by speculative ids; returns {speculative id: tree node id}.
        """
        p = self.p
        max_leaf = p.max_leaf_cnt
        self.last_batches = self.last_expanded = 0
        tid = {0: 0}
        next_sid = [1]
        state = {"num_leaf": 1, "seq": 1}
        heap = [(-float(nodes[0].rec["loss_chg"]), 0, 0)]

        def expand(batch: List[int]):
            splits, counts_only = [], []
            for sid in batch:
                lc, rc = next_sid[0], next_sid[0] + 1
                next_sid[0] += 2
                nodes[sid].children = (lc, rc)
                # children at max_depth are always terminal: only their counts are needed
                (counts_only if (p.max_depth >= 0 and nodes[sid].depth + 1 == p.max_depth)
                 else splits).append((sid, lc, rc))
            if counts_only:
                self._count_children(nodes, counts_only)
            if splits:
                self._partition(nodes, splits, copy_back=True)
                build, derived = [], []
                for sid, lc, rc in splits:
                    nl, nr = nodes[lc], nodes[rc]
                    small, large = (lc, rc) if nl.cnt_global < nr.cnt_global else (rc, lc)
                    build.append(small)
                    if nodes[sid].slot >= 0:
                        derived.append((large, sid, small))
                    else:  # parent histogram evicted from the pool: rebuild (pool miss)
                        build.append(large)
                        self.hist_miss += 1
                self._build_and_find(nodes, build, derived, fmask, f0)
            for sid in batch:  # parents' histograms are no longer needed
                release(sid)

        def release(sid):
            nd = nodes[sid]
            if nd.slot >= 0:
                self.lru.pop(sid, None)
                self.free_slots.append(nd.slot)
                nd.slot = -1

        while True:
            t_plan = time.perf_counter()
            # replay the sequential priority-queue growth as far as the known gains allow
            blocked = False
            while heap:
                _, _, sid = heap[0]
                nd = nodes[sid]
                if pop_is_leaf(nd, state["num_leaf"]):
                    heapq.heappop(heap)
                    make_leaf(sid, tid[sid])
                    if nd.children is None:
                        release(sid)
                    continue
                if nd.children is None:
                    blocked = True
                    break
                heapq.heappop(heap)
                t = tid[sid]
                lc_t, rc_t = tree.add_children(t)
                r = nd.rec
                tree.set_split(t, int(r["feat"]), int(r["bin_a"]), int(r["bin_b"]))
                state["num_leaf"] += 1
                lcs, rcs = nd.children
                tid[lcs], tid[rcs] = lc_t, rc_t
                nl, nr = nodes[lcs], nodes[rcs]
                if children_terminal(nl, nr, state["num_leaf"]):
                    leafify_children(sid, lcs, rcs, lc_t, rc_t)
                    nl.rec_used = nr.rec_used = False
                    for c in (lcs, rcs):
                        if nodes[c].children is None:
                            release(c)
                else:
                    sq = state["seq"]
                    nl.seq, nr.seq = sq, sq + 1
                    heapq.heappush(heap, (-float(nl.rec["loss_chg"]), sq, lcs))
                    heapq.heappush(heap, (-float(nr.rec["loss_chg"]), sq + 1, rcs))
                    state["seq"] = sq + 2
            if not blocked:
                break
            # expansion batch: the blocked leaf + the next candidates in pop order
            remaining = (max_leaf - state["num_leaf"]) if max_leaf > 0 else 1
            # each expansion takes 2 slots and frees its own; keep one net slot per future split
            slack = (len(self.free_slots) - remaining - 1) // 2
            k = max(1, min(remaining, slack)) if self.speculate else 1
            # candidates: continue the replay VIRTUALLY, treating the not-yet-computed
            # children of unexpanded splits as absent; the unexpanded nodes this virtual
            # replay pops as splits (within the leaf budget) are exactly the ones the real
            # replay will split unless an unknown child outranks them -> expand them now
            _, _, blocked_sid = heap[0]
            batch = [blocked_sid]
            if k > 1:
                vheap = list(heap)
                vleaf = state["num_leaf"]
                vseq = state["seq"]
                chosen = {blocked_sid}
                while vheap and len(batch) < k:
                    _, _, sid = heapq.heappop(vheap)
                    nd = nodes[sid]
                    if pop_is_leaf(nd, vleaf):
                        continue
                    vleaf += 1
                    if nd.children is None:
                        if sid not in chosen:
                            chosen.add(sid)
                            batch.append(sid)
                        continue
                    lcs, rcs = nd.children
                    nl, nr = nodes[lcs], nodes[rcs]
                    if nl.rec is None or nr.rec is None or children_terminal(nl, nr, vleaf):
                        continue
                    heapq.heappush(vheap, (-float(nl.rec["loss_chg"]), vseq, lcs))
                    heapq.heappush(vheap, (-float(nr.rec["loss_chg"]), vseq + 1, rcs))
                    vseq += 2
            t_exp = time.perf_counter()
            self.last_stats.plan += t_exp - t_plan
            expand(batch)
            self.last_batches += 1
            self.last_expanded += len(batch)
        return tid

    # ------------------------------------------------------------------ build
    def build(self, gh: torch.Tensor, ghmax: Optional[torch.Tensor] = None, ghmax_global: bool = False) -> Tree:
        """Grow one tree from gh [N, 2] (grad*w, hess*w) in row order. ``ghmax`` (optional,
        float32 [2]): max |g|, |h| over the rows, already produced by the gradient kernel."""
        p = self.p
        t_start = time.perf_counter()
        self.last_stats = TimeStats()
        self.next_slot = 0
        # loss-guided growth recycles histogram slots (a slot is free again once its node is
        # expanded or finalised as a leaf): live slots = the known-gain frontier only
        self.free_slots = list(range(self.n_slots - 1, -1, -1)) if p.grow_policy == "loss" else None
        self.lru = OrderedDict()  # speculative node id -> slot, oldest first
        self.up.reset()
        rng = np.random.default_rng((p.seed, self.tree_count))
        seed_rows = int(rng.integers(1 << 62))
        # --- instance subsampling (DataParallelTreeMaker.initAssistData :405-423)
        identity = True
        if p.instance_sample_rate < 1.0:
            g = torch.Generator(device=self.dev)
            g.manual_seed(seed_rows + self.comm.rank)
            keep = torch.rand(self.N, generator=g, device=self.dev) < p.instance_sample_rate
            sel = torch.nonzero(keep, as_tuple=False).flatten().to(torch.int32)
            n_local = int(sel.numel())
            self.rows[:n_local].copy_(sel)
            self.ghp[:n_local].copy_(gh.index_select(0, sel.long()))
            identity = False
            self._root_gh = None
            self.last_keep = keep
        elif os.environ.get("YTK_HOST_IDROOT", "1") != "0":
            # no copies: the root histogram and the first partition read the identity
            # permutation and the caller's gh directly
            n_local = self.N
            self._root_gh = gh.contiguous()
            self.last_keep = None
        else:
            n_local = self.N
            self._root_gh = None
            self.rows.copy_(self.iota)
            self.ghp.copy_(gh)
            self.last_keep = None
        # --- feature subsampling with a globally agreed seed (:432-461)
        if p.feature_sample_rate < 1.0:
            n_sam = max(1, int(round(p.feature_sample_rate * self.F)))
            perm = rng.permutation(self.F)
            fm = np.zeros(self.F, np.uint8)
            fm[np.sort(perm[:n_sam])] = 1
        else:
            fm = np.ones(self.F, np.uint8)
        f0 = int(np.nonzero(fm)[0][0])
        if not np.array_equal(fm, self.fmask_np) or not hasattr(self, "fmask"):
            self.fmask_np = fm
            self.fmask = torch.from_numpy(fm).to(self.dev)
        fmask = self.fmask

        n_global = int(self.comm.allreduce_scalars([n_local], dtype=torch.int64)[0]) if self.comm.is_dist else n_local
        # per-tree fixed-point scales from the global max |g|, |h| (identical on every rank)
        if ghmax is not None and (identity or ghmax_global):
            mx = ghmax.double()
        elif n_local > 0:
            mx = (self._root_gh if identity else self.ghp[:n_local]).abs().amax(dim=0).double()
        else:
            mx = torch.zeros(2, dtype=torch.float64, device=self.dev)
        if self.comm.is_dist and not ghmax_global:
            self.comm.allreduce_(mx, op="max")
        mx = mx.cpu().numpy()
        sg, sh = gops.fixed_point_scales(mx[0], mx[1], n_global)
        self.gp_tree = dict(self.gp, sg=sg, sh=sh)
        tree = Tree()
        if p.grow_policy == "loss" and self.native_leafwise:
            self._grow_native(tree, fmask, f0, identity, n_local, n_global)
            return self._finish_tree(tree, {}, t_start)
        nodes: Dict[int, _Node] = {0: _Node(begin=0, cnt_local=n_local, cnt_global=n_global, depth=0, seq=0)}
        self._build_and_find(nodes, [0], [], fmask, f0, identity_rows=identity)
        seq = 1
        num_leaf = 1
        max_leaf = p.max_leaf_cnt
        lr32 = np.float32(p.learning_rate)

        def pop_is_leaf(nd: _Node, num_leaf: int):
            return (nd.rec["loss_chg"] <= msl32
                    or (p.max_depth >= 0 and p.max_depth == nd.depth)
                    or (max_leaf > 0 and max_leaf == num_leaf)
                    or (p.min_split_samples > 0 and nd.cnt_global < p.min_split_samples))

        gpv = (self.gp["mcw"], self.gp["l1"], self.gp["l2"], self.gp["max_abs_leaf"])
        msl32 = float(np.float32(p.min_split_loss))  # the kernels compare float32 gains to it

        def make_leaf(nid, t=None):
            nd = nodes[nid]
            v = np.float32(gops.node_value_py(nd.G, nd.H, *gpv))
            tree.set_leaf(nid if t is None else t, float(v * lr32))

        def children_terminal(nd_l: _Node, nd_r: _Node, nleaf: int):
            return ((p.max_depth >= 0 and p.max_depth == nd_l.depth)
                    or (max_leaf > 0 and max_leaf == nleaf)
                    or (p.min_split_samples > 0 and nd_l.cnt_global < p.min_split_samples
                        and nd_r.cnt_global < p.min_split_samples))

        def leafify_children(nid, lc, rc, lt=None, rt=None):
            r = nodes[nid].rec
            nl, nr = nodes[lc], nodes[rc]
            nl.G, nl.H = float(r["gl"]), float(r["hl"])
            nr.G, nr.H = nodes[nid].G - nl.G, nodes[nid].H - nl.H
            make_leaf(lc, lt)
            make_leaf(rc, rt)

        if p.grow_policy == "level":
            level = [0]
            while level:
                splits, snapshot = [], []
                for nid in level:  # FIFO by seq
                    nd = nodes[nid]
                    if pop_is_leaf(nd, num_leaf):
                        make_leaf(nid)
                        continue
                    r = nd.rec
                    lc, rc = tree.add_children(nid)
                    tree.set_split(nid, int(r["feat"]), int(r["bin_a"]), int(r["bin_b"]))
                    num_leaf += 1
                    splits.append((nid, lc, rc))
                    snapshot.append(num_leaf)
                if not splits:
                    break
                # children of the deepest level never need their rows: skip the partition
                last_level = p.max_depth >= 0 and nodes[splits[0][0]].depth + 1 == p.max_depth
                if last_level:
                    self._count_children(nodes, splits)
                    for nid, lc, rc in splits:
                        leafify_children(nid, lc, rc)
                    break
                self._partition(nodes, splits, copy_back=False)
                build, derived, nxt = [], [], []
                for (nid, lc, rc), nl_snap in zip(splits, snapshot):
                    nl, nr = nodes[lc], nodes[rc]
                    if children_terminal(nl, nr, nl_snap):
                        leafify_children(nid, lc, rc)
                    else:
                        small, large = (lc, rc) if nl.cnt_global < nr.cnt_global else (rc, lc)
                        build.append(small)
                        derived.append((large, nid, small))
                        nl.seq, nr.seq = seq, seq + 1
                        seq += 2
                        nxt += [lc, rc]
                if build:
                    self._build_and_find(nodes, build, derived, fmask, f0)
                level = nxt
        else:  # loss-guided (leaf-wise), exact, expanded in speculative batches
            tid = self._grow_loss_guided(tree, nodes, fmask, f0, pop_is_leaf, make_leaf,
                                         children_terminal, leafify_children)
            ts, lcs, hs = [], [], []
            for sid, t in tid.items():
                nd = nodes[sid]
                ts.append(t)
                lcs.append(nd.rec["loss_chg"] if nd.rec is not None and nd.rec_used else float("-inf"))
                hs.append(nd.H)
                tree.sample_cnt[t] = nd.cnt_global
            # float32 rounding of the dumped statistics, vectorised
            for t, lc, h in zip(ts, np.asarray(lcs, np.float32).tolist(), np.asarray(hs, np.float32).tolist()):
                tree.loss_chg[t] = lc
                tree.hess_sum[t] = h
            nodes = {}

        return self._finish_tree(tree, nodes, t_start)

    def _finish_tree(self, tree: Tree, nodes: Dict[int, _Node], t_start: float) -> Tree:
        # node stats for the dump (updateTreeNodeStat)
        for nid in range(tree.num_nodes):
            nd = nodes.get(nid)
            if nd is None:
                continue
            tree.loss_chg[nid] = float(np.float32(nd.rec["loss_chg"])) if nd.rec is not None else float("-inf")
            tree.hess_sum[nid] = float(np.float32(nd.H))
            tree.sample_cnt[nid] = nd.cnt_global
        self.tree_count += 1
        self.last_stats.total = time.perf_counter() - t_start
        self.last_stats.trees = 1
        self.total_stats.add(self.last_stats)
        return tree
