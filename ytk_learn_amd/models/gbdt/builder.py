"""Data-parallel histogram tree builder (level-wise and loss-guided growth).

Reference behaviour: ``J/optimizer/gbdt/DataParallelTreeMaker.java`` (make() :229-295,
expansion conditions :249-273, smaller-child histogram + subtraction :489-508,
node stats :543-573, split enumeration :598-637, best-split sync :640-653) and
``J/optimizer/gbdt/UpdateStrategy.java``.

MI355X-first structure (not a translation):
  * all per-row state (bins, g/h, row permutation) stays resident in HBM;
  * one batched launch per level for histogram build / split search / partition
    (level-wise); loss-guided growth uses the same kernels with batch size 1;
  * histograms are indexed by a per-tree slot counter (no LRU pool: even 509
    slots x 28 features x 256 bins is 29 MB of the 288 GB HBM);
  * multi-GPU: rows are sharded; the level's freshly built histograms are one
    contiguous slab -> ONE RCCL all-reduce per level (owner-compute reduce-scatter
    is unnecessary at these sizes: the reduced slab is what every rank's split
    kernel reads, and identical inputs give identical split decisions on every
    rank, so no SplitInfo exchange is needed).
"""
from __future__ import annotations

import heapq
import math
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ...ops import gbdt as gops
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

    def gain_params(self):
        f = lambda v: float(np.float32(v))  # kernel receives float32 params
        return {"mcw": f(self.min_child_hessian_sum), "l1": f(self.l1), "l2": f(self.l2),
                "max_abs_leaf": f(self.max_abs_leaf_val)}


@dataclass
class TimeStats:
    """Per-phase timers mirroring ``J/data/gbdt/TimeStats.java`` names (host wall
    time incl. the device work the phase waits for)."""
    build_hist: float = 0.0
    comm_hist: float = 0.0
    find_split: float = 0.0
    partition: float = 0.0
    total: float = 0.0
    trees: int = 0

    def add(self, o: "TimeStats"):
        for k in ("build_hist", "comm_hist", "find_split", "partition", "total"):
            setattr(self, k, getattr(self, k) + getattr(o, k))
        self.trees += o.trees

    def stats(self) -> str:
        return (f"[time stats] trees={self.trees} total={self.total:.4f}s build_hist={self.build_hist:.4f}s "
                f"comm_hist={self.comm_hist:.4f}s find_split={self.find_split:.4f}s "
                f"partition={self.partition:.4f}s")


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


class TreeBuilder:
    # blocks of the histogram / partition launches: rows per block bounds
    MIN_ROWS_PER_BLOCK = 2048
    TARGET_BLOCKS = 1024

    def __init__(self, bins: torch.Tensor, F: int, B: int, nbins_f: np.ndarray,
                 params: TreeParams, comm: Optional[Comm] = None, profile: bool = False):
        self.bins = bins
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
        self.hist = torch.zeros((self.max_nodes, B, F, 2), dtype=torch.float32, device=self.dev)
        self.rows = torch.empty(self.N, dtype=torch.int32, device=self.dev)
        self.rows_tmp = torch.empty(self.N, dtype=torch.int32, device=self.dev)
        self.iota = torch.arange(self.N, dtype=torch.int32, device=self.dev)
        self.profile = profile
        self.last_stats = TimeStats()
        self.total_stats = TimeStats()
        self.tree_count = 0

    # ------------------------------------------------------------------ utils
    def _sync(self):
        if self.profile and self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def _to_dev(self, a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.to(self.dev, non_blocking=True) if self.dev.type == "cuda" else t

    def _chunks(self, total: int) -> int:
        return max(self.MIN_ROWS_PER_BLOCK, -(-total // self.TARGET_BLOCKS))

    def _hist_work(self, segs):
        """segs: list of (slot, begin, count) -> int32 [nwork, 4]"""
        total = sum(c for _, _, c in segs)
        ch = self._chunks(total)
        w = []
        for slot, b, c in segs:
            e = b + c
            for s in range(b, e, ch):
                w.append((slot, s, min(s + ch, e), 0))
        return np.array(w, np.int32).reshape(-1, 4)

    # ----------------------------------------------------------- primitives
    def _build_and_find(self, tree: Tree, nodes: Dict[int, _Node], build: List[int],
                        derived: List[tuple], gh: torch.Tensor, fmask: torch.Tensor, f0: int,
                        identity_rows: bool = False):
        """Histogram the ``build`` nodes, derive ``derived`` = (node, parent, sibling),
        then find the best split of every one of them."""
        st = self.last_stats
        t0 = time.perf_counter()
        s0 = self.next_slot
        for i, nid in enumerate(build):
            nodes[nid].slot = s0 + i
        for j, (nid, _, _) in enumerate(derived):
            nodes[nid].slot = s0 + len(build) + j
        self.next_slot += len(build) + len(derived)
        nb = len(build)
        if nb:
            self.hist[s0:s0 + nb].zero_()
            work = self._hist_work([(nodes[n].slot, nodes[n].begin, nodes[n].cnt_local) for n in build])
            gops.hist_build(self.bins, self.F, gh, None if identity_rows else self.rows,
                            self._to_dev(work), self.hist, self.B)
        self._sync()
        t1 = time.perf_counter()
        if nb and self.comm.is_dist:
            self.comm.allreduce_(self.hist[s0:s0 + nb])
            self._sync()
        t2 = time.perf_counter()
        items = [(nodes[n].slot, 0, 0, 0) for n in build]
        items += [(nodes[n].slot, nodes[p].slot, nodes[s].slot, 1) for n, p, s in derived]
        order = list(build) + [n for n, _, _ in derived]
        out = gops.split_find(self.hist, self.B, self.F, self.nbins_f, fmask, f0,
                              self._to_dev(np.array(items, np.int32).reshape(-1, 4)), self.gp)
        recs = out.cpu().numpy().view(gops.SPLIT_DTYPE).reshape(-1)
        t3 = time.perf_counter()
        for nid, r in zip(order, recs):
            nd = nodes[nid]
            nd.rec = r
            nd.G = float(r["g"])
            nd.H = float(r["h"])
            # canSplit (UpdateStrategy.canSplit): H >= 2*mcw and n >= min_split_samples
            if not (nd.H >= self.p.min_child_hessian_sum * 2.0 and nd.cnt_global >= self.p.min_split_samples):
                r["loss_chg"] = -np.inf
                r["feat"] = -1
        st.build_hist += t1 - t0
        st.comm_hist += t2 - t1
        st.find_split += t3 - t2

    def _partition(self, nodes: Dict[int, _Node], splits: List[tuple], copy_back: bool):
        """splits: list of (nid, left_child, right_child). Updates child segments/counts."""
        t0 = time.perf_counter()
        n = len(splits)
        total = sum(nodes[s[0]].cnt_local for s in splits)
        ch = self._chunks(total)
        items, first_blk, nblk = [], [], []
        feat = np.empty(n, np.int32)
        thr = np.empty(n, np.int32)
        nbeg = np.empty(n, np.int32)
        for i, (nid, _, _) in enumerate(splits):
            nd = nodes[nid]
            r = nd.rec
            feat[i] = int(r["feat"])
            thr[i] = (int(r["bin_a"]) + int(r["bin_b"])) // 2
            nbeg[i] = nd.begin
            first_blk.append(len(items))
            k = 0
            for s in range(nd.begin, nd.begin + nd.cnt_local, ch):
                items.append((i, s, min(s + ch, nd.begin + nd.cnt_local), k))
                k += 1
            nblk.append(k)
        left = gops.partition(self.bins, self.rows, self.rows_tmp,
                              self._to_dev(np.array(items, np.int32).reshape(-1, 4)),
                              self._to_dev(feat), self._to_dev(thr), self._to_dev(nbeg),
                              self._to_dev(np.array(first_blk, np.int32)),
                              self._to_dev(np.array(nblk, np.int32)), n)
        if copy_back:
            for nid, _, _ in splits:
                nd = nodes[nid]
                if nd.cnt_local:
                    self.rows[nd.begin:nd.begin + nd.cnt_local].copy_(
                        self.rows_tmp[nd.begin:nd.begin + nd.cnt_local])
        else:
            self.rows, self.rows_tmp = self.rows_tmp, self.rows
        left_l = left.to(torch.int64)
        if self.comm.is_dist:
            both = torch.stack([left_l, left_l]).to(self.dev)
            self.comm.allreduce_(both[1])
            both = both.cpu().numpy()
            lloc, lglob = both[0], both[1]
        else:
            lloc = left_l.cpu().numpy()
            lglob = lloc
        for i, (nid, lc, rc) in enumerate(splits):
            nd = nodes[nid]
            nodes[lc] = _Node(begin=nd.begin, cnt_local=int(lloc[i]), cnt_global=int(lglob[i]),
                              depth=nd.depth + 1)
            nodes[rc] = _Node(begin=nd.begin + int(lloc[i]), cnt_local=nd.cnt_local - int(lloc[i]),
                              cnt_global=nd.cnt_global - int(lglob[i]), depth=nd.depth + 1)
        self.last_stats.partition += time.perf_counter() - t0

    # ------------------------------------------------------------------ build
    def build(self, gh: torch.Tensor) -> Tree:
        """Grow one tree from gh [N, 2] (grad*w, hess*w)."""
        p = self.p
        t_start = time.perf_counter()
        self.last_stats = TimeStats()
        self.next_slot = 0
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
            identity = False
            self.last_keep = keep
        else:
            n_local = self.N
            self.rows.copy_(self.iota)
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
        fmask = self._to_dev(fm)

        n_global = int(self.comm.allreduce_scalars([n_local], dtype=torch.int64)[0]) if self.comm.is_dist else n_local
        tree = Tree()
        nodes: Dict[int, _Node] = {0: _Node(begin=0, cnt_local=n_local, cnt_global=n_global, depth=0, seq=0)}
        self._build_and_find(tree, nodes, [0], [], gh, fmask, f0, identity_rows=identity)
        seq = 1
        num_leaf = 1
        max_leaf = p.max_leaf_cnt

        def pop_is_leaf(nd: _Node):
            return (nd.rec["loss_chg"] <= p.min_split_loss
                    or (p.max_depth >= 0 and p.max_depth == nd.depth)
                    or (max_leaf > 0 and max_leaf == num_leaf)
                    or (p.min_split_samples > 0 and nd.cnt_global < p.min_split_samples))

        def leaf_value(G, H):
            v = np.float32(gops.node_value_np(G, H, self.gp["mcw"], self.gp["l1"], self.gp["l2"],
                                              self.gp["max_abs_leaf"]))
            return float(v * np.float32(p.learning_rate))

        def make_leaf(nid):
            nd = nodes[nid]
            tree.set_leaf(nid, leaf_value(nd.G, nd.H))

        def children_terminal(nd_l: _Node, nd_r: _Node):
            return ((p.max_depth >= 0 and p.max_depth == nd_l.depth)
                    or (max_leaf > 0 and max_leaf == num_leaf)
                    or (p.min_split_samples > 0 and nd_l.cnt_global < p.min_split_samples
                        and nd_r.cnt_global < p.min_split_samples))

        if p.grow_policy == "level":
            level = [0]
            while level:
                splits = []
                snapshot = []
                for nid in level:  # FIFO by seq
                    nd = nodes[nid]
                    if pop_is_leaf(nd):
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
                self._partition(nodes, splits, copy_back=False)
                build, derived, nxt = [], [], []
                for (nid, lc, rc), nl_snap in zip(splits, snapshot):
                    nl, nr = nodes[lc], nodes[rc]
                    saved = num_leaf
                    num_leaf = nl_snap
                    term = children_terminal(nl, nr)
                    num_leaf = saved
                    r = nodes[nid].rec
                    if term:
                        nl.G, nl.H = float(r["gl"]), float(r["hl"])
                        nr.G, nr.H = nodes[nid].G - nl.G, nodes[nid].H - nl.H
                        make_leaf(lc)
                        make_leaf(rc)
                    else:
                        small, large = (lc, rc) if nl.cnt_global < nr.cnt_global else (rc, lc)
                        build.append(small)
                        derived.append((large, nid, small))
                        nl.seq, nr.seq = seq, seq + 1
                        seq += 2
                        nxt += [lc, rc]
                if build:
                    self._build_and_find(tree, nodes, build, derived, gh, fmask, f0)
                level = nxt
        else:  # loss-guided
            heap = [(-float(nodes[0].rec["loss_chg"]), 0, 0)]
            while heap:
                _, _, nid = heapq.heappop(heap)
                nd = nodes[nid]
                if pop_is_leaf(nd):
                    make_leaf(nid)
                    continue
                r = nd.rec
                lc, rc = tree.add_children(nid)
                tree.set_split(nid, int(r["feat"]), int(r["bin_a"]), int(r["bin_b"]))
                num_leaf += 1
                self._partition(nodes, [(nid, lc, rc)], copy_back=True)
                nl, nr = nodes[lc], nodes[rc]
                if children_terminal(nl, nr):
                    nl.G, nl.H = float(r["gl"]), float(r["hl"])
                    nr.G, nr.H = nd.G - nl.G, nd.H - nl.H
                    make_leaf(lc)
                    make_leaf(rc)
                else:
                    small, large = (lc, rc) if nl.cnt_global < nr.cnt_global else (rc, lc)
                    self._build_and_find(tree, nodes, [small], [(large, nid, small)], gh, fmask, f0)
                    nl.seq, nr.seq = seq, seq + 1
                    heapq.heappush(heap, (-float(nl.rec["loss_chg"]), seq, lc))
                    heapq.heappush(heap, (-float(nr.rec["loss_chg"]), seq + 1, rc))
                    seq += 2

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
