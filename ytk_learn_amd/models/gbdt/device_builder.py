"""GPU-resident level-wise tree builder (no host synchronisation inside a tree).

Same semantics as :class:`.builder.TreeBuilder` with ``grow_policy="level"`` and a
bounded depth (reference: ``J/optimizer/gbdt/DataParallelTreeMaker.java`` make(),
FIFO queue). Every per-level decision (leaf or split, children counts, terminal
children, smaller-child choice, work lists) is taken on the device by the planner
kernels of ``csrc/hip/gbdt_level.hip``; partition / histogram / split kernels are
launched with fixed maximal grids and read their work counts from device memory.
A tree is therefore a fixed launch sequence that the host enqueues without
waiting; multi-GPU all-reduces (root count, max |g|/|h|, per-level child counts,
per-level histogram slab) are fixed-size RCCL calls on the same stream.

Histogram slot layout: the nodes at depth c use slots [2^c - 1, 2^(c+1) - 1):
built (smaller) children in the first half, derived children in the second.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ...ops import gbdt as gops
from ...ops import _ext
from ...ops._ext import CUR_STRIDE, DONE_WORDS, hip, hist_cols, ptr, stream
from ...parallel import peer as peer_mod
from ...parallel.comm import Comm
from ...utils.timestats import PhaseTimer
from .builder import TimeStats, TreeParams, resolve_hist_sync
from .tree import Tree

DNODE_DTYPE = np.dtype([
    ("G", "<f8"), ("H", "<f8"), ("gl", "<f8"), ("hl", "<f8"), ("cnt_global", "<i8"),
    ("begin", "<i4"), ("cnt_local", "<i4"), ("depth", "<i4"), ("slot", "<i4"),
    ("feat", "<i4"), ("bin_a", "<i4"), ("bin_b", "<i4"), ("left", "<i4"), ("right", "<i4"),
    ("loss_chg", "<f4"), ("value", "<f4"), ("is_leaf", "<i4")])
assert DNODE_DTYPE.itemsize == 88
ST_NUM_NODES = 0
ST_N_HIST_A = 8  # st word: hist items of the first half of a level's build slots

MAX_DEPTH_DEVICE = 30
MAX_LEVEL_NODES = 4096  # kMaxPend (csrc/hip/gbdt_level.hip): nodes of one level in the planner's LDS


def level_width(params: TreeParams) -> int:
    """Most nodes one level can hold: min(2^max_depth, max_leaf_cnt rounded up to a power of
    two) -- distinct nodes of one depth have disjoint subtrees, each with >= 1 leaf."""
    D = params.max_depth
    w = 1 << min(max(D, 0), 40)
    if params.max_leaf_cnt > 0:
        w = min(w, 1 << max(0, (params.max_leaf_cnt - 1).bit_length()))
    return w


def level_slots_needed(params: TreeParams) -> int:
    """Histogram slots of the level engine's slab (without the multi-GPU count slots)."""
    half_cap = max(1, level_width(params) // 2)
    return 1 + sum(2 * min(1 << (c - 1), half_cap) for c in range(1, max(params.max_depth, 1)))


def level_slots_pingpong(params: TreeParams, ncs: int = 0) -> int:
    """Slots of the level engine's capped slab (histogram_pool_capacity below the full one):
    only two levels are ever live -- level c's histograms are the parents its children's
    derived histograms subtract from, level c - 1's are dead once level c is searched -- so
    odd and even levels alternate between two regions (the root keeps slot 0)."""
    half_cap = max(1, level_width(params) // 2)
    reg = [0, 0]
    for c in range(1, max(params.max_depth, 1)):
        reg[c % 2] = max(reg[c % 2], 2 * min(1 << (c - 1), half_cap) + ncs)
    return 1 + reg[0] + reg[1]


class DeviceTree:
    """Handle of a tree built on the device: node-table snapshot + scoring arrays."""

    def __init__(self, nodes: torch.Tensor, st: torch.Tensor, bin_arrays, max_nodes: int,
                 snap: Optional[torch.Tensor] = None, st_bytes: int = 64):
        self.nodes = nodes
        self.st = st
        self.bin_arrays = bin_arrays
        self.max_nodes = max_nodes
        self.snap = snap          # the whole snapshot buffer (st | nodes | scoring arrays)
        self.st_bytes = st_bytes

    def split_host_snap(self, host: np.ndarray):
        """(node-table bytes, st words) views of a host copy of ``snap``."""
        nb = self.max_nodes * DNODE_DTYPE.itemsize
        return host[self.st_bytes:self.st_bytes + nb], host[:self.st_bytes].view(np.int32)

    def to_tree(self, nodes_np=None, st_np=None) -> Tree:
        nd = (nodes_np if nodes_np is not None else self.nodes.cpu().numpy())
        st = st_np if st_np is not None else self.st.cpu().numpy()
        tree = node_table_to_tree(nd, st)
        lc = getattr(self, "leaf_counts", None)
        if lc is not None:  # deferred last-level counts (this process's rows)
            leaf = np.asarray(tree.is_leaf, bool)
            sc = np.asarray(tree.sample_cnt, np.int64)
            sc[leaf] = np.rint(lc.cpu().numpy()[:leaf.size][leaf]).astype(np.int64)
            tree.sample_cnt = sc.tolist()
        return tree


def node_table_to_tree(nodes_bytes: np.ndarray, st: np.ndarray) -> Tree:
    """Device node table (DNODE_DTYPE records) -> host Tree, vectorised (no per-node loop)."""
    nn = int(st[ST_NUM_NODES])
    nd = np.asarray(nodes_bytes).view(DNODE_DTYPE).reshape(-1)[:nn]
    leaf = (nd["is_leaf"] != 0) | (nd["left"] < 0)
    inner = ~leaf
    if inner.any() and (int(nd["left"][inner].max()) >= nn or int(nd["right"][inner].max()) >= nn):
        raise RuntimeError(f"device tree engine: inconsistent node table ({nn} nodes, a child id past the end; "
                           f"leaf-wise: speculative node overflow); state words {np.asarray(st)[:16].tolist()}")
    return Tree.from_arrays(nd["left"], nd["right"], nd["feat"], nd["bin_a"], nd["bin_b"], nd["value"], leaf,
                            nd["loss_chg"], nd["H"], nd["cnt_global"])


class DeviceLevelBuilder:
    HIST_TARGET = int(os.environ.get("YTK_HIST_TARGET", 256))  # 1 block per CU (128 KiB LDS each)
    PART_TARGET = 1024
    MIN_ROWS = int(os.environ.get("YTK_HIST_MIN_ROWS", 2048))

    def __init__(self, bins: torch.Tensor, binsT: torch.Tensor, F: int, B: int, nbins_f: np.ndarray,
                 params: TreeParams, comm: Comm = None, timer: Optional[PhaseTimer] = None,
                 pool_slots: Optional[int] = None):
        assert bins.is_cuda
        self.timer = timer if timer is not None else PhaseTimer()
        p = params
        if (not (1 <= p.max_depth <= MAX_DEPTH_DEVICE) or p.grow_policy != "level"
                or level_width(p) > MAX_LEVEL_NODES):
            raise ValueError("device builder needs level-wise growth, 1 <= max_depth <= 30 and at most 4096 "
                             "nodes per level (min(2^max_depth, max_leaf_cnt))")
        if not self.supports(bins, binsT, B, F):
            raise ValueError(f"device builder: unsupported bin layout (dtype {bins.dtype}, B={B}, F={F})")
        # wide mode: uint16 bins with B > 256 -> feature-grouped LDS histograms over binsT
        self.wide = bins.dtype == torch.int16
        # wide: ~WIDE_HIST_BLOCKS (work item, feature group) blocks per level
        self.hist_target = (min(self.HIST_TARGET, max(8, gops.WIDE_HIST_BLOCKS // (-(-F // gops.wide_group(B, F)))))
                            if self.wide else self.HIST_TARGET)
        self.p = p
        self.bins, self.binsT = bins, binsT
        self.dev = bins.device
        self.N = bins.shape[0]
        self.F, self.B = F, B
        self.comm = comm or Comm.local(self.dev)
        self.nbins_f = torch.from_numpy(np.asarray(nbins_f, np.int32)).to(self.dev)
        D = p.max_depth
        ml = p.max_leaf_cnt if p.max_leaf_cnt > 0 else (1 << 30)
        self.max_nodes = int(min((1 << (D + 1)) - 1, 2 * ml - 1))
        # nodes of one level (<= 2^D, and <= the leaf budget): every per-level array and the
        # histogram slots of a level are sized by it, so deep trees with a leaf budget (e.g.
        # depth 16, 255 leaves) keep small slabs
        self.maxp = level_width(p)
        # single-pass partition: one tile reservation (a global atomic round trip) per
        # 1024 rows, so chunks stay at MIN_ROWS (2 tiles) and the latency hides behind
        # ~N/2048 resident blocks instead of ~10 serial reservations per block
        # (the kernel holds one chunk of <= 2048 rows per block in registers)
        self.part_atomic = os.environ.get("YTK_PART_ATOMIC", "1") != "0" and self.MIN_ROWS == 2048
        # Multi-GPU with fused counts: the partition kernel accumulates the level's per-split
        # row counts straight into count slots that ride in the level's histogram message,
        # so ONE all-reduce of [built slots + count slots] carries the histograms and the
        # counts of the level (reference: DataParallelTreeMaker.java:518,538 count allreduce +
        # HistogramBuilder.java:95 reduce-scatter -> one fixed-size RCCL call).
        self.fuse_counts = (self.comm.is_dist and p.min_split_samples <= 0
                            and os.environ.get("YTK_FUSE_COUNTS", "1") != "0")
        # uint8 bins: the children planner runs in the partition kernel's last block
        # (YTK_FUSE_PART_CHILDREN=0: separate launches). Multi-GPU only with fused counts: the
        # children are planned from the LOCAL counts (the smaller child by the globally
        # identical hessian sums) and the next level's planner patches the global counts
        # from the all-reduced cursors.
        # (uint16 bins too: one kernel configuration, 2048-row chunks)
        self.fuse_part_children = (self.part_atomic and bins.dtype in (torch.uint8, torch.int16)
                                   and (not self.comm.is_dist or self.fuse_counts)
                                   and os.environ.get("YTK_FUSE_PART_CHILDREN", "1") != "0")
        # rows per partition chunk (= per cursor reservation): 8 rows per thread (2048);
        # YTK_PART_CHUNK=4096 runs the fused kernel at 16 rows per thread -- half the
        # reservations on the top levels' few cursors, but 4 instead of 8 waves/SIMD.
        # Measured (profiles/r2_partition_chunk.md): root level 105 -> 100 us, deep levels
        # 93 -> 100 us, tree 1.50 ms either way
        # (multi-GPU: the last level runs the standalone 2048-row partition, so the chunk stays
        # at 2048 for every level)
        self.part_chunk = (int(os.environ.get("YTK_PART_CHUNK", "2048"))
                           if self.fuse_part_children and not self.comm.is_dist and bins.dtype == torch.uint8
                           else self.MIN_ROWS)
        self.part_target = (-(-self.N // self.part_chunk) + 1) if self.part_atomic else self.PART_TARGET
        # one GPU: split search + next level's split planning in one launch (YTK_FUSE_SPLIT_PLAN=1).
        # Off by default: the release/acquire fences it needs cost what the saved launch
        # saved (measured 24.2 -> 25.0 us per level, profiles/r2_split_plan_fusion.md)
        self.fuse_split_plan = (self.fuse_part_children and not self.wide and not self.comm.is_dist
                                and os.environ.get("YTK_FUSE_SPLIT_PLAN", "0") == "1")
        self.max_items = max(self.hist_target, self.part_target) + self.maxp + 16
        dev = self.dev
        i32 = lambda n: torch.zeros(n, dtype=torch.int32, device=dev)
        # everything a finished tree is (state, node table, scoring arrays) lives in ONE
        # buffer so the per-tree snapshot is a single device copy
        mn = self.max_nodes
        self._snap_sizes = [64, mn * DNODE_DTYPE.itemsize] + [4 * mn] * 5
        # the snapshot and, 16-B aligned right behind it, the trainer's round vector
        # [train loss, weight | test loss, weight | leaf counts] (round_vector): one readback copy
        snap_total = sum(self._snap_sizes)
        self.rv_off = (snap_total + 15) // 16 * 16
        # (+ 16 B: the in-graph readback copies whole 16-B units)
        self._snap_full = torch.zeros(self.rv_off + 8 * (4 + mn) + 16, dtype=torch.uint8, device=dev)
        self.snap = self._snap_full[:snap_total]
        (self.st, self.nodes, self.tfeat, self.tthr, self.tleft, self.tright,
         self.tval) = self._snap_views(self.snap)
        self.pending, self.next_pending = i32(self.maxp), i32(self.maxp)
        self.split_nid, self.split_snap = i32(self.maxp), i32(self.maxp)
        self.part_items = i32(self.max_items * 4)
        self.part_feat, self.part_thr, self.part_begin = i32(self.maxp), i32(self.maxp), i32(self.maxp)
        self.part_first, self.part_nblk = i32(self.maxp), i32(self.maxp)
        self.part_counts = i32(self.max_items)
        self.part_cnt = i32(self.maxp)
        # per-split left counters / partition cursors: index s (standalone partition kernels)
        # or s * CUR_STRIDE (fused partition: one cache line per cursor), then the fused
        # kernel's self-resetting done counters (csrc/hip/gbdt_partition_atomic.h)
        ncur = self.maxp * CUR_STRIDE + DONE_WORDS
        self.left_loc = torch.zeros(ncur, dtype=torch.int64, device=dev)
        self.left_glob = torch.zeros(ncur, dtype=torch.int64, device=dev)
        self.hist_items = i32(self.max_items * 4)
        self.split_items = i32(2 * self.maxp * 4)
        self.item_nid = i32(2 * self.maxp)
        self.hist_first = i32(self.maxp + 2)  # per build: first histogram item (+ the item count)
        # feature groups per node in the split search (one block per (node, group), each on
        # its own CU; the planner keeps each node's best record): YTK_SPLIT_GROUPS, default 4.
        # The owner-computes mode and the fused split + plan kernel write one record per node.
        self.owner = self.comm.is_dist and resolve_hist_sync(p.hist_sync, B * F * 2 * 8) == "owner"
        self.split_groups = (gops.split_groups(B, F) if not (self.owner or self.wide or self.fuse_split_plan)
                             else 1)
        # one GPU, uint8 bins: every gathered level's staged slot reduce and its split search run
        # as ONE launch (lv_reduce_split_kernel: the last reduce block of each (build, 8-feature
        # group) searches the built child and its derived sibling) -- one record per 8-feature
        # group, so the planner combines ceil(F / 8) records per node (opt-in: YTK_FUSE_REDUCE_SPLIT=1; default
        # hist_reduce + split_node launches)
        self.rs_group = int(os.environ.get("YTK_RS_GROUP", "4"))  # features per tail block (2 | 4 | 8)
        ng8 = -(-F // self.rs_group)
        self.fuse_rs = (not self.comm.is_dist and not self.wide and not self.fuse_split_plan
                        and bins.dtype == torch.uint8 and B <= 256 and F <= 256
                        and os.environ.get("YTK_HIST_STAGED", "1") != "0" and _ext.HIST_FW == 32
                        and (ng8 == 1 or (ng8 - 1) * -(-F // ng8) < F)
                        and os.environ.get("YTK_FUSE_REDUCE_SPLIT", "0") == "1")
        if self.fuse_rs:
            self.rs_split = int(os.environ.get("YTK_REDUCE_SPLIT", "8"))  # split-K factor (exact sums)
            self.split_groups = ng8
            # YTK_RS_PROF=1: per-level block timestamps of the fused kernel (tools/dbg_rs_prof.py)
            self.rs_prof = None
            if os.environ.get("YTK_RS_PROF") == "1":
                nbx = -(-B // (1024 // self.rs_group)) * ng8 * self.rs_split
                self.rs_prof = [torch.zeros((self._half(max(1, c)) * nbx, 16), dtype=torch.int64, device=dev)
                                for c in range(D)]
            self.rs_cnt = torch.zeros(self.maxp * ng8 + 16, dtype=torch.int32, device=dev)
        self.split_out = torch.zeros(2 * self.maxp * 48 * self.split_groups, dtype=torch.uint8, device=dev)
        # split_find runs one block per (node, feature): per-feature candidates + per-item
        # arrival counters (reset by the combining block)
        self.split_part = torch.zeros(2 * self.maxp * F * 48, dtype=torch.uint8, device=dev)
        self.split_cnt = torch.zeros(2 * self.maxp, dtype=torch.int32, device=dev)
        self.root_cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        # Histogram slots. Level c (children at depth c, 1 <= c < D) owns `half = 2^(c-1)`
        # built slots, then `ncs` count slots, then `half` derived slots; the root is slot 0.
        # The fused partition kernel's cursors sit a cache line apart (CUR_STRIDE words per
        # split) followed by its self-resetting done counters, all inside the count slots.
        slot_elems = B * F * 2
        cnt_words = (self.maxp * CUR_STRIDE + DONE_WORDS) if self.fuse_part_children else self.maxp
        self.ncs = -(-cnt_words // slot_elems) if self.fuse_counts else 0
        self.level_slots = {}
        nxt = 1
        for c in range(1, D):
            half = self._half(c)
            self.level_slots[c] = (nxt, nxt + half, nxt + half + self.ncs)  # build, count, derived
            nxt += 2 * half + self.ncs
        self.n_slots = max(1, nxt)
        # histogram_pool_capacity (HistogramPool.java:36-273 bounds the live histograms): a pool
        # below the full slab alternates odd and even levels between two regions -- a level
        # only ever subtracts from its parents' level -- and zeroes each level's built slots
        # before it accumulates into them (level_slots_pingpong)
        self.pingpong = pool_slots is not None and self.n_slots > pool_slots
        if self.pingpong:
            reg = [0, 0]
            for c in range(1, D):
                reg[c % 2] = max(reg[c % 2], 2 * self._half(c) + self.ncs)
            for c in range(1, D):
                b0 = 1 if c % 2 == 1 else 1 + reg[1]
                half = self._half(c)
                self.level_slots[c] = (b0, b0 + half, b0 + half + self.ncs)
            self.n_slots = 1 + reg[0] + reg[1]
            if self.n_slots > pool_slots:
                raise ValueError(f"histogram pool of {pool_slots} slots below the level engine's two live "
                                 f"levels ({self.n_slots} slots)")
        self.hist = torch.zeros((self.n_slots, B, F, 2), dtype=torch.int64, device=dev)
        # owner-computes sync (TreeParams.hist_sync): reduce-scatter by feature block (the
        # level's count slots ride along in every rank's block), split search on the owned
        # features, allgather of the 48-B records, device-side argmax (split_combine)
        if self.owner:
            self.fr, self.fblocks = self.comm.feature_blocks(F)
            self.own = self.fblocks[self.comm.rank]
            self.split_local = torch.zeros(2 * self.maxp * 48, dtype=torch.uint8, device=dev)
            self._own_cache = {}
            self._pack = None
            self._allr = None
        self._slot_bytes = slot_elems * 8
        self._root_fixed = False
        # staged histogram flush: block partials to a staging slab with plain stores, then a
        # split-K slot reduce (8 int64 atomics per value instead of one per block)
        max_hist_items = self.hist_target + (self.maxp // 2) + 2
        self.staged = os.environ.get("YTK_HIST_STAGED", "1") != "0"
        # multi-GPU: overlap the all-reduce of half a level's histograms with the build of
        # the other half (BASELINE: histogram all-reduce overlapped with the next block's build)
        # Only with enough local rows: at a small shard (strong scaling, e.g. Higgs / 8) a
        # level's build is ~10-20 us, less than the launch latency of the second collective.
        self.overlap = (os.environ.get("YTK_HIST_OVERLAP", "1") != "0"
                        and self.N >= int(os.environ.get("YTK_HIST_OVERLAP_MIN_ROWS", "2000000")))
        # single-node multi-GPU (default; YTK_PEER_REDUCE=0: RCCL): every level message -- and
        # the round's loss vector (trainer) -- is ONE peer-memory exchange kernel
        # (parallel/peer.py) instead of an RCCL call; owner mode: the level's reduce-scatter by
        # feature block and the split-record all-gather are one kernel each. Stream-ordered and
        # host-free, so the half-level overlap is not needed, and a round whose collectives are
        # all peer exchanges can be graph-captured on any process-group backend.
        self.peer = None
        if self.comm.is_dist:
            lvl = max([1] + [self.level_slots[c][2] - self.level_slots[c][0] for c in self.level_slots]) * slot_elems
            cap = max(lvl, slot_elems, self.maxp * CUR_STRIDE + DONE_WORDS, 4 + self.max_nodes)
            if self.owner:  # the largest packed level ([P][build slots x own block + count slots])
                P = self.comm.world
                nb = max([1] + [self._half(c) for c in range(1, D)])
                cap = max(cap, P * (nb * B * self.fr * 2 + self.ncs * B * F * 2) + 2 * P,
                          P * self.split_local.numel() // 8)
            self.peer = peer_mod.make(self.comm, cap)
            if self.peer is not None:
                self.overlap = False
        # peer path: levels with >= 8 built slots may exchange their first half on a side stream
        # (a second peer group, a small exchange grid that fits beside the histogram blocks)
        # while the second half's histograms build; the split waits for both (BASELINE:
        # histogram exchange overlapped with the next block's build).
        # YTK_PEER_OVERLAP=auto (default): measured per job -- trees 1..4 (eager rounds, before
        # any graph capture) alternate overlap off / on with device events around each build,
        # the ranks agree on the max-over-ranks times and the faster mode builds the rest
        # (overlap_tune()). Whether it pays depends on the shard (the second half's build must
        # outlast the exchange) and on the links, so it is not decided blind. Ranks sharing one
        # GPU (a rehearsal) never overlap under auto: their exchanges contend with each other's
        # builds (auto_force: tune there too -- tests). 1: always on, 0: never.
        self.peer2 = None
        self.peer_overlap = False
        self.overlap_mode = os.environ.get("YTK_PEER_OVERLAP", "auto")
        auto = self.overlap_mode in ("auto", "auto_force")
        self.overlap_trial = None  # auto: [(tree, on, start event, end event)], then None
        self.overlap_times = None  # auto: (off us, on us) per tree, max over ranks
        if (self.peer is not None and not self.owner and self.staged and (auto or self.overlap_mode == "1")
                and not (self.overlap_mode == "auto" and getattr(self.peer, "shared_gpu", False))):
            half_max = max([1] + [self._half(c) // 2 for c in range(1, D)])
            if half_max >= 4:
                self.peer2 = peer_mod.make(self.comm, half_max * slot_elems)
                if self.peer2 is not None:
                    hip().peer_set_grid_cap(self.peer2.hnd, int(os.environ.get("YTK_PEER_OVERLAP_GRID", "32")))
                    self._side = torch.cuda.Stream(device=dev)
                    self.peer_overlap = self.overlap_mode == "1"
                    if auto:
                        self.overlap_trial = []
        self.staging = (torch.empty(max_hist_items * hist_cols(F) * B * 2, dtype=torch.int64, device=dev)
                        if self.staged else None)
        # small slabs are zeroed whole once per tree; a ping-pong slab reuses its regions within
        # the tree, so every level zeroes its own built slots
        self._zero_all = self.hist.numel() * 8 <= (64 << 20) and not self.pingpong
        self._slab_zeroed = False  # the whole slab was zeroed at the end of the previous tree
        # YTK_ZERO_AT_END=1: zero the slab with a fill launch at the end of each tree (instead of
        # in the next gradient pass)
        self._zero_at_end = os.environ.get("YTK_ZERO_AT_END") == "1"
        self._raw_req = None       # test-set raw tree written by the tree tail (set_raw_request)
        self._raw_ready = False
        # True: each tree's snapshot is a copy (K trees per round need their own); the
        # trainer clears it for K == 1 -- the round reads the snapshot (gradient pass,
        # host readback) before the next tree overwrites it, in stream order
        self.snapshot_copy = True
        self.rows = torch.empty(self.N, dtype=torch.int32, device=dev)
        self.rows_tmp = torch.empty(self.N, dtype=torch.int32, device=dev)
        self.ghp = torch.empty((self.N, 2), dtype=torch.float32, device=dev)
        self.gh_tmp = torch.empty((self.N, 2), dtype=torch.float32, device=dev)
        self.flags = torch.empty(self.N, dtype=torch.uint8, device=dev)
        # levels [0, PART_SCAN_LEVELS) of the fused partition reserve their chunks through a
        # count pass + one-block scan instead of the split cursor atomics (the root level's
        # 5127 Higgs chunks on ONE cursor line serialise ~62 us): root partition 77 -> 30 us,
        # 1.248 -> 1.219 / 1.215 / 1.219 ms per tree with 1 / 2 / 3 levels
        # (profiles/r6/part_scan/); YTK_PART_SCAN_LEVELS=0: off
        self.part_scan_levels = min(int(os.environ.get("YTK_PART_SCAN_LEVELS", "2")), 8)
        # a small shard's few chunks contend little (1/8 of Higgs: 641 root chunks, ~8 us of
        # serialised atomics) and the count + scan launches cost ~19 us: 0.393 -> 0.397 ms
        if self.N < int(os.environ.get("YTK_PART_SCAN_MIN_ROWS", 4_000_000)):
            self.part_scan_levels = 0
        # per-chunk counts (<= max_blocks of a level) then their sums per 32 chunks (zero between
        # levels: the partition's last block re-zeroes them)
        cap = self.N // 2048 + self.maxp + 4
        self.chunk_io = (torch.zeros(cap + cap // 32 + 8, dtype=torch.int64, device=dev)
                         if self.part_scan_levels > 0 else None)
        self.scales = torch.ones(2, dtype=torch.float32, device=dev)
        self.inv_scales = torch.ones(2, dtype=torch.float64, device=dev)
        self.gp = p.gain_params()
        self.ip = [p.max_depth, p.max_leaf_cnt, p.min_split_samples, self.hist_target, self.part_target,
                   self.MIN_ROWS, self.part_chunk, self.split_groups, 0]  # [8]: small_only (per build)
        self._ip_cur = self.ip
        self.tree_count = 0
        # set by the trainer when its fused gradient pass counts the rows per leaf
        # (tree_grad leaf_counts): the last level then needs no counting partition and no
        # count all-reduce -- its children are leaves, and only their sample counts were
        # still missing
        self.defer_leaf_counts = False
        # set by the trainer when its K == 1 gradient pass also builds the NEXT tree's root
        # histogram (tree_grad_hist): the root slot then arrives pre-built (root_ready) and
        # is zeroed again at the end of every tree for the next pass to accumulate into
        self.fuse_root = False
        self.root_ready = False
        self._root_bufs = None
        self.last_keep = None
        self.total_stats = TimeStats()
        self._fmask_cache = {}

    def _half(self, c: int) -> int:
        """Built-child slots of level c: at most one per split of level c - 1."""
        return min(1 << (c - 1), max(1, self.maxp // 2))

    @staticmethod
    def supports(bins: torch.Tensor, binsT: Optional[torch.Tensor], B: int, F: int) -> bool:
        """Bin layouts the device kernels handle: uint8 row-major bins (B <= 256, 32-aligned
        stride) for the 32-feature LDS histogram, or uint16 bins + a contiguous column-major
        binsT with one feature's planes within the LDS budget for the wide kernel."""
        if bins.dtype == torch.uint8:
            stride = bins.shape[1]
            return B <= 256 and stride % 32 == 0 and stride >= ((F + 31) // 32) * 32
        if bins.dtype == torch.int16:
            fg = gops.wide_group(B, F)
            return (binsT is not None and binsT.dtype == torch.int16 and binsT.shape[0] == F
                    and binsT.is_contiguous() and fg > 0 and bins.shape[1] % fg == 0 and bins.is_contiguous())
        return False

    def _snap_views(self, buf):
        out, off = [], 0
        dts = [torch.int32, torch.uint8, torch.int32, torch.int32, torch.int32, torch.int32, torch.float32]
        for sz, dt in zip(self._snap_sizes, dts):
            out.append(buf[off:off + sz].view(dt))
            off += sz
        return out

    def _fp(self):
        p = self.p
        return [float(np.float32(v)) for v in (p.min_split_loss, p.min_child_hessian_sum, p.l1, p.l2,
                                              p.max_abs_leaf_val, p.learning_rate)]

    def _count_ptr(self, c: int) -> int:
        """Device address of level c's count slots (fused-count mode)."""
        return ptr(self.hist) + self.level_slots[c][1] * self._slot_bytes

    def _ptrs(self, loc: int = None, glob: int = None):
        out = [ptr(t) for t in (self.st, self.nodes, self.pending, self.next_pending, self.split_nid,
                                self.split_snap, self.part_items, self.part_feat, self.part_thr,
                                self.part_begin, self.part_first, self.part_nblk, self.part_counts,
                                self.left_loc, self.left_glob, self.hist_items, self.split_items,
                                self.item_nid, self.split_out, self.tfeat, self.tthr, self.tleft,
                                self.tright, self.tval, self.root_cnt, self.part_cnt, self.hist_first)]
        if loc is not None:
            out[13] = loc
        if glob is not None:
            out[14] = glob
        return out

    # ------------------------------------------------------------------ overlap auto-tune
    OVERLAP_TRIAL = (1, 2, 3, 4)  # trees timed (tree 0 warms up): off, on, off, on

    @property
    def tuning(self) -> bool:
        """True while the overlap auto-tune still needs eager (uncaptured) trees."""
        return self.overlap_trial is not None

    def _trial_begin(self):
        """Auto-tune: the mode of this tree and its start event (None outside the trial)."""
        if self.overlap_trial is None or self.tree_count not in self.OVERLAP_TRIAL:
            return None
        self.peer_overlap = (self.tree_count - self.OVERLAP_TRIAL[0]) % 2 == 1
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.dev))
        return ev

    def _trial_end(self, ev0):
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record(torch.cuda.current_stream(self.dev))
        self.overlap_trial.append((self.tree_count, self.peer_overlap, ev0, ev1))
        if len(self.overlap_trial) == len(self.OVERLAP_TRIAL):
            self._trial_decide()

    def _trial_decide(self):
        """The faster mode over the trial trees (device time, max over ranks: the slowest
        rank sets the pace), identical on every rank."""
        off = on = 0.0
        for _, o, e0, e1 in self.overlap_trial:
            e1.synchronize()
            t = 1000.0 * e0.elapsed_time(e1)
            if o:
                on += t
            else:
                off += t
        off, on = self.comm.allreduce_scalars([off, on], op="max")
        n = len(self.OVERLAP_TRIAL) // 2
        self.overlap_times = (round(off / n, 1), round(on / n, 1))
        self.peer_overlap = on < off
        self.overlap_trial = None

    def _hist_allreduce(self, t: torch.Tensor):
        """A level's histogram (+ count) slots (or any int64 / fp64 device message): the
        peer-memory exchange kernel, or RCCL."""
        if self.peer is not None:
            self.peer.allreduce_(t.view(-1))
        else:
            self.comm.allreduce_(t)

    def close(self):
        """Release the peer-memory groups (collective: every rank calls it)."""
        if self.peer is not None:
            self.peer.close()
            self.peer = None
        if self.peer2 is not None:
            self.peer2.close()
            self.peer2 = None

    def _owner_reduce(self, base: int, nslots: int, ncs: int = 0):
        """Reduce-scatter slots [base, base + nslots) by feature block (+ the ncs count slots
        that follow them, replicated into every block so every rank gets their sums)."""
        P, fr, B, F = self.comm.world, self.fr, self.B, self.F
        nb_el = nslots * B * fr * 2
        C = ncs * B * F * 2
        # persistent pack / result buffers sized for the largest level (no per-level alloc)
        need = P * (nb_el + C)
        if self._pack is None or self._pack.numel() < need:
            self._pack = torch.empty(need, dtype=torch.int64, device=self.dev)
            self._pack_out = torch.empty(need // P, dtype=torch.int64, device=self.dev)
        x = self._pack[:need].view(P, nb_el + C)
        out = self._pack_out[:nb_el + C]
        s = stream(self.bins)
        h = hip()
        slot_ptr = ptr(self.hist) + base * self._slot_bytes
        cnt_ptr = slot_ptr + nslots * self._slot_bytes if C else 0
        h.owner_pack(slot_ptr, ptr(x), nslots, B, F, fr, P, cnt_ptr, C, s)  # one launch
        if self.peer is not None and self.peer.fits_segments(x.view(-1)):
            out = self.peer.reduce_scatter_(x.view(-1))  # one kernel, this rank's block in place
        else:
            self.comm.reduce_scatter_(out, x)
        h.owner_unpack(ptr(out), slot_ptr, nslots, B, F, fr, self.comm.rank, cnt_ptr, C, s)

    def _owner_fmask(self, fmask_np: np.ndarray):
        """(owned sampled-feature mask on the device, its first feature, totals rank)."""
        key = fmask_np.tobytes()
        if key not in self._own_cache:
            lo, hi = self.own
            fm = fmask_np.copy()
            fm[:lo] = 0
            fm[hi:] = 0
            nz = np.flatnonzero(fm)
            f0 = int(nz[0]) if nz.size else (lo if hi > lo else 0)
            tot = next(r for r, (a, b) in enumerate(self.fblocks) if b > a and fmask_np[a:b].any())
            if len(self._own_cache) > 64:
                self._own_cache.clear()
            self._own_cache[key] = (torch.from_numpy(fm).to(self.dev), f0, tot)
        return self._own_cache[key]

    def _split(self, fmask, f0: int, fmask_np: np.ndarray, nitems: int, nitems_dev: int, s):
        """Split search over the items (all-reduce mode: every feature; owner mode: the
        owned features, then allgather + device argmax into split_out)."""
        gp, h = self.gp, hip()
        out = self.split_out
        if self.owner:
            fmask, f0, tot = self._owner_fmask(fmask_np)
            out = self.split_local
        if self.split_groups > 1 and not self.owner:
            if h.split_node_grouped(ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fmask), f0,
                                    ptr(self.split_items), nitems, ptr(out), gp["mcw"], gp["l1"], gp["l2"],
                                    gp["max_abs_leaf"], nitems_dev, ptr(self.inv_scales), self.split_groups, s):
                return
            raise RuntimeError("split_node_grouped: node-resident split search does not apply "
                               f"(B={self.B}, F={self.F}); set YTK_SPLIT_GROUPS=1")
        h.split_find(ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fmask), f0,
                     ptr(self.split_items), nitems, ptr(out), gp["mcw"], gp["l1"], gp["l2"],
                     gp["max_abs_leaf"], 1.0, 1.0, nitems_dev, ptr(self.inv_scales), ptr(self.split_part),
                     ptr(self.split_cnt), s)
        if self.owner:
            if self.peer is not None:  # the records' all-gather as one peer kernel
                if self._allr is None:
                    self._allr = torch.zeros(self.comm.world * self.split_local.numel(), dtype=torch.uint8,
                                             device=self.dev)
                n = self.split_local.numel()
                allr = self._allr
                allr[self.comm.rank * n:(self.comm.rank + 1) * n].copy_(self.split_local)
                self.peer.allgather_(allr.view(torch.int64))
            else:
                allr = self.comm.allgather(self.split_local)
            cap = self.split_local.numel() // 48
            h.split_combine(ptr(allr), self.comm.world, cap, nitems_dev, min(nitems, cap), tot,
                            ptr(self.split_out), s)

    def _split_plan(self, ptrs, fp, fmask, f0: int, nitems: int, s):
        """One GPU: this level's split search fused with the next level's split planning
        (lv_split_plan_kernel: the last node block plans) -- one launch instead of two."""
        gp = self.gp
        hip().lv_split_plan(ptrs, self._ip_cur, fp, ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fmask),
                            f0, nitems, [gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"]], ptr(self.inv_scales),
                            ptr(self.split_part), ptr(self.split_cnt), 1 if self.part_atomic else 0, self.maxp, s)

    def _fmask(self, rng):
        p = self.p
        if p.feature_sample_rate < 1.0:
            n_sam = max(1, int(round(p.feature_sample_rate * self.F)))
            perm = rng.permutation(self.F)
            fm = np.zeros(self.F, np.uint8)
            fm[np.sort(perm[:n_sam])] = 1
        else:
            fm = np.ones(self.F, np.uint8)
        key = fm.tobytes()
        if key not in self._fmask_cache:
            if len(self._fmask_cache) > 64:
                self._fmask_cache.clear()
            self._fmask_cache[key] = torch.from_numpy(fm).to(self.dev)
        self._fmask_np = fm
        return self._fmask_cache[key], int(np.nonzero(fm)[0][0])

    # ------------------------------------------------------------------ build
    def build(self, gh: torch.Tensor, ghmax: torch.Tensor = None, ghmax_global: bool = False) -> DeviceTree:
        """Enqueue one tree. ``gh`` [N, 2] contiguous (g, h); ``ghmax`` (float32 [2], optional)
        = max |g|, max |h| over all local rows, already produced by the gradient kernel."""
        trial = self._trial_begin()
        dt = self._build(gh, ghmax, ghmax_global)
        if trial is not None:
            self._trial_end(trial)
        return dt

    def _build(self, gh: torch.Tensor, ghmax: torch.Tensor = None, ghmax_global: bool = False) -> DeviceTree:
        p = self.p
        h = hip()
        s = stream(self.bins)
        fp = self._fp()
        rng = np.random.default_rng((p.seed, self.tree_count))
        seed_rows = int(rng.integers(1 << 62))
        dist = self.comm.is_dist
        sampled = p.instance_sample_rate < 1.0
        assert gh.is_contiguous() and gh.shape == (self.N, 2)
        # small_only: the last level is not partitioned (deferred leaf counts), so the level
        # before it writes only the rows of the children that get histograms
        # (YTK_SMALL_ONLY=0: both children, as on every other level)
        small_only = (self.defer_leaf_counts and not sampled and self.fuse_part_children
                      and os.environ.get("YTK_SMALL_ONLY", "1") != "0")
        ip = self._ip_cur = self.ip[:8] + [1 if small_only else 0]
        # gh_rows: the root partition moves only the row ids and the first gathered level
        # (its histograms and its partition) reads (g, h) by row id from the caller's array:
        # one full (g, h) read + write less per tree (YTK_GH_ROWS=0: moved at the root too)
        gh_mode = os.environ.get("YTK_GH_ROWS", "2")
        gh_rows = (not sampled and self.fuse_part_children and not self.wide and self.staged and p.max_depth >= 3
                   and gh_mode != "0" and os.environ.get("YTK_PART_PREFETCH", "2") != "0")
        # gh_all (YTK_GH_ROWS=2, default): (g, h) is never moved -- every partition moves the
        # row ids only (5 B read + 4 B written per row instead of 13 + 12) and every histogram
        # level gathers (g, h) by row id next to the row's bins (the leaf-wise engine's layout)
        gh_all = gh_rows and gh_mode == "2"
        # rows / position-ordered (g, h). Without sampling the root level reads the identity
        # permutation and the caller's gh directly; the first partition writes the buffers.
        if sampled:
            g = torch.Generator(device=self.dev)
            g.manual_seed(seed_rows + self.comm.rank)
            keep = torch.rand(self.N, generator=g, device=self.dev) < p.instance_sample_rate
            # stable compaction without a host sync: sampled rows first, in order
            key = (~keep).to(torch.int32)
            _, order = torch.sort(key, stable=True)
            self.rows.copy_(order.to(torch.int32))
            self.ghp.copy_(gh.index_select(0, order))
            self.root_cnt[0] = keep.sum()
            self.last_keep = keep
            rows0, gh0 = ptr(self.rows), ptr(self.ghp)
        else:
            self.last_keep = None
            rows0, gh0 = 0, ptr(gh)
        fmask, f0 = self._fmask(rng)
        if sampled:
            self.root_cnt[1] = self.root_cnt[0]
            if dist:
                self.comm.allreduce_(self.root_cnt[1:2])
            self._root_fixed = False
        elif not self._root_fixed:
            # unsampled: (local, global) row counts are constants -- set once, not per tree
            self.root_cnt[0] = self.N
            self.root_cnt[1] = self.N
            if dist:
                self.comm.allreduce_(self.root_cnt[1:2])
            self._root_fixed = True
        # fixed-point scales from the global max |g|, |h| over the tree's rows
        if ghmax is not None and ghmax_global:  # a global bound: identical on every rank
            mx = ghmax
        elif sampled:
            mx = (gh.abs() * keep[:, None]).amax(dim=0)
        elif ghmax is not None:
            mx = ghmax
        else:
            mx = gh.abs().amax(dim=0)
        if dist and not ghmax_global:
            mx = mx.clone()
            self.comm.allreduce_(mx, op="max")
        tm = self.timer
        # root (+ the tree's fixed-point scales in the same launch)
        ptrs = self._ptrs()
        st_ptr = self.st.data_ptr()
        off = lambda w: st_ptr + 4 * w
        h.lv_init_scales(ptrs, ip, fp, ptr(mx), ptr(self.scales), ptr(self.inv_scales), s)
        tm.mark("init_stats")

        # YTK_REDUCE_KNOWN=0: the slot reduce scans the work list for each slot's items instead
        # of reading the ranges the children planner wrote (hist_first) / the root's one slot
        known = os.environ.get("YTK_REDUCE_KNOWN", "1") != "0"

        def build_hist(gh_ptr, rows_ptr, nitems, slot_base, nslots, n_dev=None, work_off=0, by_row=0, first=0):
            if self._zero_all:
                if slot_base == 0:
                    self.hist.zero_()  # every slot of the tree in one fill (small slabs)
            else:
                self.hist[slot_base:slot_base + nslots].zero_()
            if self.wide:
                # row-major uint16 rows (one vector load per row and feature group), staged
                # flush + split-K reduce into the level's slots
                h.hist_wide_rm(ptr(self.bins), self.bins.shape[1], self.F, gh_ptr, rows_ptr, ptr(self.hist_items),
                               nitems, ptr(self.hist), self.B, 1.0, 1.0, off(5) if n_dev is None else n_dev,
                               ptr(self.scales), work_off, ptr(self.staging) if self.staged else 0, slot_base,
                               nslots, ptr(self.binsT), self.binsT.shape[1], s)
                return
            if self.staged:
                h.hist_fx_staged(ptr(self.bins), self.bins.shape[1], self.F, gh_ptr, rows_ptr,
                                 ptr(self.hist_items), nitems, ptr(self.hist), self.B, 1.0, 1.0,
                                 off(5) if n_dev is None else n_dev, ptr(self.scales), ptr(self.staging),
                                 slot_base, nslots, 0, work_off, s, by_row, first if known else 0,
                                 1 if (known and slot_base == 0 and nslots == 1) else 0)
                return
            assert not by_row, "row-indexed (g, h) needs the staged histogram kernel"
            h.hist_fx(ptr(self.bins), self.bins.shape[1], self.F, gh_ptr, rows_ptr, ptr(self.hist_items),
                      nitems, ptr(self.hist), self.B, 1.0, 1.0, off(5), ptr(self.scales), s)

        if self.root_ready and not sampled:
            # the root histogram came with the previous round's gradient pass (the other
            # slots were zeroed with the root slot at the end of the previous tree)
            if self._zero_all and not self._slab_zeroed:
                self.hist[1:].zero_()
        else:
            build_hist(gh0, rows0, self.hist_target + 1, 0, 1)
        self.root_ready = False
        tm.mark("build_hist_compute")
        if dist:
            if self.owner:
                self._owner_reduce(0, 1)
            else:
                self._hist_allreduce(self.hist[0:1])
            tm.mark("build_hist_comm")
        if self.fuse_split_plan:
            self._split_plan(ptrs, fp, fmask, f0, 1, s)
        else:
            self._split(fmask, f0, self._fmask_np, 1, off(6), s)
        tm.mark("find_best_split")
        bb = 1 if self.bins.dtype == torch.uint8 else 2
        fused = self.fuse_counts
        tail_children = None
        for d in range(p.max_depth):
            c = d + 1  # depth of the children created at this level
            last = c == p.max_depth
            if fused:
                # split counters of this level accumulate into level c's count slots; the
                # previous level's (all-reduced) count slots patch cnt_global of depth d
                loc = self.left_loc if last else None
                ptrs = self._ptrs(loc=ptr(loc) if loc is not None else self._count_ptr(c),
                                  glob=self._count_ptr(d) if d >= 1 else None)
            # apply splits + pop depth d (arg0 = 1: the single-pass partition needs no work list)
            if not self.fuse_split_plan:  # else: planned by the previous split launch
                # the previous level's counts: line-spaced cursors when its partition was fused
                patch = (2 if self.fuse_part_children else 1) if (fused and d >= 1) else 0
                h.lv_step(1, ptrs, ip, fp, 1 if self.part_atomic else 0, patch, s)
            tm.mark("plan")
            if last and self.defer_leaf_counts and not sampled:
                # children planning with zero cursors: the leaves' sample counts are placeholders
                # until the round's gradient pass (tree_grad) has walked every row to its leaf;
                # run by the tree-tail launch below together with finalize + raw tree
                tail_children = self._half(c) | (1 << 30)
                break
            npart = self.part_target + min(1 << d, self.maxp) + 1
            lloc = ptrs[13]
            rows_in = rows0 if d == 0 else ptr(self.rows)
            gh_in = gh0 if d == 0 else ptr(self.ghp)
            part_gh_rows = 0
            if gh_rows and (d == 0 or gh_all):
                gh_in = 0  # the partition moves the row ids only
            elif gh_rows and d == 1:
                gh_in, part_gh_rows = gh0, 1  # (g, h) by row id; this level writes it in position order
            half = self._half(c)
            if last:
                base, ncs = 0, 0  # no histograms at the last level
            else:
                base, cbase, dbase = self.level_slots[c]
                ncs = dbase - cbase
            # partition + children planning in one launch (last block plans); multi-GPU: not on
            # the last level, whose counts need their own all-reduce before the planning
            fused_part = self.fuse_part_children and not (dist and last)
            if fused_part:
                scan = self.chunk_io is not None and d < self.part_scan_levels and bb == 1 and not last
                h.lv_partition_children(ptrs, ip, fp, ptr(self.binsT), self.binsT.shape[1], rows_in, gh_in,
                                        ptr(self.rows_tmp), ptr(self.gh_tmp) if gh_in else 0, npart,
                                        1 if last else 0, base,
                                        half | (ncs << 14) | ((1 if fused else 0) << 29) | (1 << 30),
                                        self.maxp, s, bb, part_gh_rows, ptr(self.chunk_io) if scan else 0)
                tm.mark("partition")
            # the flag kernel also accumulates the per-split left totals into left_loc
            elif self.part_atomic:
                # the split cursors are the (zeroed) per-split left counters: low half = left
                # rows, high half = right rows; the last level only counts
                h.partition_atomic(ptr(self.binsT), bb, self.binsT.shape[1], rows_in, ptr(self.rows_tmp),
                                   gh_in, ptr(self.gh_tmp) if gh_in else 0, ptr(self.part_first), off(3), off(4), npart,
                                   ptr(self.part_feat), ptr(self.part_thr), ptr(self.part_begin),
                                   ptr(self.part_cnt), lloc, 1 if last else 0, 0, s)
            elif last:
                h.partition_count(ptr(self.binsT), bb, self.binsT.shape[1], rows_in, ptr(self.flags),
                                  ptr(self.part_items), npart, ptr(self.part_feat), ptr(self.part_thr),
                                  ptr(self.part_counts), off(4), lloc, s)
            else:
                h.partition(ptr(self.binsT), bb, self.binsT.shape[1], rows_in, ptr(self.rows_tmp),
                            gh_in, ptr(self.gh_tmp) if gh_in else 0, ptr(self.flags), ptr(self.part_items), npart,
                            ptr(self.part_feat), ptr(self.part_thr), ptr(self.part_begin),
                            ptr(self.part_first), ptr(self.part_nblk), ptr(self.part_counts), 0, off(4),
                            lloc, s)
            if not fused_part:
                tm.mark("partition")
                lvl_fused = fused and not last
                if dist and not lvl_fused:
                    self.left_glob.copy_(self.left_loc)
                    self._hist_allreduce(self.left_glob)
                    tm.mark("sync_counts")
                use_loc = (not dist) or lvl_fused
                if fused and last:  # the last level reads the separately all-reduced counts
                    ptrs = self._ptrs()
                h.lv_step(3, ptrs, ip, fp, base,
                          half | (ncs << 14) | ((1 if lvl_fused else 0) << 29) | ((1 if use_loc else 0) << 30), s)
                tm.mark("plan")
            if last:
                break
            self.rows, self.rows_tmp = self.rows_tmp, self.rows
            self.ghp, self.gh_tmp = self.gh_tmp, self.ghp
            ptrs = self._ptrs()
            nmax = self.hist_target + half + 1
            # the first gathered level reads (g, h) by row id from the caller's array (gh_rows)
            hgh, hrow = (gh0, 1) if (gh_rows and (d == 0 or gh_all)) else (ptr(self.ghp), 0)
            if dist and self.peer_overlap and half >= 8:
                # first half's exchange on the side stream (second peer group) overlaps the
                # second half's build; the split search waits for both
                hs = half // 2
                build_hist(hgh, ptr(self.rows), nmax, base, hs, n_dev=off(ST_N_HIST_A), by_row=hrow,
                           first=ptr(self.hist_first))
                main = torch.cuda.current_stream(self.dev)
                side = self._side
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    self.peer2.allreduce_(self.hist[base:base + hs].view(-1))
                build_hist(hgh, ptr(self.rows), nmax, base + hs, half - hs, n_dev=off(5),
                           work_off=off(ST_N_HIST_A), by_row=hrow, first=ptr(self.hist_first) + 4 * hs)
                tm.mark("build_hist_compute")
                self._hist_allreduce(self.hist[base + hs:base + half + ncs])
                main.wait_stream(side)
                tm.mark("build_hist_comm")
            elif dist and self.overlap and half >= 8 and self.staged and not self.owner:  # large levels only:
                # small ones are latency bound and a second collective would cost more
                # two node halves: the first half's all-reduce (RCCL, async) overlaps the
                # second half's histogram build; the split search waits for both
                hs = half // 2
                build_hist(hgh, ptr(self.rows), nmax, base, hs, n_dev=off(ST_N_HIST_A), by_row=hrow,
                           first=ptr(self.hist_first))
                work = self.comm.allreduce_(self.hist[base:base + hs], async_op=True)
                build_hist(hgh, ptr(self.rows), nmax, base + hs, half - hs, n_dev=off(5),
                           work_off=off(ST_N_HIST_A), by_row=hrow, first=ptr(self.hist_first) + 4 * hs)
                tm.mark("build_hist_compute")
                if work is not None:
                    work.wait()
                self.comm.allreduce_(self.hist[base + hs:base + half + ncs])
                tm.mark("build_hist_comm")
            elif self.fuse_rs:
                # block partials, then reduce + split search in one launch (no _split below)
                if not self._zero_all:
                    self.hist[base:base + half].zero_()
                h.hist_fx_stage(ptr(self.bins), self.bins.shape[1], self.F, hgh, ptr(self.rows),
                                ptr(self.hist_items), nmax, self.B, off(5), ptr(self.scales), ptr(self.staging), s,
                                hrow)
                tm.mark("build_hist_compute")
                gp = self.gp
                h.lv_reduce_split(self._ptrs(), ptr(self.staging), ptr(self.hist), self.B, self.F, base, half,
                                  ptr(self.nbins_f), ptr(fmask), f0,
                                  [gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"]], ptr(self.inv_scales),
                                  ptr(self.rs_cnt), self.rs_split, s,
                                  ptr(self.rs_prof[c]) if self.rs_prof is not None else 0, self.rs_group)
                tm.mark("find_best_split")
                continue
            else:
                build_hist(hgh, ptr(self.rows), nmax, base, half, by_row=hrow, first=ptr(self.hist_first))
                tm.mark("build_hist_compute")
                if dist:
                    # built slots (+ this level's count slots when fused): one collective
                    if self.owner:
                        self._owner_reduce(base, half, ncs)
                    else:
                        self._hist_allreduce(self.hist[base:base + half + ncs])
                    tm.mark("build_hist_comm")
            if self.fuse_split_plan:
                self._split_plan(ptrs, fp, fmask, f0, min(1 << c, self.maxp), s)
            else:
                self._split(fmask, f0, self._fmask_np, min(1 << c, self.maxp), off(6), s)
            tm.mark("find_best_split")
        # tree tail in one launch: [deferred children planning] + finalize + raw tree (when the
        # trainer registered its test-set request, set_raw_request)
        rq = self._raw_req
        ro = rq["out"] if rq is not None else None
        h.lv_tail(self._ptrs(), ip, fp, 1 if tail_children is not None else 0, 0,
                  tail_children if tail_children is not None else 0, self.max_nodes,
                  ptr(rq["cand"]) if rq else 0, ptr(rq["coff"]) if rq else 0, ptr(rq["fill"]) if rq else 0,
                  rq["median"] if rq else 0, ptr(ro["nfeat"]) if rq else 0, ptr(ro["nthr"]) if rq else 0,
                  ptr(ro["nleft"]) if rq else 0, ptr(ro["nright"]) if rq else 0, ptr(ro["ndefl"]) if rq else 0,
                  ptr(ro["nval"]) if rq else 0, s)
        self._raw_ready = rq is not None
        # fuse_root: the next gradient pass (tree_grad_hist, root_target()'s zero range) zeroes
        # the whole slab (small slabs) or slot 0 before it accumulates the next root into slot
        # 0 -- no fill launch here. When that pass does not run fused (root_ready stays False),
        # the next build's root histogram zeroes the slab itself.
        self._slab_zeroed = self.fuse_root and self._zero_all and not self._zero_at_end
        if self.fuse_root and self._zero_at_end:
            if self._zero_all:
                self.hist.zero_()
                self._slab_zeroed = True
            else:
                self.hist[0].zero_()
        tm.mark("plan")
        self.tree_count += 1
        snap = self.snap.clone() if self.snapshot_copy else self.snap
        st, nodes, *arrays = self._snap_views(snap)
        dt = DeviceTree(nodes, st, tuple(arrays), self.max_nodes, snap, self._snap_sizes[0])
        if not self.snapshot_copy:
            dt.snap_full, dt.rv_off = self._snap_full, self.rv_off
        return dt

    def round_vector(self, n: int) -> torch.Tensor:
        """float64 [n] device vector stored right behind the snapshot (n <= 4 + max_nodes)."""
        assert n <= 4 + self.max_nodes
        return self._snap_full[self.rv_off:self.rv_off + 8 * n].view(torch.float64)

    def swap_ping_pong(self):
        """One tree's net effect on the Python-side buffer assignment (the partition swaps
        rows / (g, h) with their ping-pong buffers once per split level). Used when the
        trainer leaves graph replay after an odd number of replayed trees."""
        if max(self.p.max_depth - 1, 0) & 1:
            self.rows, self.rows_tmp = self.rows_tmp, self.rows
            self.ghp, self.gh_tmp = self.gh_tmp, self.ghp

    def root_target(self):
        """Arguments of the fused gradient + root histogram pass (gops.tree_grad root=)."""
        if self._root_bufs is None:
            grid = hip().tree_grad_hist_grid(self.N)
            self._root_bufs = (torch.empty(grid * 256 * 32 * 2, dtype=torch.int64, device=self.dev),
                               torch.zeros(4 * grid, dtype=torch.int32, device=self.dev))
        stg, work = self._root_bufs
        zero_n = 0 if self._zero_at_end else (self.hist.numel() if self._zero_all else self.hist[0].numel())
        return {"slot": ptr(self.hist), "scales": ptr(self.scales), "staging": ptr(stg), "work": ptr(work),
                "B": self.B, "F": self.F, "zero": ptr(self.hist) if zero_n else 0, "zero_n": zero_n}

    def live_tree_views(self):
        """(node table, leaf-value array) the engine's raw_tree / next snapshot read."""
        return self.nodes, self.tval

    def set_raw_request(self, cand: torch.Tensor, coff: torch.Tensor, fill: torch.Tensor, split_median: bool):
        """Have every build() also write the raw-threshold tree (for test-set scoring) into
        persistent arrays, by its tree-tail launch; raw_tree() with the same tables then
        returns them without a launch."""
        mn = self.max_nodes
        out = {
            "nfeat": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "nthr": torch.empty(mn, dtype=torch.float32, device=self.dev),
            "nleft": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "nright": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "ndefl": torch.empty(mn, dtype=torch.uint8, device=self.dev),
            "nval": torch.empty(mn, dtype=torch.float32, device=self.dev),
        }
        self._raw_req = {"cand": cand, "coff": coff, "fill": fill, "median": 1 if split_median else 0, "out": out}
        self._raw_ready = False

    def raw_tree(self, cand: torch.Tensor, coff: torch.Tensor, fill: torch.Tensor, split_median: bool):
        """Raw-threshold arrays of the LAST built tree (for test-set scoring), one forest entry."""
        rq = self._raw_req
        if (self._raw_ready and rq["cand"] is cand and rq["coff"] is coff and rq["fill"] is fill
                and rq["median"] == (1 if split_median else 0)):
            return rq["out"]
        mn = self.max_nodes
        out = {
            "nfeat": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "nthr": torch.empty(mn, dtype=torch.float32, device=self.dev),
            "nleft": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "nright": torch.empty(mn, dtype=torch.int32, device=self.dev),
            "ndefl": torch.empty(mn, dtype=torch.uint8, device=self.dev),
            "nval": torch.empty(mn, dtype=torch.float32, device=self.dev),
        }
        hip().lv_raw_tree(self._ptrs(), mn, ptr(cand), ptr(coff), ptr(fill), 1 if split_median else 0,
                          ptr(out["nfeat"]), ptr(out["nthr"]), ptr(out["nleft"]), ptr(out["nright"]),
                          ptr(out["ndefl"]), ptr(out["nval"]), stream(self.bins))
        return out
