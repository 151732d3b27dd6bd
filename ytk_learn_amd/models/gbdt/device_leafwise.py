"""GPU-resident leaf-wise (loss-guided) tree builder: no host round trip inside a tree.

Same trees as :class:`.builder.TreeBuilder` with ``grow_policy="loss"`` (reference:
``J/optimizer/gbdt/DataParallelTreeMaker.java`` make() :104-115,219-295, priority queue by
lossChg; host equivalent ``csrc/native/leafwise.cpp``). The queue replay, the speculative
batch choice and the child bookkeeping run in the planner kernels of
``csrc/hip/gbdt_leafwise.hip``; partition / histogram / split reuse the level engine's
kernels with device-resident work counts. Per batch the host only ENQUEUES a fixed
launch sequence; it polls a done flag one batch behind (pinned copy + event), so the GPU
always has the next batch queued and never waits for the host.

Rows live in a 2N-entry ping-pong buffer: a partition writes a node's children into the
other half at the same positions (no copy-back of the partitioned segments). (g, h) moves
with the row ids so the histogram reads it in position order (measured: leaving it
row-indexed -- 9 instead of 25 B per partitioned row -- cut the partition by 22 % but
the histogram's extra gather cost more).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ...ops import gbdt as gops
from ...ops._ext import CUR_STRIDE, DONE_WORDS, hip, hist_cols, ptr, stream
from ...parallel import peer as peer_mod
from ...parallel.comm import Comm
from ...utils.timestats import PhaseTimer
from .builder import TimeStats, TreeParams, resolve_hist_sync
from .device_builder import DNODE_DTYPE, DeviceTree

LW_CAP_MAX = 2304      # speculative nodes per tree of the LDS-resident planner (kLwCap)
LW_LEAF_MAX = 512      # kLwLeafMax: max_leaf_cnt of the LDS-resident planner
# larger trees: the planner keeps its node arrays and queues in a global workspace
LW_CAP_MAX_BIG = 16384  # kLwCapBig
LW_LEAF_MAX_BIG = 4096  # kLwLeafMaxBig
LW_DONE = 8
LW_BATCHES, LW_EXPANDED, LW_OVERFLOW = 12, 13, 11
# st words read by the fixed-grid kernels
W_N_SPLIT, W_N_PBLK, W_N_HIST, W_N_SITEMS, W_N_BUILD, W_N_ZERO = 3, 4, 5, 6, 7, 14
PART_CHUNK = 2048      # rows per partition block (partition_atomic_kernel)
REDUCE_DIRECT = 16     # kReduceDirect: slots with <= 16 staged items are stored, not atomically added


class DeviceLeafBuilder:
    HIST_TARGET = int(os.environ.get("YTK_HIST_TARGET", 256))
    MIN_ROWS = int(os.environ.get("YTK_HIST_MIN_ROWS", 2048))
    REDUCE_Y = 8        # slot reduce: y blocks striding over the batch's multi-item slots
    # batches enqueued ahead of the done-flag check (capturing batches in HIP graphs was
    # measured: no gain -- the gaps between dependent kernels are on the device side)
    POLL_LAG = int(os.environ.get("YTK_LW_POLL_LAG", 2))
    POLL_TIMEOUT_S = 60.0
    # small-node subtrees (opt-in YTK_LW_SUB_ROWS > 0; single GPU, byte bins, F <= 32): batch
    # entries with <= SUB_ROWS rows are grown by one workgroup each (lw_subtree_kernel), up to
    # SUB_MAX more splits, through nodes whose path-minimum gain is >= SUB_ALPHA x the previous
    # tree's smallest split gain (speculative: the trees are identical whatever these are).
    # Off by default: one CU per subtree needs ~25-45 us per split, slower than the batch
    # pipeline at every setting measured (500 trees: 4.06 -> 5.1-24 ms, docs/performance.md)
    SUB_ROWS_DEFAULT, SUB_MAX_DEFAULT, SUB_ALPHA_DEFAULT = 0, 32, 1.0

    def __init__(self, bins: torch.Tensor, binsT: torch.Tensor, F: int, B: int, nbins_f: np.ndarray,
                 params: TreeParams, comm: Comm = None, timer: Optional[PhaseTimer] = None):
        if not self.supports(bins, binsT, B, F, params, comm):
            raise ValueError("device leaf-wise builder: unsupported configuration")
        p = params
        self.p = p
        self.timer = timer if timer is not None else PhaseTimer()
        self.bins, self.binsT = bins, binsT
        # uint16 bins (B > 256, e.g. the reference's 5000-bin run): row-major feature-group LDS
        # histograms (hist_wide_staged_dev), fewer work items per batch (one per group per CU)
        self.wide = bins.dtype == torch.int16
        if self.wide:
            groups = -(-F // gops.wide_group(B, F))
            self.HIST_TARGET = min(self.HIST_TARGET, max(8, gops.WIDE_HIST_BLOCKS // groups))
            # the slot reduce's y extent is REDUCE_Y x groups: one y block per group already
            # gives 14 x 40 x 8 blocks at 5000 bins (8 per group launched ~36k mostly idle ones)
            self.REDUCE_Y = max(1, self.REDUCE_Y // groups)
        self.dev = bins.device
        self.N = N = bins.shape[0]
        self.F, self.B = F, B
        self.comm = comm or Comm.local(self.dev)
        self.nbins_f = torch.from_numpy(np.asarray(nbins_f, np.int32)).to(self.dev)
        ml = p.max_leaf_cnt
        self.max_leaf = ml
        self.max_nodes = 2 * ml - 1
        self.cap = self.slots_needed(p)
        dev = self.dev
        i32 = lambda n: torch.zeros(max(1, n), dtype=torch.int32, device=dev)  # noqa: E731
        mn = self.max_nodes
        # snapshot buffer: st (64 B) | tree node table | scoring arrays (as the level engine)
        self._snap_sizes = [64, mn * DNODE_DTYPE.itemsize] + [4 * mn] * 5
        # snapshot + the trainer's round vector 16-B aligned behind it (one readback copy)
        snap_total = sum(self._snap_sizes)
        self.rv_off = (snap_total + 15) // 16 * 16
        self._snap_full = torch.zeros(self.rv_off + 8 * (4 + mn), dtype=torch.uint8, device=dev)
        self.snap = self._snap_full[:snap_total]
        self._raw_req = None   # test-set raw tree written by the tree-tail launch
        self._raw_ready = False
        self.snapshot_copy = True  # the trainer clears it for K == 1 rounds
        (self.st, self.tnodes, self.tfeat, self.tthr, self.tleft, self.tright,
         self.tval) = self._snap_views(self.snap)
        cap = self.cap
        self.nd_f64 = torch.zeros((5, cap), dtype=torch.float64, device=dev)  # G, H, gl, hl, cnt (as i64)
        self.nd_i32 = torch.zeros((11, cap), dtype=torch.int32, device=dev)
        self.nd_loss = torch.zeros(cap, dtype=torch.float32, device=dev)
        self.heap, self.batch = i32(ml + 8), i32(ml)
        self.part = torch.zeros((6, ml), dtype=torch.int32, device=dev)
        # split cursors a cache line apart + the partition kernel's done counters
        self.cursor = torch.zeros(ml * CUR_STRIDE + DONE_WORDS, dtype=torch.int64, device=dev)
        self.hist_bound = self.HIST_TARGET + ml + 2
        self.hist_items = i32(4 * self.hist_bound)
        self.build_ids = i32(ml + 1)
        self.zero_ids = i32(ml + 1)
        self.zero_range = i32(2 * (ml + 1))
        self.n_sitems = 2 * ml + 2
        self.split_items = i32(4 * self.n_sitems)
        self.item_sid = i32(self.n_sitems)
        # split search in feature groups (one block per (node, group); the planner keeps each
        # node's best record) -- as DeviceLevelBuilder, YTK_SPLIT_GROUPS (default 4)
        # owner-computes sync (TreeParams.hist_sync, multi-GPU): each batch reduce-scatters its
        # built slots by feature block (the split cursors ride in every block), every rank
        # searches its own features, and the 48-B split records are all-gathered and combined
        # on the device (split_combine) -- HistogramBuilder.java:95's reduceScatterArray
        self.owner = self.comm.is_dist and resolve_hist_sync(p.hist_sync, B * F * 16) == "owner"
        self.split_groups = 1 if self.owner else gops.split_groups(B, F)
        self.split_out = torch.zeros(self.n_sitems * 48 * self.split_groups, dtype=torch.uint8, device=dev)
        if self.owner:
            P = self.comm.world
            self.fr, self.fblocks = self.comm.feature_blocks(F)
            self.own = self.fblocks[self.comm.rank]
            self.split_local = torch.zeros(self.n_sitems * 48, dtype=torch.uint8, device=dev)
            self._allr = torch.zeros(P * self.n_sitems * 48, dtype=torch.uint8, device=dev)
            kmax = min(ml, LW_LEAF_MAX)  # batches hold <= 512 splits
            self._own_per = kmax * (B * self.fr * 2 + CUR_STRIDE)  # the largest segment
            self._own_x = torch.zeros(P * self._own_per, dtype=torch.int64, device=dev)
            self._own_out = torch.zeros(self._own_per, dtype=torch.int64, device=dev)
            self._own_cache = {}
        self.split_part = torch.zeros(self.n_sitems * F * 48, dtype=torch.uint8, device=dev)
        self.split_cnt = torch.zeros(self.n_sitems, dtype=torch.int32, device=dev)
        self.root_cnt = torch.zeros(2, dtype=torch.int64, device=dev)
        # histogram slots: one per speculative node (never recycled inside a tree)
        self.hist = torch.zeros((cap, B, F, 2), dtype=torch.int64, device=dev)
        self.slot_bytes = B * F * 16
        self.staging = torch.empty(self.hist_bound * hist_cols(F) * B * 2, dtype=torch.int64, device=dev)
        self.rows2 = torch.empty(2 * N, dtype=torch.int32, device=dev)
        # YTK_LW_GH_ROWS=1 (byte-B bins): (g, h) stays ROW-indexed through the tree -- the
        # partition moves row ids only (4 instead of 12 B per row, both ways) and the histogram
        # gathers (g, h) by row id, as the level engine's gh_all mode. Off by default: on the
        # 255-leaf Higgs tree the partition saves what the histogram gathers cost (late tree
        # partition 1164 -> 1057 us, histograms 678 -> 764 us; 500 trees 3.99 -> 4.05 ms,
        # profiles/r5/leaf_gh_rows_*)
        self.gh_rows = os.environ.get("YTK_LW_GH_ROWS", "0") == "1" and not self.wide
        # first batches (root: one split, then <= 2) reserve partition chunks by count + scan
        self.PART_SCAN = min(int(os.environ.get("YTK_LW_PART_SCAN", "2")), 8)
        if N < int(os.environ.get("YTK_PART_SCAN_MIN_ROWS", 4_000_000)):
            self.PART_SCAN = 0  # few chunks per split: the atomics contend little (level engine)
        # per-chunk counts (<= max_pblocks) then their sums per 32 chunks (kept zero between
        # batches by the partition's last block)
        cap = N // PART_CHUNK + ml + 4
        self.chunk_io = torch.zeros(cap + cap // 32 + 8, dtype=torch.int64, device=dev)
        self._ghr = 0  # the tree's row-indexed (g, h) (build)
        self.gh2 = (torch.empty((2 * N, 2), dtype=torch.float32, device=dev) if not self.gh_rows
                    else torch.empty((1, 2), dtype=torch.float32, device=dev))
        self.scales = torch.ones(2, dtype=torch.float32, device=dev)
        self.inv_scales = torch.ones(2, dtype=torch.float64, device=dev)
        self.gp = p.gain_params()
        self.max_pblocks = -(-N // PART_CHUNK) + ml + 1
        # done flag: the planner writes it straight into pinned host memory (no copy launch)
        self._done_host = torch.zeros(16, dtype=torch.int32).pin_memory()
        # [0] done flag, [1] batches planned, [2] split count of the last planned batch
        # (written by lw_plan)
        self._dh_np = self._done_host.numpy()
        self.idle_hook = None  # called once per tree while the host waits on the planner
        self._done_dev = hip().host_device_ptr(self._done_host.data_ptr())
        self.tree_count = 0
        self.last_keep = None
        self.last_batches = self.last_expanded = 0
        self.hist_miss = 0  # slots are never evicted on the device (TreeBuilder API parity)
        self.total_stats = TimeStats()
        self._fmask_cache = {}
        self._lr = float(np.float32(p.learning_rate))
        # YTK_LW_PROF=1: planner phase times + work counters accumulated on the device
        self.prof = (torch.zeros(32, dtype=torch.int64, device=dev)
                     if os.environ.get("YTK_LW_PROF") == "1" else None)
        self.SUB_ROWS = int(os.environ.get("YTK_LW_SUB_ROWS", self.SUB_ROWS_DEFAULT))
        self.SUB_MAX = int(os.environ.get("YTK_LW_SUB_MAX", self.SUB_MAX_DEFAULT))
        self.SUB_ALPHA = float(os.environ.get("YTK_LW_SUB_ALPHA", self.SUB_ALPHA_DEFAULT))
        self.sub_on = (self.SUB_ROWS > 0 and not self.comm.is_dist and not self.wide and F <= 32 and B <= 256)
        self.sub_words = i32(8)
        self.sub_list = i32(2 * ml)
        # max_leaf_cnt > 512: the planner's per-node arrays and queues in global memory
        ws = int(hip().lw_ws_bytes(self.cap, ml))
        self.plan_ws = torch.zeros(ws, dtype=torch.uint8, device=dev) if ws > 0 else None
        self._handle = hip().lw_create(self._ptrs(), self._ip(), self._fp())
        self._ghmax_buf = None
        # multi-GPU: one message per batch = its built slots + its split cursors (lw_msg)
        self.slot_elems = B * F * 2
        self.msg = (torch.empty(ml * (self.slot_elems + CUR_STRIDE), dtype=torch.int64, device=dev)
                    if self.comm.is_dist else None)
        # single-node multi-GPU (default; YTK_PEER_REDUCE=0: RCCL): each batch message is ONE
        # peer-memory exchange kernel that reads its size (built slots, split cursors) from the
        # planner's device words -- the batch loop is the N = 1 loop, no host wait per batch
        self.peer = None
        if self.comm.is_dist:
            cap = max(self.msg.numel(), self.slot_elems, 4 + self.max_nodes)
            if self.owner:
                cap = max(cap, self._own_x.numel(), self._allr.numel() // 8)
            self.peer = peer_mod.make(self.comm, cap)
        # the trainer's K == 1 gradient pass can build the next tree's root histogram (slot 0,
        # tree_grad_hist); it is zeroed again when a tree is done
        self.staged = True
        self.fuse_root = False
        self.root_ready = False
        self._zero_at_end = os.environ.get("YTK_ZERO_AT_END") == "1"  # as DeviceLevelBuilder
        self._root_bufs = None
        self._root_glob = None

    # ------------------------------------------------------------------ setup
    @staticmethod
    def slots_needed(params: TreeParams) -> int:
        """Histogram slots the engine allocates (one per speculative node, never evicted)."""
        ml = max(params.max_leaf_cnt, 2)
        return int(min(8 * ml + 64, LW_CAP_MAX if ml <= LW_LEAF_MAX else LW_CAP_MAX_BIG))

    @staticmethod
    def supports(bins: torch.Tensor, binsT: Optional[torch.Tensor], B: int, F: int, params: TreeParams,
                 comm: Optional[Comm] = None) -> bool:
        """uint8 row-major bins (B <= 256, 32-aligned stride), a column-major binsT,
        2 <= max_leaf_cnt <= 4096 (above 512 the planner's queue lives in global memory). Multi-GPU: needs
        min_split_samples <= 0 (the children's global counts arrive with the batch's
        all-reduce, after the children planning)."""
        if os.environ.get("YTK_DEVICE_LEAFWISE", "1") == "0":
            return False
        if comm is not None and comm.is_dist and (params.min_split_samples > 0
                                                  or os.environ.get("YTK_DEVICE_LEAFWISE_DIST", "1") == "0"):
            return False
        if params.grow_policy != "loss" or not (2 <= params.max_leaf_cnt <= LW_LEAF_MAX_BIG):
            return False
        if bins.dtype == torch.int16:  # wide bins: uint16 rows, feature-group LDS histograms
            fg = gops.wide_group(B, F)
            return (binsT is not None and binsT.dtype == torch.int16 and binsT.shape[0] == F
                    and binsT.is_contiguous() and bins.is_contiguous() and fg > 0 and bins.shape[1] % fg == 0
                    and 2 * bins.shape[0] < (1 << 31))
        if bins.dtype != torch.uint8 or binsT is None or binsT.dtype != torch.uint8 or B > 256:
            return False
        stride = bins.shape[1]
        if stride % 32 != 0 or stride < ((F + 31) // 32) * 32 or binsT.shape[0] != F or not binsT.is_contiguous():
            return False
        return 2 * bins.shape[0] < (1 << 31)

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
                                              p.max_abs_leaf_val, p.learning_rate, self.SUB_ALPHA)]

    def _ip(self):
        p = self.p
        # speculation: 0 = one node per batch; else the percentage of the remaining leaf
        # budget the batch choice ranks within (100 = the host planner's virtual replay)
        spec = int(os.environ.get("YTK_LW_SPEC_PCT", "100")) if os.environ.get("YTK_LOSSGUIDE_SPEC", "1") != "0" else 0
        return [p.max_depth, p.max_leaf_cnt, p.min_split_samples, spec, self.HIST_TARGET, self.MIN_ROWS,
                self.cap, self.N, self.split_groups, 1 if self.comm.is_dist else 0, 2 if self.wide else 1,
                self.SUB_ROWS if self.sub_on else 0, self.SUB_MAX]

    def _ptrs(self):
        f, i = self.nd_f64, self.nd_i32
        nodes = [ptr(f[0]), ptr(f[1]), ptr(f[2]), ptr(f[3]), ptr(f[4])]
        ints = [ptr(i[k]) for k in range(11)]  # begin cnt_local depth feat bin_a bin_b lc tid seq state
        return ([ptr(self.st), ptr(self.tnodes)] + nodes + ints[:10] + [ptr(self.nd_loss), ptr(self.heap),
                ptr(self.batch)] + [ptr(self.part[k]) for k in range(6)]
                + [ptr(self.cursor), ptr(self.hist_items), ptr(self.build_ids), ptr(self.split_items),
                   ptr(self.item_sid), ptr(self.split_out), ptr(self.root_cnt),
                   ptr(self.prof) if self.prof is not None else 0, self._done_dev, ptr(self.zero_ids),
                   ptr(self.zero_range), ptr(self.plan_ws) if self.plan_ws is not None else 0,
                   ptr(self.sub_words), ptr(self.sub_list)])

    def _lv_ptrs(self):
        """Pointer list of the level engine's finalize / raw-tree kernels (st, nodes, arrays)."""
        out = [0] * 27
        out[0], out[1] = ptr(self.st), ptr(self.tnodes)
        out[19:24] = [ptr(self.tfeat), ptr(self.tthr), ptr(self.tleft), ptr(self.tright), ptr(self.tval)]
        return out

    def _fmask(self, rng):
        p = self.p
        if p.feature_sample_rate < 1.0:
            n_sam = max(1, int(round(p.feature_sample_rate * self.F)))
            perm = rng.permutation(self.F)
            fm = np.zeros(self.F, np.uint8)
            fm[np.sort(perm[:n_sam])] = 1
        else:
            fm = np.ones(self.F, np.uint8)
        self._fmask_np = fm
        key = fm.tobytes()
        if key not in self._fmask_cache:
            if len(self._fmask_cache) > 64:
                self._fmask_cache.clear()
            self._fmask_cache[key] = torch.from_numpy(fm).to(self.dev)
        return self._fmask_cache[key], int(np.nonzero(fm)[0][0])

    # ------------------------------------------------------------------ build
    def _hist_split(self, h, rows_ptr, gh_ptr, fmask, f0, s):
        self._hist(h, rows_ptr, gh_ptr, s)
        self._split(h, fmask, f0, s)

    def _part(self, h, hd, rows_in, gh_in, s, it=-1):
        """lw_partition of the current batch into rows2 (+ gh2 unless (g, h) is row-indexed).
        Batches it < PART_SCAN (one or two splits, thousands of chunks each) reserve their
        chunks through a count pass + scan instead of the split cursor atomics."""
        if self._ghr:
            h.lw_partition(hd, ptr(self.binsT), self.binsT.shape[1], rows_in, 0, ptr(self.rows2), 0,
                           self.max_pblocks, s)
        else:
            scan = 0 <= it < self.PART_SCAN and not self.wide
            h.lw_partition(hd, ptr(self.binsT), self.binsT.shape[1], rows_in, gh_in, ptr(self.rows2), ptr(self.gh2),
                           self.max_pblocks, s, ptr(self.chunk_io) if scan else 0)

    def _hist(self, h, rows_ptr, gh_ptr, s):
        st = ptr(self.st)
        gh_rows = 0
        if self._ghr and rows_ptr:  # gathered rows: (g, h) by row id
            gh_ptr, gh_rows = self._ghr, 1
        # sole-item slots are stored by the hist kernel, <= 16-item slots by the reduce, larger
        # ones zeroed by their first hist item and reduced split-K
        if self.wide:
            h.hist_wide_staged_dev(ptr(self.bins), self.bins.shape[1], self.F, gh_ptr, rows_ptr, ptr(self.hist_items),
                                   self.hist_bound, st + 4 * W_N_HIST, ptr(self.hist), self.B, ptr(self.scales),
                                   ptr(self.staging), ptr(self.zero_ids), st + 4 * W_N_ZERO, ptr(self.zero_range),
                                   self.REDUCE_Y, s)
            return
        h.hist_fx_staged_dev(ptr(self.bins), self.bins.shape[1], self.F, gh_ptr, rows_ptr, ptr(self.hist_items),
                             self.hist_bound, st + 4 * W_N_HIST, ptr(self.hist), self.B, ptr(self.scales),
                             ptr(self.staging), ptr(self.zero_ids), st + 4 * W_N_ZERO, ptr(self.zero_range),
                             self.REDUCE_Y, s, gh_rows)

    def _owner_fmask(self, fmask, f0):
        """(owned sampled-feature mask on the device, its first feature, the rank whose block
        holds the first sampled feature -- its records carry the node totals)."""
        fm_np = self._fmask_np  # the tree's sampled-feature mask (host copy, set by _fmask)
        key = fm_np.tobytes()
        if key not in self._own_cache:
            lo, hi = self.own
            fm = fm_np.copy()
            fm[:lo] = 0
            fm[hi:] = 0
            nz = np.flatnonzero(fm)
            f0o = int(nz[0]) if nz.size else (lo if hi > lo else 0)
            tot = next(r for r, (a, b) in enumerate(self.fblocks) if b > a and fm_np[a:b].any())
            if len(self._own_cache) > 64:
                self._own_cache.clear()
            self._own_cache[key] = (torch.from_numpy(fm).to(self.dev), f0o, tot)
        return self._own_cache[key]

    def _owner_sync(self, h, hd, s, kcap=-1):
        """Reduce-scatter the batch's built slots by feature block (+ its cursors): pack, one
        peer kernel sized on the device (kcap < 0) or an RCCL reduce-scatter of kcap-split
        segments, unpack this rank's block."""
        P = self.comm.world
        fr = self.fr
        if self.peer is not None and kcap < 0:
            h.lw_owner(hd, ptr(self.hist), self.slot_elems, self.B, self.F, fr, P, self.comm.rank, ptr(self._own_x),
                       -1, 0, s)
            st = ptr(self.st)
            self.peer.reduce_scatter_dev_(self._own_x, self.B * fr * 2, st + 4 * W_N_BUILD, st + 4 * W_N_SPLIT,
                                          CUR_STRIDE, st + 4 * LW_DONE)
            # unpack 2: this rank's segment starts at rank x its device-counted size
            h.lw_owner(hd, ptr(self.hist), self.slot_elems, self.B, self.F, fr, P, self.comm.rank, ptr(self._own_x),
                       -1, 2, s)
            return
        per = kcap * (self.B * fr * 2 + CUR_STRIDE)
        if per == 0:
            return
        x = self._own_x[:P * per]
        h.lw_owner(hd, ptr(self.hist), self.slot_elems, self.B, self.F, fr, P, self.comm.rank, ptr(x), kcap, 0, s)
        out = self._own_out[:per]
        if self.peer is not None:
            self.peer.reduce_scatter_(x)
            out = x[self.comm.rank * per:(self.comm.rank + 1) * per]
        else:
            self.comm.reduce_scatter_(out, x.view(P, per))
        h.lw_owner(hd, ptr(self.hist), self.slot_elems, self.B, self.F, fr, P, self.comm.rank, ptr(out), kcap, 1, s)

    def _split(self, h, fmask, f0, s):
        st = ptr(self.st)
        gp = self.gp
        if self.owner:
            fm_own, f0o, tot = self._owner_fmask(fmask, f0)
            h.split_find(ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fm_own), f0o, ptr(self.split_items),
                         self.n_sitems, ptr(self.split_local), gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"], 1.0,
                         1.0, st + 4 * W_N_SITEMS, ptr(self.inv_scales), ptr(self.split_part), ptr(self.split_cnt), s)
            n = self.split_local.numel()
            r = self.comm.rank
            if self.peer is not None:
                self._allr[r * n:(r + 1) * n].copy_(self.split_local)
                self.peer.allgather_(self._allr.view(torch.int64), st + 4 * LW_DONE)
                allr = self._allr
            else:
                allr = self.comm.allgather(self.split_local)
            h.split_combine(ptr(allr), self.comm.world, self.n_sitems, st + 4 * W_N_SITEMS, self.n_sitems, tot,
                            ptr(self.split_out), s)
            return
        if self.split_groups > 1:
            if not h.split_node_grouped(ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fmask), f0,
                                        ptr(self.split_items), self.n_sitems, ptr(self.split_out), gp["mcw"], gp["l1"],
                                        gp["l2"], gp["max_abs_leaf"], st + 4 * W_N_SITEMS, ptr(self.inv_scales),
                                        self.split_groups, s):
                raise RuntimeError("split_node_grouped does not apply; set YTK_SPLIT_GROUPS=1")
            return
        h.split_find(ptr(self.hist), self.B, self.F, ptr(self.nbins_f), ptr(fmask), f0, ptr(self.split_items),
                     self.n_sitems, ptr(self.split_out), gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"], 1.0, 1.0,
                     st + 4 * W_N_SITEMS, ptr(self.inv_scales), ptr(self.split_part), ptr(self.split_cnt), s)

    def build(self, gh: torch.Tensor, ghmax: torch.Tensor = None, ghmax_global: bool = False) -> DeviceTree:
        """Enqueue one tree from ``gh`` [N, 2] (g, h); ``ghmax`` = max |g|, |h| (optional)."""
        p = self.p
        h = hip()
        s = stream(self.bins)
        lr = float(np.float32(p.learning_rate))
        if lr != self._lr:
            h.lw_set_lr(self._handle, lr)
            self._lr = lr
        rng = np.random.default_rng((p.seed, self.tree_count))
        seed_rows = int(rng.integers(1 << 62))
        sampled = p.instance_sample_rate < 1.0
        dist = self.comm.is_dist
        assert gh.is_contiguous() and gh.shape == (self.N, 2)
        self._ghr = ptr(gh) if self.gh_rows else 0
        if sampled:  # sampled rows first (stable), in the first half of the ping-pong buffers
            g = torch.Generator(device=self.dev)
            g.manual_seed(seed_rows + self.comm.rank)
            keep = torch.rand(self.N, generator=g, device=self.dev) < p.instance_sample_rate
            _, order = torch.sort((~keep).to(torch.int32), stable=True)
            self.rows2[:self.N].copy_(order.to(torch.int32))
            if not self.gh_rows:
                self.gh2[:self.N].copy_(gh.index_select(0, order))
            self.root_cnt[0] = keep.sum()
            self.root_cnt[1] = self.root_cnt[0]
            if dist:
                self.comm.allreduce_(self.root_cnt[1:2])
            self.last_keep = keep
            rows0, gh0 = ptr(self.rows2), ptr(self.gh2)
            mx = ghmax if (ghmax is not None and ghmax_global) else (gh.abs() * keep[:, None]).amax(dim=0)
        else:
            self.last_keep = None
            if self._root_glob is None:  # (local, global) rows: constants of an unsampled run
                self.root_cnt[0] = self.N
                self.root_cnt[1] = self.N
                if dist:
                    self.comm.allreduce_(self.root_cnt[1:2])
                self._root_glob = True
            rows0, gh0 = 0, ptr(gh)
            mx = ghmax if ghmax is not None else gh.abs().amax(dim=0)
        if sampled:
            self._root_glob = None
        if dist and not ghmax_global:
            mx = mx.clone()
            self.comm.allreduce_(mx, op="max")
        fmask, f0 = self._fmask(rng)
        h.lv_scales(ptr(mx), ptr(self.root_cnt), ptr(self.scales), ptr(self.inv_scales), s)
        tm = self.timer
        tm.mark("init_stats")
        hd = self._handle
        # the previous tree's batches all finished (its done flag was observed), so no
        # kernel writes the flag while it is reset
        self._done_host[0] = 0
        self._done_host[1] = 0
        self._done_host[2] = 0
        h.lw_step(hd, 0, s)
        root_done = self.root_ready and not sampled  # built by the previous gradient pass
        self.root_ready = False
        if dist and self.peer is None:  # RCCL: the host sizes every batch message
            if not root_done:
                self._hist(h, rows0, gh0, s)
            self._allreduce(self.hist[0:1].view(-1))  # the root slot
            self._split(h, fmask, f0, s)
            tm.mark("root")
            it = self._build_dist(h, hd, rows0, gh0, fmask, f0, s)
            return self._finish(h, s, it)
        if not root_done:
            self._hist(h, rows0, gh0, s)
        if dist:
            self._allreduce(self.hist[0:1].view(-1))  # the root slot (peer exchange)
        self._split(h, fmask, f0, s)
        tm.mark("root")
        # Launch throttle without events (a recorded event put a ~6 us gap before every
        # planner launch): the planner writes its batch count to pinned host memory, the
        # host keeps at most POLL_LAG batches queued beyond the last one planned and stops
        # at the done flag. While it waits it runs the idle hook once per tree (the trainer
        # converts the previous round's tree there, off the GPU's critical path).
        dh = self._dh_np
        idle = self.idle_hook
        it = 0
        t_wait = None
        while True:
            self._batch(h, hd, rows0 if it == 0 else ptr(self.rows2), gh0 if it == 0 else ptr(self.gh2),
                        fmask, f0, s, it)
            it += 1
            if it > 4 * self.max_leaf + 8:
                raise RuntimeError("device leaf-wise builder did not terminate")
            if dh[0] != 0:
                break
            if dh[1] >= it - self.POLL_LAG:
                continue
            if idle is not None:
                idle()
                idle = None
            t_wait = time.perf_counter()
            while dh[0] == 0 and dh[1] < it - self.POLL_LAG:
                if time.perf_counter() - t_wait > self.POLL_TIMEOUT_S:
                    raise RuntimeError(f"device leaf-wise builder: no planner progress for {self.POLL_TIMEOUT_S} s "
                                       f"(batch {it}, planned {int(dh[1])})")
            if dh[0] != 0:
                break
        if idle is not None:
            idle()
        return self._finish(h, s, it)

    # RCCL batch loop: splits per batch capped at min(2^batch, YTK_LW_RCCL_KCAP) -- a
    # schedule every rank knows without reading the device, so each batch's message is a
    # fixed-size collective the host can issue ahead like the peer loop
    RCCL_KCAP = int(os.environ.get("YTK_LW_RCCL_KCAP", 32))

    def _rccl_cap(self, it: int) -> int:
        return max(1, min(self.RCCL_KCAP, min(self.max_leaf, LW_LEAF_MAX), 1 << min(it, 20)))

    def _build_dist(self, h, hd, rows0, gh0, fmask, f0, s) -> int:
        """Multi-GPU batch loop over RCCL (the peer path off or voted down): plan -> partition
        (+ children planning) -> histograms -> one fixed-size all-reduce of the batch's built
        slots + split cursors (device pack / unpack; the planner caps the batch at the
        message's split capacity, a host schedule identical on every rank) -> split search.
        The host never waits for a batch's planner (round 4 spun on each one to learn its
        split count): it queues up to POLL_LAG batches ahead and stops at the done flag, and
        at the end of the tree the ranks agree on the number of batches issued (one host
        scalar all-reduce) -- the ones past the tree's end are no-ops on the device, but their
        collectives must pair up. Every rank's planner takes identical decisions from the
        identical all-reduced histograms (reference shape: DataParallelTreeMaker.java:229-295)."""
        dh = self._dh_np
        idle = self.idle_hook
        it = 0

        def one(it):
            kc = self._rccl_cap(it)
            h.lw_set_batch_cap(hd, kc)
            h.lw_step(hd, 1, s)
            self._part(h, hd, rows0 if it == 0 else ptr(self.rows2), gh0 if it == 0 else ptr(self.gh2), s, it)
            self._hist(h, ptr(self.rows2), ptr(self.gh2), s)
            if self.owner:
                self._owner_sync(h, hd, s, kcap=kc)
            else:
                n = kc * (self.slot_elems + CUR_STRIDE)
                h.lw_msg(hd, ptr(self.hist), self.slot_elems, ptr(self.msg), kc, 0, s)
                self.comm.allreduce_(self.msg[:n])
                h.lw_msg(hd, ptr(self.hist), self.slot_elems, ptr(self.msg), kc, 1, s)
            self._split(h, fmask, f0, s)

        while True:
            one(it)
            it += 1
            if it > 4 * self.max_leaf + 8:
                raise RuntimeError("device leaf-wise builder did not terminate")
            if dh[0] != 0:
                break
            if dh[1] >= it - self.POLL_LAG:
                continue
            if idle is not None:
                idle()
                idle = None
            t_wait = time.perf_counter()
            while dh[0] == 0 and dh[1] < it - self.POLL_LAG:
                if time.perf_counter() - t_wait > self.POLL_TIMEOUT_S:
                    raise RuntimeError(f"device leaf-wise builder: no planner progress for {self.POLL_TIMEOUT_S} s "
                                       f"(batch {it}, planned {int(dh[1])})")
            if dh[0] != 0:
                break
        # every rank issues the same collectives: pad to the largest batch count issued
        it_all = int(self.comm.allreduce_scalars([it], op="max")[0])
        while it < it_all:
            one(it)
            it += 1
        h.lw_set_batch_cap(hd, 0)
        if idle is not None:
            idle()
        return it

    def _allreduce(self, t: torch.Tensor):
        if self.peer is not None:
            self.peer.allreduce_(t)
        else:
            self.comm.allreduce_(t)

    def root_target(self):
        """Arguments of the fused gradient + root histogram pass (gops.tree_grad root=)."""
        if self._root_bufs is None:
            grid = hip().tree_grad_hist_grid(self.N)
            self._root_bufs = (torch.empty(grid * 256 * 32 * 2, dtype=torch.int64, device=self.dev),
                               torch.zeros(4 * grid, dtype=torch.int32, device=self.dev))
        stg, work = self._root_bufs
        zero_n = 0 if self._zero_at_end else self.hist[0].numel()
        return {"slot": ptr(self.hist), "scales": ptr(self.scales), "staging": ptr(stg), "work": ptr(work),
                "B": self.B, "F": self.F, "zero": ptr(self.hist) if zero_n else 0, "zero_n": zero_n}

    def _finish(self, h, s, it) -> DeviceTree:
        self.timer.mark("batches")
        # finalize (+ the raw-threshold tree for the test-set pass) in one launch
        rq = self._raw_req
        ro = rq["out"] if rq is not None else None
        h.lv_tail(self._lv_ptrs(), [0] * 9, [0.0] * 6, 0, 0, 0, self.max_nodes,
                  ptr(rq["cand"]) if rq else 0, ptr(rq["coff"]) if rq else 0, ptr(rq["fill"]) if rq else 0,
                  rq["median"] if rq else 0, ptr(ro["nfeat"]) if rq else 0, ptr(ro["nthr"]) if rq else 0,
                  ptr(ro["nleft"]) if rq else 0, ptr(ro["nright"]) if rq else 0, ptr(ro["ndefl"]) if rq else 0,
                  ptr(ro["nval"]) if rq else 0, s)
        self._raw_ready = rq is not None
        if self.fuse_root and self._zero_at_end:
            self.hist[0].zero_()  # the next gradient pass accumulates the next root here
        # (default: that pass zeroes slot 0 itself, root_target()'s zero range)
        self.tree_count += 1
        self.last_batches = it
        # K > 1 rounds build several trees before their arrays are consumed: copies; a K == 1
        # round consumes the tree (gradient pass, test pass, readback copy) before the next build
        snap = self.snap.clone() if self.snapshot_copy else self.snap
        st_t, nodes, *arrays = self._snap_views(snap)
        dt = DeviceTree(nodes, st_t, tuple(arrays), self.max_nodes, snap, self._snap_sizes[0])
        if not self.snapshot_copy:
            dt.snap_full, dt.rv_off = self._snap_full, self.rv_off
        return dt

    def round_vector(self, n: int) -> torch.Tensor:
        """float64 [n] device vector (the trainer's round losses + leaf counts)."""
        assert n <= 4 + self.max_nodes
        return self._snap_full[self.rv_off:self.rv_off + 8 * n].view(torch.float64)

    def set_raw_request(self, cand: torch.Tensor, coff: torch.Tensor, fill: torch.Tensor, split_median: bool):
        """As DeviceLevelBuilder.set_raw_request: the tree tail writes the raw tree."""
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

    def prof_report(self) -> dict:
        """Accumulated planner phase times (us, 100 MHz wall clock) and work counters."""
        if self.prof is None:
            return {}
        v = self.prof.cpu().numpy()
        names = ["apply", "stage", "replay", "events", "select", "expand", "writeback"]
        out = {f"plan_{n}_us": round(float(v[i]) / 100.0, 1) for i, n in enumerate(names)}
        out["plan_queue_sort_us"] = round(float(v[7]) / 100.0, 1)
        out.update(plan_calls=int(v[8]), part_blocks=int(v[9]), replay_events=int(v[10]), candidates=int(v[11]),
                   hist_rows=int(v[12]), built_slots=int(v[13]), hist_items=int(v[14]),
                   replay_sorted_pops=int(v[21]), sub_roots=int(v[16]), sub_splits=int(v[17]))
        for i, n in ((22, "jump"), (23, "keys"), (24, "rank")):  # parts of "select"
            out[f"plan_select_{n}_us"] = round(float(v[i]) / 100.0, 1)
        return out

    def _batch(self, h, hd, rows_in, gh_in, fmask, f0, s, it=-1):
        """One speculative batch: plan, partition (+ children planning), histograms, splits.
        Multi-GPU (peer path): the batch's built slots + split cursors are all-reduced between
        the histograms and the split search by one exchange kernel sized on the device (a
        no-op once the planner has marked the tree done -- every rank takes the same planning
        decisions, so the exchanges pair up however many batches a host queued past the end)."""
        h.lw_step(hd, 1, s)
        self._part(h, hd, rows_in, gh_in, s, it)
        if self.peer is None:
            self._hist_split(h, ptr(self.rows2), ptr(self.gh2), fmask, f0, s)
            if self.sub_on:  # the batch's small entries: whole subtrees, one workgroup each
                h.lw_subtree(hd, ptr(self.bins), self.bins.shape[1], ptr(self.binsT), self.binsT.shape[1], rows_in,
                             gh_in, ptr(self.rows2), ptr(self.gh2), self._ghr, ptr(self.hist), self.B, self.F,
                             ptr(self.nbins_f), ptr(fmask), f0, ptr(self.scales), ptr(self.inv_scales), s)
            return
        self._hist(h, ptr(self.rows2), ptr(self.gh2), s)
        if self.owner:  # reduce-scatter by feature block (one kernel sized on the device)
            self._owner_sync(h, hd, s)
        else:
            st = ptr(self.st)
            self.peer.allreduce_slots_(self.hist, self.slot_elems, ptr(self.build_ids), st + 4 * W_N_BUILD,
                                       self.cursor, st + 4 * W_N_SPLIT, CUR_STRIDE, st + 4 * LW_DONE)
        self._split(h, fmask, f0, s)

    def close(self):
        """Release the peer-memory group (collective: every rank calls it)."""
        if self.peer is not None:
            self.peer.close()
            self.peer = None

    def stats(self):
        """(batches, expanded nodes, overflow flag) of the last tree (synchronises)."""
        st = self.st.cpu().numpy()
        return int(st[LW_BATCHES]), int(st[LW_EXPANDED]), int(st[LW_OVERFLOW])

    def live_tree_views(self):
        """(node table, leaf-value array) the engine's raw_tree reads."""
        return self.tnodes, self.tval

    def raw_tree(self, cand: torch.Tensor, coff: torch.Tensor, fill: torch.Tensor, split_median: bool):
        """Raw-threshold arrays of the LAST built tree (test-set scoring)."""
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
        hip().lv_raw_tree(self._lv_ptrs(), mn, ptr(cand), ptr(coff), ptr(fill) if fill is not None else 0,
                          1 if split_median else 0, ptr(out["nfeat"]), ptr(out["nthr"]), ptr(out["nleft"]),
                          ptr(out["nright"]), ptr(out["ndefl"]), ptr(out["nval"]), stream(self.bins))
        return out
