"""Exact-greedy, level-wise tree maker on presorted columns (``tree_maker = "feature"``).

Reference: ``J/optimizer/gbdt/FeatureParallelTreeMakerByLevel.java`` (make :150-185,
initNodeStats :277-312, findSplit :315-343, enumerateSplit :346-398, resetPosition
:424-444) over ``J/data/gbdt/FeatureColData.java:38-58`` (every column sorted by value
once, (value, row) pairs). Every distinct value is a split candidate -- no binning, so any
number of distinct values (a Higgs column has millions) is supported.

Device design (GPU or CPU tensors, no per-row host work):
  * presort once: ``ord[f]`` = rows of column f in ascending value order (stable).
  * node-segmented order: every level keeps, for every feature, the rows of each expanding
    node contiguous and still sorted by value; the node boundaries are the same for every
    feature (a node holds the same rows in every column). After a level's splits each
    segment is stably partitioned into its children (one segmented scan of the go-left flags
    over [F, N] + one scatter), so no re-sort is ever needed.
  * split search: (g, h) gathered in segment order as exact int64 fixed point (the same
    power-of-two scales as the histogram path), inclusive prefix sums per feature, the left
    sums of every candidate = prefix - the node's base; candidates where the value changes
    by more than MIN_FEA_SPLIT_GAP (1e-16f, Constants.java:34) with both children's hessian
    >= min_child_hessian_sum; lossChg = (float)(gain(L) + gain(R) - rootGain) exactly as the
    reference, the best per node = largest lossChg, ties -> lower feature, then lower value
    (SplitInfo.needReplace :99-104 in the reference's scan order); threshold = (v_prev + v)
    * 0.5f.
  * rows go left iff value < threshold (resetPosition :436).
Features are processed in chunks to bound the [F, N] temporaries.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ...ops import gbdt as gops
from ...parallel.comm import Comm
from .builder import TimeStats, TreeParams
from .tree import Tree


def _row_cumsum(x: torch.Tensor) -> torch.Tensor:
    """Inclusive prefix sums along dim 1 of an int64 [C, n] tensor, exact. One device-wide scan
    of the flattened tensor, then each row's start subtracted: torch's scan along the inner
    dimension of a 2-D tensor runs one block per row (~5 ms per [4, 2M] call on MI355X, 80 %
    of an exact-greedy tree), the flat scan is memory bound. Integer wraparound past 2^63
    cancels in the subtraction (each row's true prefix fits in int64)."""
    C, n = x.shape
    if C == 0 or n == 0:
        return torch.cumsum(x, dim=1)
    flat = torch.cumsum(x.reshape(-1), 0).view(C, n)
    if C > 1:
        starts = flat[:-1, -1:].clone()  # sum of all rows before row r, at row r - 1's end
        flat[1:] -= starts
    return flat


MIN_FEA_SPLIT_GAP = np.float32(1e-16)  # Constants.java:34


class ExactGreedyBuilder:
    def __init__(self, X: torch.Tensor, params: TreeParams, comm: Optional[Comm] = None,
                 feat_chunk: Optional[int] = None, engine: Optional[str] = None):
        comm = comm or Comm.local(X.device)
        if comm.is_dist:
            # GBDTDataFlow.java:102-107: feature parallel only supports a single machine
            raise ValueError("[GBDT] feature parallel only support single machine")
        if params.grow_policy != "level" or params.max_depth < 1:
            raise ValueError("the exact-greedy maker grows level-wise with max_depth >= 1")
        self.p = params
        self.comm = comm
        self.dev = X.device
        self.N, self.F = X.shape
        # [F, N] raw values (NaN already filled) and the presorted row order of every column
        self.XT = X.t().contiguous().float()
        self.ord = torch.argsort(self.XT, dim=1, stable=True).to(torch.int64)
        self.chunk = int(feat_chunk or os.environ.get("YTK_EXACT_CHUNK", 8))
        gp = params.gain_params()
        self.gpv = (gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"])
        # on a GPU the level loop runs as the HIP kernels of csrc/hip/gbdt_exact.hip
        # (YTK_EXACT_TORCH=1: the tensor-op formulation below, kept as the CPU path and the
        # GPU test oracle)
        engine = engine or ("torch" if os.environ.get("YTK_EXACT_TORCH", "0") == "1" else "hip")
        self.hip = self.dev.type == "cuda" and engine == "hip"
        if self.hip and not self._hip_fits():
            self.hip = False
        if self.hip:
            self._init_hip()
        self.tree_count = 0
        self.last_keep = None
        self.binsT = None  # API parity with the histogram builders
        self.total_stats = TimeStats()
        self.last_stats = TimeStats()

    # ------------------------------------------------------------------ gains
    def _gain(self, G: torch.Tensor, H: torch.Tensor) -> torch.Tensor:
        """UpdateStrategy.calcGain (:64-80) on float64 tensors."""
        mcw, l1, l2, mal = self.gpv
        if mal <= 0:
            t = G if l1 == 0.0 else torch.sign(G) * torch.clamp(G.abs() - l1, min=0.0)
            gain = t * t / (H + l2)
        else:
            v = self._value(G, H)
            gain = -2.0 * (G * v + 0.5 * (H + l2) * v * v + l1 * v.abs())
        return torch.where(H < mcw, torch.zeros_like(gain), gain)

    def _value(self, G: torch.Tensor, H: torch.Tensor) -> torch.Tensor:
        """UpdateStrategy.calcNodeValue (:83-100)."""
        mcw, l1, l2, mal = self.gpv
        t = G if l1 == 0.0 else torch.sign(G) * torch.clamp(G.abs() - l1, min=0.0)
        v = -t / (H + l2)
        if mal > 0:
            v = v.clamp(-mal, mal)
        return torch.where(H < mcw, torch.zeros_like(v), v)

    # ------------------------------------------------------------------ HIP engine
    HIP_BYTES_PER_CELL = 4 + 4 + 2 * (4 + 4 + 8)  # ord0, val0, ping-pong ordw / valw / qvw (float (g, h))

    def _hip_fits(self) -> bool:
        """The HIP engine holds ~40 B per (feature, row) cell on top of XT (the tensor path ~12 B,
        in feature chunks): check it against the free device memory (the int64 presort order,
        8 B per cell, is released during the set-up) and fall back to the tensor engine, with a
        log line, when it does not fit."""
        need = self.F * self.N * self.HIP_BYTES_PER_CELL
        free, _ = torch.cuda.mem_get_info(self.dev)
        avail = free + self.F * self.N * 8
        if need <= 0.9 * avail:
            return True
        from ...utils.logging import get_logger
        get_logger().info(f"[GBDT] exact greedy: the HIP engine needs {need / 2**30:.1f} GiB for {self.F} x {self.N} "
                          f"cells, {avail / 2**30:.1f} GiB free; using the tensor engine")
        return False

    REC_DTYPE = np.dtype([("G", "<f8"), ("H", "<f8"), ("cnt", "<i8"), ("chg", "<f4"), ("thr", "<f4"),
                          ("value", "<f4"), ("feat", "<i4"), ("split", "<i4"), ("pad", "<i4")])

    def _init_hip(self):
        """Device buffers of the HIP exact-greedy engine: the presorted columns as int32 row
        ids + their values, ping-pong work columns, per-level tiles / node tables / records."""
        from ...ops._ext import hip, ptr
        p, dev, F, N = self.p, self.dev, self.F, self.N
        h = hip()
        T = h.ex_tile()
        self.ord0 = self.ord.to(torch.int32).contiguous()
        self.val0 = torch.gather(self.XT, 1, self.ord).contiguous()
        del self.ord
        self.ord = None
        D = p.max_depth
        kcap = 2 * p.max_leaf_cnt if p.max_leaf_cnt > 0 else (1 << min(D, 22))
        self.Kmax = Kmax = int(max(1, min(N, kcap)))
        self.max_tiles = mt = -(-max(N, 1) // T) + Kmax + 1
        i32 = lambda n: torch.zeros(max(1, n), dtype=torch.int32, device=dev)  # noqa: E731
        i64 = lambda n: torch.zeros(max(1, n), dtype=torch.int64, device=dev)  # noqa: E731
        self.ordw = [torch.empty((F, N), dtype=torch.int32, device=dev) for _ in range(2)]
        self.valw = [torch.empty((F, N), dtype=torch.float32, device=dev) for _ in range(2)]
        # (g, h) travel with the rows as float32 (the kernels convert to the exact int64 fixed
        # point where they sum: rint(g * sg), the q of the tensor engine)
        self.qvw = [torch.empty((F, N, 2), dtype=torch.float32, device=dev) for _ in range(2)]
        self.ex_tiles = [i32(4 * mt), i32(4 * mt)]
        self.ex_nbeg = [i32(Kmax + 1), i32(Kmax + 1)]
        self.ex_ftile = [i32(Kmax + 1), i32(Kmax + 1)]
        self.ex_ctl = i32(128)
        self.ex_st_gh, self.ex_st_cnt = i64(F * mt * 2), i64(F * mt)
        self.ex_tpart = i64(mt * 5)
        self.ex_nbase, self.ex_nkey = i64((Kmax + 1) * 5), i64(F * Kmax)
        self.ex_ntot = i64(Kmax * 2)
        self.ex_go_feat, self.ex_go_thr = i32(Kmax), torch.zeros(Kmax, dtype=torch.float32, device=dev)
        self.ex_csplit, self.ex_cbeg = i32(Kmax), i32(2 * Kmax)
        # left_row bytes [align16(N)] followed by the same flags as bits [ceil(N / 32)] words
        self.ex_left = torch.zeros(((N + 15) // 16) * 16 + 4 * ((N + 31) // 32) + 16, dtype=torch.uint8, device=dev)
        ks = [min(Kmax, 1 << min(d, 40)) for d in range(D + 1)]
        self.rec_off = np.concatenate([[0], np.cumsum(ks)[:-1]]).astype(np.int64)
        self.ex_rec = torch.zeros(int(sum(ks)) * self.REC_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        self.ex_rec_off = torch.from_numpy(self.rec_off).to(dev)
        self.ex_rec_k = i32(D + 1)
        gp = p.gain_params()
        ptrs = [ptr(self.ord0), ptr(self.val0), ptr(self.ordw[0]), ptr(self.ordw[1]), ptr(self.valw[0]),
                ptr(self.valw[1]), ptr(self.qvw[0]), ptr(self.qvw[1]), ptr(self.XT), ptr(self.ex_tiles[0]),
                ptr(self.ex_tiles[1]), ptr(self.ex_nbeg[0]), ptr(self.ex_nbeg[1]), ptr(self.ex_ftile[0]),
                ptr(self.ex_ftile[1]), ptr(self.ex_ctl), ptr(self.ex_st_gh), ptr(self.ex_st_cnt),
                ptr(self.ex_tpart), ptr(self.ex_nbase), ptr(self.ex_nkey), ptr(self.ex_ntot),
                ptr(self.ex_go_feat), ptr(self.ex_go_thr), ptr(self.ex_csplit), ptr(self.ex_cbeg), ptr(self.ex_left),
                ptr(self.ex_rec), ptr(self.ex_rec_off), ptr(self.ex_rec_k)]
        ip = [N, N, N, mt, Kmax, p.min_split_samples, p.max_leaf_cnt]
        fp = [gp["mcw"], gp["l1"], gp["l2"], gp["max_abs_leaf"], float(np.float32(p.min_split_loss)),
              float(np.float32(p.learning_rate))]
        self.ex_handle = h.ex_create(ptrs, ip, fp)
        self._fidx_cache = {}

    def _build_hip(self, gh: torch.Tensor) -> Tree:
        """One tree on the HIP engine: the whole level loop is enqueued by one call
        (csrc/hip/gbdt_exact.hip), then the level records come back in one copy and become
        the host tree (same node order, values and statistics as the tensor path)."""
        from ...ops._ext import hip, ptr, stream
        p, dev = self.p, self.dev
        t_start = time.perf_counter()
        rng = np.random.default_rng((p.seed, self.tree_count))
        seed_rows = int(rng.integers(1 << 62))
        if p.feature_sample_rate < 1.0:
            n_sam = max(1, int(round(p.feature_sample_rate * self.F)))
            feats = np.sort(rng.permutation(self.F)[:n_sam])
        else:
            feats = np.arange(self.F)
        key = feats.tobytes()
        if key not in self._fidx_cache:
            if len(self._fidx_cache) > 64:
                self._fidx_cache.clear()
            self._fidx_cache[key] = torch.from_numpy(feats.astype(np.int32)).to(dev)
        fidx = self._fidx_cache[key]
        nf = len(feats)
        sampled = p.instance_sample_rate < 1.0
        if sampled:  # each searched column's kept rows, still in value order, into work slab 0
            g = torch.Generator(device=dev)
            g.manual_seed(seed_rows)
            keep = torch.rand(self.N, generator=g, device=dev) < p.instance_sample_rate
            self.last_keep = keep
            o = self.ord0[fidx.long()]
            km = keep[o.long()]
            n = int(km[0].sum()) if nf else 0
            self.ordw[0][:nf, :n] = o[km].view(nf, n)
            self.valw[0][:nf, :n] = self.val0[fidx.long()][km].view(nf, n)
            ghk = gh[keep]
        else:
            keep = None
            self.last_keep = None
            n = self.N
            ghk = gh
        mx = ghk.abs().amax(dim=0).double().cpu().numpy() if n > 0 else np.zeros(2)
        sg, sh = gops.fixed_point_scales(mx[0], mx[1], 4 * max(n, 1))  # |sums| < 2^60 (look-back words)
        ghf = gh.float().contiguous()  # the kernels quantize rint(g * sg) themselves (== quantize_gh)
        D = p.max_depth
        hip().ex_tree(self.ex_handle, ptr(ghf), ptr(fidx), nf, n, 1 if sampled else 0, 1.0 / sg, 1.0 / sh, D,
                      float(np.float32(p.learning_rate)), stream(ghf))
        recs = self.ex_rec.cpu().numpy().view(self.REC_DTYPE)
        rec_k = self.ex_rec_k.cpu().numpy()
        err = int(self.ex_ctl[5].item())
        if err:
            raise RuntimeError(f"exact-greedy engine: capacity exceeded (code {err}, Kmax={self.Kmax}, "
                               f"tiles={self.max_tiles})")
        tree = Tree()
        expand = [0]
        for d in range(D + 1):
            K = int(rec_k[d])
            if not expand or K == 0:
                break
            assert K == len(expand), (d, K, len(expand))
            r = recs[self.rec_off[d]:self.rec_off[d] + K]
            new_expand = []
            for k, nid in enumerate(expand):
                tree.hess_sum[nid] = float(np.float32(r["H"][k]))
                tree.sample_cnt[nid] = int(r["cnt"][k])
                tree.loss_chg[nid] = float(r["chg"][k])
                if r["split"][k]:
                    lc, rc = tree.add_children(nid)
                    tree.feat[nid] = int(r["feat"][k])
                    tree.cond[nid] = float(r["thr"][k])
                    tree.is_leaf[nid] = False
                    new_expand += [lc, rc]
                else:
                    tree.set_leaf(nid, float(r["value"][k]))
            expand = new_expand
        tree.converted = True
        self.tree_count += 1
        self.last_stats = TimeStats()
        self.last_stats.total = time.perf_counter() - t_start
        self.last_stats.trees = 1
        self.total_stats.add(self.last_stats)
        return tree

    # ------------------------------------------------------------------ build
    def build(self, gh: torch.Tensor, ghmax: Optional[torch.Tensor] = None, ghmax_global: bool = False) -> Tree:
        if self.hip:
            return self._build_hip(gh)
        p = self.p
        t_start = time.perf_counter()
        dev = self.dev
        rng = np.random.default_rng((p.seed, self.tree_count))
        seed_rows = int(rng.integers(1 << 62))
        # --- instance / feature subsampling (initAssistData :188-247)
        if p.instance_sample_rate < 1.0:
            g = torch.Generator(device=dev)
            g.manual_seed(seed_rows)
            keep = torch.rand(self.N, generator=g, device=dev) < p.instance_sample_rate
            self.last_keep = keep
            order = self.ord[keep[self.ord]].view(self.F, -1)  # each column's kept rows, still sorted
        else:
            keep = None
            self.last_keep = None
            order = self.ord
        n = order.shape[1]
        if p.feature_sample_rate < 1.0:
            n_sam = max(1, int(round(p.feature_sample_rate * self.F)))
            feats = np.sort(rng.permutation(self.F)[:n_sam])
        else:
            feats = np.arange(self.F)
        # exact int64 fixed point (g, h): order-independent sums, the histogram path's scales
        ghk = gh if keep is None else gh[keep]
        mx = ghk.abs().amax(dim=0).double().cpu().numpy() if n > 0 else np.zeros(2)
        # the HIP engine's scales (|sums| < 2^60): both engines build identical trees
        sg, sh = gops.fixed_point_scales(mx[0], mx[1], 4 * max(n, 1))
        q = torch.empty((self.N, 2), dtype=torch.int64, device=dev)
        q[:, 0] = torch.round(gh[:, 0].float() * np.float32(sg)).to(torch.int64)
        q[:, 1] = torch.round(gh[:, 1].float() * np.float32(sh)).to(torch.int64)
        inv = torch.tensor([1.0 / sg, 1.0 / sh], dtype=torch.float64, device=dev)
        inv_g, inv_h = 1.0 / sg, 1.0 / sh
        qT = q.t().contiguous()  # [2, N]
        mcw, l1, l2, mal = self.gpv
        lr32 = np.float32(p.learning_rate)
        msl = float(np.float32(p.min_split_loss))

        tree = Tree()
        # node of every position of the segmented order (same for every feature)
        seg = [(0, n)]            # (begin, end) per expanding node, in expand order
        expand = [0]
        leaf_cnt = 1
        stats = {}                # nid -> (G, H, cnt, best lossChg)
        pos_node = torch.zeros(n, dtype=torch.int64, device=dev)
        for depth in range(p.max_depth):
            if p.max_leaf_cnt > 0 and leaf_cnt >= p.max_leaf_cnt:
                break
            K = len(expand)
            bnd = torch.tensor([b for b, _ in seg] + [seg[-1][1] if seg else 0], dtype=torch.int64, device=dev)
            cnt = (bnd[1:] - bnd[:-1])
            # node sums (initNodeStats): column 0's contiguous node segments, exact int64
            # prefix differences (no atomics)
            rows0 = order[0]
            sums = self._seg_sums(q[rows0], bnd)
            Gd = sums.double() * inv  # [K, 2] float64 totals
            root_gain = self._gain(Gd[:, 0], Gd[:, 1]).float()
            can = (Gd[:, 1] >= 2.0 * mcw) & (cnt >= max(p.min_split_samples, 0))  # canSplit
            first = torch.zeros(n, dtype=torch.bool, device=dev)
            first[bnd[:-1][cnt > 0]] = True  # the first row of a node is never a candidate
            nf = len(feats)
            mx_all = torch.empty((nf, K), dtype=torch.float32, device=dev)
            thr_all = torch.empty((nf, K), dtype=torch.float32, device=dev)
            pad = self._pad_layout(bnd, cnt, pos_node, K, n)
            for c0 in range(0, nf, self.chunk):
                fs = torch.from_numpy(feats[c0:c0 + self.chunk]).to(dev)
                C = fs.numel()
                o = order[fs]                                   # [C, n] rows
                v = torch.gather(self.XT[fs], 1, o)             # [C, n] values, sorted per node
                # (g, h) as separate [C, n] planes: the prefix sums run along the innermost
                # dimension (torch's parallel scan; a middle-dimension scan is sequential)
                lg, lh = [], []
                for comp in (0, 1):
                    x = qT[comp][o]                             # [C, n] int64
                    excl = _row_cumsum(x) - x                    # sums of the rows before i
                    base = excl[:, bnd[:-1].clamp(max=max(n - 1, 0))]  # [C, K] node start
                    (lg if comp == 0 else lh).append(excl - base[:, pos_node])
                left_g, left_h = lg[0], lh[0]
                Lg, Lh = left_g.double() * inv_g, left_h.double() * inv_h
                Rg = (sums[pos_node, 0][None] - left_g).double() * inv_g
                Rh = (sums[pos_node, 1][None] - left_h).double() * inv_h
                dv = torch.zeros_like(v)
                dv[:, 1:] = (v[:, 1:] - v[:, :-1]).abs()
                ok = (~first[None]) & (dv > MIN_FEA_SPLIT_GAP) & (left_h != 0)
                ok &= (Lh >= mcw) & (Rh >= mcw) & can[pos_node][None]
                chg = (self._gain(Lg, Lh) + self._gain(Rg, Rh) - root_gain[pos_node][None].double()).float()
                # a 0/0 gain (zero-hessian child, mcw = l2 = 0) is never taken: the reference's
                # `newLossChg > lossChg` is false for NaN
                chg = torch.where(ok & ~torch.isnan(chg), chg, torch.full_like(chg, float("-inf")))
                # per (feature, node): max lossChg and its FIRST position (the scan order), as
                # ONE int64 max over keys (orderable lossChg bits << 31 | ~position), reduced
                # per tile of a segment-aligned padded layout, then over each node's tiles
                pi, mx = self._seg_argmax(chg, pad)
                thr = (torch.gather(v, 1, pi) + torch.gather(v, 1, (pi - 1).clamp(min=0))) * np.float32(0.5)
                mx_all[c0:c0 + C] = mx
                thr_all[c0:c0 + C] = thr
                del o, v, lg, lh, left_g, left_h, Lg, Lh, Rg, Rh, chg, dv, ok
            # features in ascending order, replaced only when strictly greater: the max
            # lossChg, ties -> the lowest feature (SplitInfo.needReplace)
            best_chg = mx_all.max(dim=0).values if nf else torch.full((K,), float("-inf"), device=dev)
            fi = torch.argmax((mx_all == best_chg[None]).to(torch.int8), dim=0)  # first feature at the max
            best_f = torch.from_numpy(feats).to(dev)[fi]
            best_v = thr_all.gather(0, fi[None])[0]
            # no candidate at all <=> -inf (a +inf lossChg -- a zero-hessian child with
            # min_child_hessian_sum = l2 = 0 -- is a candidate, as the reference's > takes it)
            best_f = torch.where(best_chg > float("-inf"), best_f, torch.full_like(best_f, -1))
            # --- tree update (findSplit :327-342), host side over the level's nodes
            bc, bf, bv = best_chg.cpu().numpy(), best_f.cpu().numpy(), best_v.cpu().numpy()
            Gh = Gd.cpu().numpy()
            vals = (self._value(Gd[:, 0], Gd[:, 1]).float().cpu().numpy()) * lr32
            cnt_h = cnt.cpu().numpy()
            split_nodes, new_expand = [], []
            go_feat = np.full(K, -1, np.int64)
            go_thr = np.zeros(K, np.float32)
            for k, nid in enumerate(expand):
                stats[nid] = (float(Gh[k, 1]), int(cnt_h[k]), float(bc[k]))
                if (p.max_leaf_cnt < 0 or leaf_cnt < p.max_leaf_cnt) and bc[k] > msl:
                    lc, rc = tree.add_children(nid)
                    leaf_cnt += 1
                    tree.feat[nid] = int(bf[k])
                    tree.cond[nid] = float(bv[k])
                    tree.is_leaf[nid] = False
                    split_nodes.append(k)
                    new_expand += [lc, rc]
                    go_feat[k] = bf[k]
                    go_thr[k] = bv[k]
                else:
                    tree.set_leaf(nid, float(vals[k]))
            if not split_nodes:
                expand, seg = [], []
                break
            # --- resetPosition + stable re-segmentation of every column's order
            gf = torch.from_numpy(go_feat).to(dev)
            gt = torch.from_numpy(go_thr).to(dev)
            order, pos_node, seg = self._resegment(order, pos_node, bnd, gf, gt, K)
            n = order.shape[1]  # the rows of nodes that became leaves left the order
            expand = new_expand
        # remaining expand nodes become leaves (make :176-180)
        if expand:
            K = len(expand)
            rows0 = order[0]
            bnd = torch.tensor([b for b, _ in seg] + [seg[-1][1] if seg else 0], dtype=torch.int64, device=dev)
            sums = self._seg_sums(q[rows0], bnd)
            Gd = sums.double() * inv
            vals = (self._value(Gd[:, 0], Gd[:, 1]).float().cpu().numpy()) * lr32
            cnts = (bnd[1:] - bnd[:-1]).cpu().numpy()
            Gh = Gd.cpu().numpy()
            for k, nid in enumerate(expand):
                tree.set_leaf(nid, float(vals[k]))
                stats[nid] = (float(Gh[k, 1]), int(cnts[k]), float("-inf"))
        for nid, (hs, c, chg) in stats.items():  # updateTreeNodeStat
            tree.hess_sum[nid] = float(np.float32(hs))
            tree.sample_cnt[nid] = c
            tree.loss_chg[nid] = float(np.float32(chg))
        tree.converted = True  # raw thresholds already
        self.tree_count += 1
        self.last_stats = TimeStats()
        self.last_stats.total = time.perf_counter() - t_start
        self.last_stats.trees = 1
        self.total_stats.add(self.last_stats)
        return tree

    TILE = 1024

    def _pad_layout(self, bnd, cnt, pos_node, K, n):
        """Segment-aligned padded positions: node k's rows start on a tile boundary, so every
        tile of TILE positions belongs to one node."""
        T = self.TILE
        tiles = (cnt + T - 1) // T
        pstart = (torch.cumsum(tiles, 0) - tiles) * T
        ppos = torch.arange(n, device=self.dev) - bnd[:-1][pos_node] + pstart[pos_node]
        ntile = int(tiles.sum())
        tile_seg = torch.repeat_interleave(torch.arange(K, device=self.dev), tiles)
        return ppos, ntile, tile_seg, K

    def _seg_argmax(self, chg: torch.Tensor, pad):
        """(first position of the max, the max) of chg [C, n] over each node segment."""
        ppos, ntile, tile_seg, K = pad
        C, n = chg.shape
        T = self.TILE
        u = chg.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        u = torch.where(u >= 0x80000000, 0xFFFFFFFF - u, u | 0x80000000)  # order-preserving
        key = (u << 31) | (0x7FFFFFFF - torch.arange(n, device=self.dev))[None]
        kp = torch.full((C, max(ntile, 1) * T), -1, dtype=torch.int64, device=self.dev)
        kp[:, ppos] = key
        tmax = kp.view(C, -1, T).amax(dim=2)[:, :ntile]
        best = torch.full((C, K), -1, dtype=torch.int64, device=self.dev)
        best.scatter_reduce_(1, tile_seg[None].expand(C, ntile), tmax, "amax")
        pos = (0x7FFFFFFF - (best & 0x7FFFFFFF)).clamp(0, max(n - 1, 0))
        mx = torch.where(best >= 0, torch.gather(chg, 1, pos), torch.full_like(pos, 0, dtype=chg.dtype)
                         .fill_(float("-inf")))
        return pos, mx

    @staticmethod
    def _seg_sums(x: torch.Tensor, bnd: torch.Tensor) -> torch.Tensor:
        """Sums of x [n, ...] over the contiguous segments [bnd[k], bnd[k + 1]) (exact for
        integers): prefix-sum differences, no atomics."""
        xt = x.reshape(x.shape[0], -1).t().contiguous()  # scan along the innermost dimension
        z = torch.zeros((xt.shape[0], 1), dtype=x.dtype, device=x.device)
        cs = torch.cat([z, _row_cumsum(xt)], 1)
        out = (cs[:, bnd[1:]] - cs[:, bnd[:-1]]).t()
        return out.reshape((bnd.numel() - 1,) + tuple(x.shape[1:]))

    def leaf_ids_of(self, tree: Tree) -> torch.Tensor:
        """Leaf node id of every training row (raw-threshold walk; l1 leaf refine)."""
        f, c, l, r, d, v = tree.raw_arrays()
        fl = {"nfeat": f, "nthr": c, "nleft": l, "nright": r, "ndefl": d, "nval": v,
              "troot": np.zeros(1, np.int32), "tout": np.zeros(1, np.int32)}
        fl = {k: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev) for k, a in fl.items()}
        out = torch.zeros((self.N, 1), dtype=torch.int32, device=self.dev)
        gops.forest_predict(self.XT.t().contiguous(), fl, None, 1.0, leaf_out=out)
        return out[:, 0].to(torch.int64)

    def _resegment(self, order, pos_node, bnd, go_feat, go_thr, K):
        """Children segments of the split nodes, stably partitioned in every column; rows of
        nodes that became leaves leave the order. Returns (order, pos_node, segments)."""
        dev = self.dev
        n = order.shape[1]
        rows0 = order[0]
        split = go_feat >= 0                                  # [K]
        nf = go_feat[pos_node].clamp(min=0)
        val = self.XT[nf, rows0]                              # row's value of its node's split feature
        left_row = torch.zeros(self.N, dtype=torch.bool, device=dev)
        left_row[rows0] = val < go_thr[pos_node]              # resetPosition: value < cond -> left
        alive_pos = split[pos_node]                           # rows staying in the order
        # children sizes (identical for every column)
        nl = self._seg_sums((left_row[rows0] & alive_pos).to(torch.int64), bnd)
        cnt = bnd[1:] - bnd[:-1]
        nr = torch.where(split, cnt - nl, torch.zeros_like(cnt))
        nl = torch.where(split, nl, torch.zeros_like(nl))
        sizes = torch.stack([nl, nr], 1).reshape(-1)          # child order: (left, right) per node
        cbeg = torch.cumsum(sizes, 0) - sizes                 # new segment begins
        n_new = int(sizes.sum())
        new_order = torch.empty((self.F, n_new), dtype=torch.int64, device=dev)
        for c0 in range(0, self.F, self.chunk):
            o = order[c0:c0 + self.chunk]
            C = o.shape[0]
            lf = left_row[o]                                  # [C, n]
            alive = alive_pos[None].expand(C, n)
            li = (lf & alive).to(torch.int64)
            ri = ((~lf) & alive).to(torch.int64)
            lc = _row_cumsum(li) - li                         # lefts before i (whole column)
            rcs = _row_cumsum(ri) - ri
            lbase = lc[:, bnd[:-1].clamp(max=max(n - 1, 0))]  # [C, K] at each node start
            rbase = rcs[:, bnd[:-1].clamp(max=max(n - 1, 0))]
            k2 = 2 * pos_node[None].expand(C, n)
            dest = torch.where(lf, cbeg[k2] + lc - lbase[:, pos_node], cbeg[k2 + 1] + rcs - rbase[:, pos_node])
            dest = torch.where(alive, dest, torch.full_like(dest, n_new))  # dropped rows -> scratch column
            tmp = torch.empty((C, n_new + 1), dtype=torch.int64, device=dev)
            tmp.scatter_(1, dest, o)
            new_order[c0:c0 + C] = tmp[:, :n_new]
        nz = sizes > 0
        segs_all = list(zip(cbeg.cpu().tolist(), (cbeg + sizes).cpu().tolist()))
        # expand-order children of the split nodes (empty children are still tree nodes)
        seg = [segs_all[2 * k + j] for k in torch.nonzero(split).flatten().cpu().tolist() for j in (0, 1)]
        node_of = torch.repeat_interleave(torch.arange(2 * K, device=dev)[nz], sizes[nz])
        # renumber child slots 2k / 2k+1 of split nodes to 0 .. 2 * nsplit - 1
        remap = torch.full((2 * K,), -1, dtype=torch.int64, device=dev)
        sk = torch.nonzero(split).flatten()
        remap[torch.stack([2 * sk, 2 * sk + 1], 1).reshape(-1)] = torch.arange(2 * sk.numel(), device=dev)
        return new_order, remap[node_of], seg
