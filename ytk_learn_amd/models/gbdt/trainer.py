"""GBDT training driver (gradient boosting and random forest).

Reference: ``J/optimizer/GBDTOptimizer.java`` (init :211-335, train loop :406-480,
doBoost :482-488, predictAndCalcLossGrad :513-609, convertModel :663-690) and
``J/operation/GBDTOperation.java``.

Device-resident design: raw test features, binned train matrix (row- and
column-major), scores, predictions, labels, weights and (g, h) live in HBM for the
whole run. On a GPU with level-wise growth the tree builder is GPU-resident too
(``device_builder.py``): a boosting round is enqueued without any host
synchronisation; the host only reads loss scalars when it logs and converts the
device node tables into model trees lazily (``materialize``).
"""
from __future__ import annotations

import os
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from ...losses import create_loss
from ...metrics.evaluators import EvalSet
from ...ops import gbdt as gops
from ...ops._ext import hip
from ...parallel.comm import Comm
from ...utils.javafmt import java_double_str as jd
from ...utils.fault import fault_point
from ...utils.logging import get_logger
from ...utils.timestats import PhaseTimer, profiling_enabled
from .binning import BinMapper, SamplerSpec, compute_missing_fill
from .builder import TimeStats, TreeBuilder, TreeParams
from .device_builder import (MAX_DEPTH_DEVICE, MAX_LEVEL_NODES, DeviceLevelBuilder,
                             level_slots_pingpong, level_width, node_table_to_tree)
from .device_leafwise import DeviceLeafBuilder
from .exact import ExactGreedyBuilder
from .refine import TreeRefiner
from .tree import CandTable, GBDTModel, Tree


@dataclass
class GBDTParams:
    round_num: int = 50
    loss_function: str = "sigmoid"
    class_num: int = 1
    type: str = "gradient_boosting"  # | random_forest
    uniform_base_prediction: float = 0.5
    sample_dependent_base_prediction: bool = False
    sigmoid_zmax: float = 0.0
    lad_refine_appr: bool = True
    eval_metric: List[str] = field(default_factory=lambda: ["auc"])
    watch_train: bool = False
    watch_test: bool = False
    split_type: str = "mean"
    missing_value: str = "value"
    approximate: List[dict] = field(default_factory=lambda: [{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255}])
    dump_freq: int = -1
    verbose: bool = False
    device_builder: bool = True  # use the GPU-resident builder when applicable
    tree_maker: str = "data"      # "data" (histogram, data parallel) | "feature" (exact greedy)
    histogram_pool_capacity: float = -1.0
    just_evaluate: bool = False
    filter_threshold: int = 0
    tree: TreeParams = field(default_factory=TreeParams)


@dataclass
class GBDTData:
    """One dataset shard on a device. X is raw float features (NaN = missing)."""
    X: torch.Tensor                     # [N, F] float32
    y: torch.Tensor                     # [N, K] float32
    weight: Optional[torch.Tensor] = None  # [N] float32
    init_pred: Optional[torch.Tensor] = None  # [N, K] prediction-space init (sample dependent)

    @property
    def n(self):
        return self.X.shape[0]


class GBDTTrainer:
    def __init__(self, params: GBDTParams, train: GBDTData, test: Optional[GBDTData] = None,
                 comm: Optional[Comm] = None, feature_names: Optional[Sequence[str]] = None,
                 model: Optional[GBDTModel] = None, log=None, profile: bool = False):
        self.p = params
        self.comm = comm or Comm.local(train.X.device)
        self.dev = train.X.device
        self.train_data = train
        self.test_data = test
        self.F = train.X.shape[1]
        self.K = params.class_num
        self.feature_names = list(feature_names) if feature_names is not None else [str(i) for i in range(self.F)]
        self.log = log or get_logger(self.comm)
        self.loss = create_loss(params.loss_function)
        if params.loss_function.lower().startswith("sigmoid"):
            self.loss.set_param(sigmoid_zmax=params.sigmoid_zmax)
        self.rf = params.type == "random_forest"
        self.model = model or GBDTModel(params.uniform_base_prediction, self.K, self.loss.name)
        self.profile = profiling_enabled(profile or None)
        self.timer = PhaseTimer(self.dev, self.profile)
        self.kernel_loss = self.loss.gbdt_kernel_id
        self._prepared = False
        self._acc = None            # (train acc, test acc) device tensors of the last round
        self.rounds_done = 0
        # rounds whose trees / losses are still in flight: (round, dev trees, host buffer, event)
        self._inflight = deque()
        self._rb_free = []          # recycled pinned readback buffers
        self.round_losses = {}      # round -> (train loss, test loss), filled as rounds land
        self._round_stats = {}      # round -> phase times of THAT round (for the metric sink)
        self._names_arr = None
        self._graphs = None         # captured rounds (see _graph_round)
        self._graph_hosts = set()   # pinned readback buffers owned by captured graphs
        self._rb_dev = None         # the round's [train | test | leaf counts] vector (see _step_dev)
        self._eager_rounds = 0

    # ------------------------------------------------------------ preparation
    def _specs(self) -> List[SamplerSpec]:
        default = SamplerSpec()
        per_col = {}
        name2idx = {n: i for i, n in enumerate(self.feature_names)}
        for ent in self.p.approximate:
            spec = SamplerSpec.from_dict(ent)
            cols = str(ent.get("cols", "default"))
            if cols == "default":
                default = spec
            else:
                for c in cols.split(","):
                    c = c.strip()
                    if c in name2idx:
                        per_col[name2idx[c]] = spec
        return [per_col.get(i, default) for i in range(self.F)]

    def _base_score(self, data: GBDTData) -> torch.Tensor:
        base = float(np.float32(self.loss.pred2score(self.p.uniform_base_prediction)))
        init = torch.full((data.n, self.K), base, dtype=torch.float32, device=self.dev)
        if self.p.sample_dependent_base_prediction and data.init_pred is not None:
            init += self.loss.pred2score(data.init_pred.double()).float()
        return init

    def prepare(self):
        t0 = time.perf_counter()
        tr = self.train_data
        # missing values (FillMissingValue): computed on train, applied to train/test
        self.missing_fill = compute_missing_fill(tr.X, tr.weight, self.p.missing_value, self.comm)
        self.fill_dev = torch.from_numpy(self.missing_fill).to(self.dev)
        Xf = torch.where(torch.isnan(tr.X), self.fill_dev[None, :], tr.X)
        # tree_maker = "feature": exact greedy on presorted raw columns (no binning at all)
        self.exact = self.p.tree_maker == "feature" and os.environ.get("YTK_EXACT_BINNED", "0") != "1"
        if self.exact:
            self._prepare_exact(Xf)
            return
        self.mapper = BinMapper.fit(Xf, tr.weight, self._specs(), self.comm, self.p.split_type,
                                    seed=self.p.tree.seed)
        self.bins, self.binsT = self.mapper.transform(Xf)
        del Xf
        self.B = self.mapper.hist_bins()
        self.cand_dev = torch.from_numpy(np.concatenate(self.mapper.cands).astype(np.float32)).to(self.dev)
        self.coff_dev = torch.from_numpy(np.concatenate(
            [[0], np.cumsum([len(c) for c in self.mapper.cands])]).astype(np.int32)).to(self.dev)
        self.refiner = TreeRefiner(self.comm, self.p.lad_refine_appr) if self.loss.name == "l1" else None
        tp = self.p.tree
        # histogram_pool_capacity (MB, DataParallelTreeMaker.java:192-204): the level engine
        # honours a pool below its full slab with two alternating level regions (the only live
        # histograms: a level's and its parents', level_slots_pingpong); the leaf-wise engine keeps
        # every speculative node's slot resident, so a pool below that slab (or below the level
        # engine's two regions) sends the run to the host-driven builder, whose LRU pool honours
        # the cap (HistogramPool.java:36-273)
        pool_mb = self.p.histogram_pool_capacity
        slot_bytes = self.B * self.F * 16
        pool_slots = (int(pool_mb * (1 << 20) // slot_bytes)
                      if (pool_mb is not None and pool_mb > 0) else None)

        def fits_pool(n_slots: int) -> bool:
            return pool_slots is None or n_slots <= pool_slots

        lvl_ncs = 1 if self.comm.is_dist else 0  # the multi-GPU count slots (one per level)
        self.use_device_builder = (self.p.device_builder and self.dev.type == "cuda" and tp.grow_policy == "level"
                                   and 1 <= tp.max_depth <= MAX_DEPTH_DEVICE and level_width(tp) <= MAX_LEVEL_NODES
                                   and fits_pool(level_slots_pingpong(tp, lvl_ncs))
                                   and DeviceLevelBuilder.supports(self.bins, self.binsT, self.B, self.F))
        # leaf-wise (the reference's Higgs configuration): GPU-resident queue replay
        use_leaf = (not self.use_device_builder and self.p.device_builder and self.dev.type == "cuda"
                    and tp.grow_policy == "loss"
                    and fits_pool(DeviceLeafBuilder.slots_needed(tp))
                    and DeviceLeafBuilder.supports(self.bins, self.binsT, self.B, self.F, tp, self.comm))
        if (self.p.device_builder and self.dev.type == "cuda" and pool_mb is not None and pool_mb > 0
                and not (self.use_device_builder or use_leaf)):
            need = (level_slots_pingpong(tp, lvl_ncs) if tp.grow_policy == "level"
                    else DeviceLeafBuilder.slots_needed(tp))
            if not fits_pool(need):  # not silent: the capped pool costs the GPU engines
                self.log.info(f"[GBDT] histogram_pool_capacity {pool_mb:g} MB < the GPU engine's resident "
                              f"histogram slab ({need} slots x {slot_bytes / (1 << 20):.2f} MB): the tree is "
                              f"grown by the host-driven builder, whose LRU pool honours the cap (the model is "
                              f"the same; set histogram_pool_capacity = -1 to keep the GPU engine)")
        if use_leaf:
            self.use_device_builder = True
            self.builder = DeviceLeafBuilder(self.bins, self.binsT, self.F, self.B, self.mapper.nbins, tp, self.comm,
                                             timer=self.timer)
            # the builder waits on its planner while a tree grows: land the previous rounds
            # (tree conversion, loss log) in that wait instead of between trees (multi-GPU:
            # the host gap between trees cost +9 % per leaf-wise tree at the 1/8 shard,
            # profiles/r5). Landing a round that logs eval metrics runs their collectives
            # (distributed AUC), and ranks reach this wait at different batches of their trees
            # -- a rank blocked in a host collective here would wait on a peer whose GPU waits
            # on this rank's not-yet-enqueued batch exchange -- so on several ranks the hook
            # stops before such a round (run_round lands it after the tree)
            if not self.comm.is_dist:
                self.builder.idle_hook = lambda: self._drain(0)
            else:
                self.builder.idle_hook = lambda: self._drain(0, collective_free=True)
            self.builder.snapshot_copy = self.K != 1
            self._fuse_root_pending = True
        elif self.use_device_builder:
            self.builder = DeviceLevelBuilder(self.bins, self.binsT, self.F, self.B, self.mapper.nbins, tp, self.comm,
                                              timer=self.timer, pool_slots=pool_slots)
            # the fused K == 1 gradient pass counts the rows per leaf: the level engine's last
            # level skips its counting partition (and, multi-GPU, the count all-reduce: the
            # counts ride in the round's loss all-reduce)
            self.builder.snapshot_copy = self.K != 1
            self._fuse_root_pending = True  # decided once the gradient bound is known (below)
            self.builder.defer_leaf_counts = (self.K == 1 and self.kernel_loss is not None
                                              and self.kernel_loss != "softmax"
                                              and gops.leaf_counts_fit(self.builder.max_nodes)
                                              and os.environ.get("YTK_DEFER_LEAF_COUNTS", "1") != "0")
        else:
            self.builder = TreeBuilder(self.bins, self.binsT, self.F, self.B, self.mapper.nbins, tp,
                                       self.comm, profile=self.profile,
                                       pool_mb=self.p.histogram_pool_capacity)
        self._finish_prepare(t0)
        nb = self.mapper.nbins
        self.log.info(f"[GBDT] generate sorted global feature bins complete! feature dim:{self.F}, "
                      f"total feature bin cnt:{int(nb.sum())}")

    def _finish_prepare(self, t0: float):
        """Score / gradient buffers, loss bounds, test set, evaluators (every tree maker)."""
        tr = self.train_data
        tp = self.p.tree
        N = tr.n
        self.score = torch.zeros((N, self.K), dtype=torch.float32, device=self.dev)
        self.init_score = self._base_score(tr)
        self.pred = torch.zeros((N, self.K), dtype=torch.float32, device=self.dev)
        self.gh = torch.zeros((self.K, N, 2), dtype=torch.float32, device=self.dev)
        # max |g|, |h| per class, produced by the gradient kernel for the next trees' scales
        self.ghmax = torch.zeros((self.K, 2), dtype=torch.float32, device=self.dev)
        self.y = tr.y.contiguous()
        self.w = tr.weight.contiguous() if tr.weight is not None else None
        sums = self.comm.allreduce_scalars([float(tr.weight.sum()) if tr.weight is not None else float(N), float(N)])
        self.train_wsum, self.train_real = sums
        # Sigmoid: |g| <= w and h <= w * max(1/4, 1/zmax) for every row, so the fixed-point
        # scales come from this global bound instead of a per-tree max all-reduce (one RCCL
        # latency less per tree). Used on any world size -> trees stay bitwise identical.
        self.ghmax_fixed = None
        if self.kernel_loss == "sigmoid" and self.K == 1 and os.environ.get("YTK_GH_BOUND", "1") != "0":
            wmax = float(tr.weight.max()) if (tr.weight is not None and N > 0) else 1.0
            wmax = self.comm.allreduce_scalars([wmax], op="max")[0]
            zmax = float(self.p.sigmoid_zmax)
            hb = max(0.25, 1.0 / zmax) if zmax > 0 else 0.25
            self.ghmax_fixed = torch.tensor([wmax, wmax * hb], dtype=torch.float32, device=self.dev)
        if getattr(self, "_fuse_root_pending", False):
            # the K == 1 gradient pass also builds the next tree's root histogram: needs the
            # fixed-point scales fixed before the pass (the sigmoid bound), every row in the
            # root (no row sampling) and the 32-byte uint8 rows of the 32-feature LDS histogram
            b = self.builder
            b.fuse_root = (self.ghmax_fixed is not None and self.K == 1 and tp.instance_sample_rate >= 1.0
                           and self.refiner is None and not b.wide and b.staged
                           and self.bins.dtype == torch.uint8 and self.bins.stride(0) == 32
                           and self.F <= 32 and self.B <= 256
                           and os.environ.get("YTK_FUSE_ROOT_HIST", "1") != "0")
            self._fuse_root_pending = False
        if self.test_data is not None:
            te = self.test_data
            self.Xte = torch.where(torch.isnan(te.X), self.fill_dev[None, :], te.X).contiguous()
            if (isinstance(getattr(self, "builder", None), (DeviceLevelBuilder, DeviceLeafBuilder)) and self.K == 1
                    and self.refiner is None):
                # the tree-tail launch writes the raw-threshold tree for the test-set pass (one
                # persistent set of arrays: K > 1 rounds keep one raw tree per class; l1 refines
                # the leaf values after the build)
                self.builder.set_raw_request(self.cand_dev, self.coff_dev, self.fill_dev, self.p.split_type == "median")
            self.te_score = torch.zeros((te.n, self.K), dtype=torch.float32, device=self.dev)
            self.te_init = self._base_score(te)
            self.te_pred = torch.zeros((te.n, self.K), dtype=torch.float32, device=self.dev)
            self.te_gh = torch.zeros((self.K, te.n, 2), dtype=torch.float32, device=self.dev)
            sums = self.comm.allreduce_scalars([float(te.weight.sum()) if te.weight is not None else float(te.n),
                                                float(te.n)])
            self.te_wsum, self.te_real = sums
        self.eval_train = EvalSet(self.p.eval_metric, self.comm)
        self.eval_test = EvalSet(self.p.eval_metric, self.comm)
        self._one_tree = {k: (torch.zeros(1, dtype=torch.int32, device=self.dev),
                              torch.full((1,), k, dtype=torch.int32, device=self.dev)) for k in range(self.K)}
        if self.model.trees:  # continue-train: replay loaded trees on train/test scores
            self._replay_loaded_trees()
        self.rounds_done = len(self.model.trees) // self.K
        self._prepared = True
        self.prep_time = time.perf_counter() - t0

    def _prepare_exact(self, Xf: torch.Tensor):
        """Exact-greedy maker (FeatureParallelTreeMakerByLevel): presorted raw columns; the
        round's train scores come from raw-threshold walks of the new trees."""
        t0 = time.perf_counter()
        tp = self.p.tree
        self.Xtr = Xf.contiguous()
        self.mapper = None
        self.bins = self.binsT = None
        self.B = 0
        self.use_device_builder = False
        self.refiner = TreeRefiner(self.comm, self.p.lad_refine_appr) if self.loss.name == "l1" else None
        self.builder = ExactGreedyBuilder(self.Xtr, tp, self.comm)
        self._finish_prepare(t0)
        self.log.info(f"[GBDT] exact greedy (presorted columns) ready! feature dim:{self.F}, rows:{self.Xtr.shape[0]}")

    def _replay_loaded_trees(self):
        """continue_train: score existing trees with raw features (isOriginTree)."""
        name2idx = {n: i for i, n in enumerate(self.feature_names)}
        for t in self.model.trees:
            t.update_feature_index(name2idx)
        fl = {k: torch.from_numpy(v).to(self.dev) for k, v in self.model.flatten().items()}
        Xf = torch.where(torch.isnan(self.train_data.X), self.fill_dev[None, :], self.train_data.X).contiguous()
        gops.forest_predict(Xf, fl, self.score, 1.0)
        if self.test_data is not None:
            gops.forest_predict(self.Xte, fl, self.te_score, 1.0)

    # ------------------------------------------------------------ loss / grad
    def _score_div(self, rounds_done: int) -> float:
        if self.rf:
            return float(rounds_done if rounds_done > 0 else 1)
        return 1.0

    def _kparam(self):
        return self.p.sigmoid_zmax if self.kernel_loss == "sigmoid" else getattr(self.loss, "delta", 0.0)

    def _loss_grad(self, score, init, y, w, pred, gh, rounds_done, want_grad=True):
        div = self._score_div(rounds_done)
        if self.kernel_loss is not None:
            ghmax = None
            if want_grad:
                ghmax = self.ghmax
                ghmax.zero_()
            return gops.grad_hess(score, init, y, w, self.kernel_loss, self._kparam(), div, pred, gh, want_grad,
                                  ghmax)
        # generic loss (torch on device): GBDT derivative from the float prediction
        z = score.double() / div + init.double()
        yy = y.double()
        ww = w.double() if w is not None else torch.ones(score.shape[0], dtype=torch.float64, device=score.device)
        if self.loss.multi:
            lv = self.loss.loss(z, yy)
            p = self.loss.predict(z)
        else:
            lv = self.loss.loss(z[:, 0], yy[:, 0])[:, None]
            p = self.loss.predict(z)
        pred.copy_(p.float())
        if want_grad:
            g, h = self.loss.fast_deriv(pred.double(), yy)
            gh[:, :, 0] = (g * ww[:, None]).float().t()
            gh[:, :, 1] = (h * ww[:, None]).float().t()
            self.ghmax.copy_(gh.abs().amax(dim=1))
        return torch.stack([(lv.reshape(lv.shape[0], -1).sum(1) * ww).sum(), ww.sum()])

    def init_gradients(self):
        """initPred: prediction, loss and gradients of the current model."""
        r = self.rounds_done
        acc = self._loss_grad(self.score, self.init_score, self.y, self.w, self.pred, self.gh, r)
        acc_te = None
        if self.test_data is not None:
            te = self.test_data
            acc_te = self._loss_grad(self.te_score, self.te_init, te.y, te.weight, self.te_pred, self.te_gh, r, False)
        self._acc = (acc, acc_te)

    # ------------------------------------------------------------------ train
    def train(self, rounds: Optional[int] = None, on_round: Optional[Callable[[int, "GBDTTrainer"], None]] = None,
              dump_cb: Optional[Callable[[int], None]] = None):
        if not self._prepared:
            self.prepare()
        p = self.p
        total_rounds = p.round_num if rounds is None else rounds
        cur = self.rounds_done
        self.log.info(f"gbdt start train! total round_num={total_rounds}, current round_num={cur}")
        self.init_gradients()
        self._train_start = time.perf_counter()
        for i in range(cur, total_rounds):
            fault_point("gbdt", i, self.comm.rank)
            self.run_round(i)
            if on_round is not None:
                self.materialize()
                on_round(i, self)
            # GBDTOptimizer.java:434-435 -- note Java's (i+1) % -1 == 0 dumps every round
            if dump_cb is not None and p.dump_freq != 0 and ((i + 1) % p.dump_freq == 0):
                self.materialize()
                dump_cb(i)
        self.materialize()
        self.total_train_time = time.perf_counter() - self._train_start
        final = self.final_eval()
        self.log.info(f"training end, {self.total_train_time:.5f} sec in all\n{final}")
        if self.profile:
            self.log.info(self.timer.report() if self.use_device_builder else f"[GBDT] {self.builder.total_stats}")
        return self.model

    def run_round(self, i: int, lag: int = 1):
        """One reference round (GBDTOptimizer.java:406-462): build the tree(s), update the
        train score + gradients, score the test set, then -- pipelined -- read the round's
        trees and (train, test) losses back through pinned memory and convert / log them.
        With ``lag`` = 1 the host converts round i-1 while the GPU runs round i, so the
        model conversion and the per-round loss readback cost no GPU idle time. Rounds that
        log eval metrics (watch_train / watch_test) drain synchronously: the metrics read
        the current predictions."""
        if not hasattr(self, "_train_start"):
            self._train_start = time.perf_counter()
        self.timer.begin()
        self.step(i)
        per = self.timer.end()
        if per:  # this round's phase times, logged when the round lands (one round later)
            self._round_stats[i] = dict(per)
        logs = self.p.verbose or self.log.enabled_for_round(i)
        if per and logs:
            self.log.info(f"[GBDT] time stats tree {i + 1}: {PhaseTimer.fmt(per)}")
        elif self.profile and not self.use_device_builder and logs:
            self.log.info(f"[GBDT] time stats tree {i + 1}: {self.builder.last_stats}")
        watch = logs and (self.p.watch_train or self.p.watch_test)
        self._drain(0 if watch else lag)

    # ----------------------------------------------------------- readback pipe
    def _rb_buffer(self, nbytes: int) -> torch.Tensor:
        while self._rb_free:
            buf = self._rb_free.pop()
            if buf.numel() >= nbytes:
                return buf
        buf = torch.empty(max(nbytes, 64), dtype=torch.uint8)
        return buf.pin_memory() if self.dev.type == "cuda" else buf

    def _enqueue_readback(self, i: int, dev_trees, acc, acc_te):
        """Copy the round's tree snapshots + loss sums into one pinned buffer (async)."""
        self._bound_inflight()
        accs, nlc = self._readback_accs(dev_trees, acc, acc_te)
        self._readback_copy(i, dev_trees, accs, acc_te is not None, nlc)

    def _bound_inflight(self):
        while len(self._inflight) >= 4:  # bounded: at most 4 rounds in flight
            self._drain(len(self._inflight) - 1)

    def _readback_accs(self, dev_trees, acc, acc_te):
        """Device side of the readback: the round's loss sums (+ leaf counts) in one vector."""
        rbd = getattr(self, "_rb_dev", None)
        if rbd is not None:  # already one vector (_step_dev's round tail)
            self._rb_dev = None
            accs, nlc = rbd
            if self.comm.is_dist:
                self._round_allreduce(accs)
            return accs, nlc
        accs = torch.stack([acc, acc_te if acc_te is not None else torch.zeros_like(acc)]).to(self.dev).reshape(-1)
        # rows per leaf from the gradient pass (level engine, deferred last-level counts):
        # local counts, summed across ranks by the same all-reduce as the losses
        lcs = [getattr(dt, "leaf_counts", None) for dt in dev_trees]
        nlc = [0 if c is None else c.numel() for c in lcs]
        if any(nlc):
            accs = torch.cat([accs] + [c for c in lcs if c is not None])
        if self.comm.is_dist:
            self._round_allreduce(accs)  # GBDTOptimizer.java:502 (loss, weight) allreduce
        return accs, nlc

    def _round_allreduce(self, accs: torch.Tensor):
        """The round's (loss, weight | leaf counts) vector: the engine's peer-memory exchange
        (fp64, rank-order sums) when it has one, else the process group."""
        peer = getattr(self.builder, "peer", None)
        if peer is not None and peer.fits(accs):
            peer.allreduce_(accs)
        else:
            self.comm.allreduce_(accs)

    def close(self):
        """Release the engine's device resources shared with other ranks (the peer-memory
        group). Collective on multi-GPU runs: every rank calls it after its last round."""
        self.materialize()
        close = getattr(self.builder, "close", None)
        if close is not None:
            close()

    def _readback_copy(self, i: int, dev_trees, accs, has_te: bool, nlc):
        """Host side: async copies into a pinned buffer + an event; landed by _drain."""
        dt0 = dev_trees[0] if len(dev_trees) == 1 else None
        rv_off = getattr(dt0, "rv_off", None)
        if rv_off is not None and accs.data_ptr() == dt0.snap.data_ptr() + rv_off:
            # the round vector sits right behind the snapshot: ONE copy of [snap | pad | vector]
            nb = rv_off + 8 * accs.numel()
            host = self._rb_buffer(nb)
            host[:nb].copy_(dt0.snap_full[:nb], non_blocking=True)
            ev = None
            if self.dev.type == "cuda":
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.dev))
            self._inflight.append((i, dev_trees, host, ev, has_te, nlc, rv_off))
            return
        sizes = [dt.snap.numel() for dt in dev_trees]
        head = 8 * accs.numel()
        host = self._rb_buffer(head + sum(sizes))
        host[:head].view(torch.float64).copy_(accs, non_blocking=True)
        off = head
        for dt, sz in zip(dev_trees, sizes):
            host[off:off + sz].copy_(dt.snap, non_blocking=True)
            off += sz
        ev = None
        if self.dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
        self._inflight.append((i, dev_trees, host, ev, has_te, nlc, None))

    def _lands_with_collectives(self, i: int) -> bool:
        """Landing round i logs eval metrics of the current predictions (watch_train /
        watch_test on a logged round): their evaluators all-reduce across ranks."""
        logs = self.p.verbose or self.log.enabled_for_round(i)
        return bool(logs and (self.p.watch_train or self.p.watch_test) and i + 1 == self.rounds_done)

    def _drain(self, lag: int = 0, collective_free: bool = False):
        """Land every in-flight round but the newest ``lag``: trees -> model, losses -> log.
        ``collective_free``: stop before a round whose landing runs collectives."""
        while len(self._inflight) > lag:
            if (collective_free and self.comm.is_dist
                    and self._lands_with_collectives(self._inflight[0][0])):
                return
            i, dev_trees, host, ev, has_te, nlc, rv_off = self._inflight.popleft()
            if ev is not None:
                ev.synchronize()
            for peer in (getattr(self.builder, "peer", None), getattr(self.builder, "peer2", None)):
                if peer is not None:  # a timed-out flag wait (lost / stalled peer) fails the job here
                    peer.check()
            hb = host.numpy()
            head = 32 + 8 * sum(nlc)
            if rv_off is None:  # [vector | snapshots]
                a = hb[:head].view(np.float64)
                off = head
            else:  # [snapshot | pad | vector]
                a = hb[rv_off:rv_off + head].view(np.float64)
                off = 0
            coff = 4
            for dt, nc in zip(dev_trees, nlc):
                sz = dt.snap.numel()
                nodes_b, st = dt.split_host_snap(hb[off:off + sz])
                tree = node_table_to_tree(nodes_b, st)
                if nc:  # leaf sample counts from the gradient pass
                    cnt = a[coff:coff + nc]
                    coff += nc
                    leaf = np.asarray(tree.is_leaf, bool)
                    sc = np.asarray(tree.sample_cnt, np.int64)
                    sc[leaf] = np.rint(cnt[:leaf.size][leaf]).astype(np.int64)
                    tree.sample_cnt = sc.tolist()
                self._convert(tree)
                self.model.trees.append(tree)
                off += sz
            trl = float(a[0]) / max(self.train_wsum, 1e-300)
            tel = float(a[2]) / max(self.te_wsum, 1e-300) if has_te else None
            if host.data_ptr() not in self._graph_hosts:  # graph-owned buffers stay with their graph
                self._rb_free.append(host)
            self.round_losses[i] = (trl, tel)
            self._log_round(i, trl, tel, current=(i + 1 == self.rounds_done))

    def _log_round(self, i: int, trl: float, tel: Optional[float], current: bool):
        stats = self._round_stats.pop(i, None)
        if not (self.p.verbose or self.log.enabled_for_round(i)):
            return
        metric = getattr(self.log, "metric", None)
        if metric is not None:
            metric(model="gbdt", loss=self.loss.name, round=i + 1, train_loss=trl, test_loss=tel,
                   time_stats=stats if self.timer.enabled else None)
        out = [f"train loss = {jd(trl)}\n"]
        if self.p.watch_train and current:
            out.append(self._eval_str(True))
        if tel is not None:
            out.append(f"test loss = {jd(tel)}\n")
            if self.p.watch_test and current:
                out.append(self._eval_str(False))
        cost = time.perf_counter() - getattr(self, "_train_start", time.perf_counter())
        self.log.info(f"[model=gbdt] [loss={self.loss.name}] [iter={i + 1}]  {cost:.5f} sec elapse\n"
                      + "".join(out))

    def _tree_to_dev(self, tree):
        """Bin-threshold node arrays of a host tree packed into one H2D copy."""
        f, t, l, r, v = tree.bin_arrays()
        n = f.shape[0]
        packed = np.concatenate([f, t, l, r, v.view(np.int32)]).astype(np.int32)
        d = torch.from_numpy(packed)
        if self.dev.type == "cuda":
            d = d.pin_memory().to(self.dev, non_blocking=True)
        return (d[:n], d[n:2 * n], d[2 * n:3 * n], d[3 * n:4 * n], d[4 * n:5 * n].view(torch.float32))

    def step(self, i: int):
        """One boosting round: K trees, score update, loss + next gradients, test scoring.
        Enqueues device work only (no host synchronisation on the device-builder path)."""
        if self._graph_eligible() and self._graph_round(i):
            return
        self._graph_release()
        dev_trees, acc, acc_te, _ = self._step_dev(i)
        self._acc = (acc, acc_te)
        self.rounds_done = i + 1
        self._eager_rounds += 1
        self._enqueue_readback(i, dev_trees, acc, acc_te)

    # ------------------------------------------------------------ graph rounds
    def _graph_eligible(self) -> bool:
        """A level-engine round is a fixed launch sequence with device-resident counts, so on
        one GPU the whole round (tree, score/gradient + next root histogram, test scoring,
        loss vector) can be captured once and replayed: the host then spends one graph launch
        instead of ~45 kernel launches and the Python around them per round (at a 1/8 shard the
        eager host work, ~0.44 ms per round, was as long as the GPU work). Only rounds whose
        launch arguments never change qualify: K == 1, no row / feature sampling, no random
        forest averaging, no L1 refine, no per-phase profiling. Multi-GPU rounds qualify when
        every collective of a round is an RCCL call on device tensors (nccl backend: the
        level messages, the round's loss vector) -- the collectives are captured into the
        graph with the kernels, so a replayed round costs the host one graph launch instead
        of ~45 kernel launches + 7 collective calls (YTK_GRAPH_DIST=0: eager multi-GPU rounds)."""
        if self._graphs is False:
            return False
        tp = self.p.tree
        ok = (self.dev.type == "cuda" and self.use_device_builder and isinstance(self.builder, DeviceLevelBuilder)
              and (not self.comm.is_dist or self._dist_capturable())
              and self.K == 1 and self.kernel_loss not in (None, "softmax")
              and not self.rf and self.refiner is None and not self.exact and not self.profile
              and tp.instance_sample_rate >= 1.0 and tp.feature_sample_rate >= 1.0
              and getattr(self.builder, "fuse_root", False) and not self.builder.snapshot_copy
              and os.environ.get("YTK_GRAPH", "1") != "0")
        if not ok:
            self._graph_release()
            self._graphs = False
        return ok

    def _dist_capturable(self) -> bool:
        """Every collective of a multi-GPU round can be captured: RCCL on device tensors, or
        peer-memory exchange kernels (level messages + the round vector; their epochs live in
        device memory, so every replay synchronises afresh) on any backend."""
        if os.environ.get("YTK_GRAPH_DIST", "1") == "0" or self.comm.group is None:
            return False
        if getattr(self.builder, "peer", None) is not None:
            return True
        try:
            return torch.distributed.get_backend(self.comm.group) == "nccl"
        except Exception:
            return False

    def _graph_round(self, i: int) -> bool:
        """Replay the captured round (capturing it first). The engine swaps its row / (g, h)
        ping-pong buffers an odd number of times per tree, so consecutive trees alternate
        between two buffer assignments: two graphs, replayed alternately."""
        if self._graphs is None:
            if self._eager_rounds < 1:  # the first round builds its root eagerly
                return False
            if getattr(self.builder, "tuning", False):  # the overlap auto-tune times eager trees
                return False
            torch.cuda.synchronize(self.dev)
            # the nccl watchdog must hold no eager work while the rounds are captured: its
            # event queries inside a capture abort the process (Comm.drain_pending)
            self.comm.drain_pending()
            b = self.builder
            saved = (b.rows, b.rows_tmp, b.ghp, b.gh_tmp, b.tree_count, b.root_ready)
            graphs, pool, err = [], None, None
            stats0 = dict(self.comm.stats)
            log0 = len(self.comm.log) if self.comm.log is not None else 0
            # in-graph readback (YTK_GRAPH_READBACK=1): each graph ends with a copy kernel of
            # [snapshot | round vector] into ITS OWN pinned buffer (a blit copy launched by the
            # host after every replay cost ~4 us + ~15 us of gaps per round): four graphs, two
            # per ping-pong parity, so a buffer is rewritten only after its round has landed
            # (_bound_inflight keeps at most 4 rounds in flight)
            ngraph = 4 if os.environ.get("YTK_GRAPH_READBACK", "1") != "0" else 2
            try:
                for j in range(ngraph):
                    g = torch.cuda.CUDAGraph()
                    c0 = dict(self.comm.stats)
                    fault = os.environ.get("YTK_FAULT_CAPTURE")  # fault injection (tests): vote + eager fallback
                    # the graph's pinned readback buffer, allocated outside the capture
                    sf = getattr(self.builder, "_snap_full", None)
                    host_j = None
                    if ngraph == 4 and sf is not None:
                        host_j = torch.empty(sf.numel(), dtype=torch.uint8).pin_memory()
                        host_j = (host_j, hip().host_device_ptr(host_j.data_ptr()))
                    # thread_local: only this thread's capture-unsafe calls are checked (the
                    # drain above keeps the watchdog from querying events meanwhile)
                    with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                        dev_trees, acc, acc_te, host_trees = self._step_dev(i)
                        if fault == "2":  # inside the capture: the round's launches half recorded
                            raise RuntimeError("injected failure inside the capture")
                        accs, nlc = self._readback_accs(dev_trees, acc, acc_te)
                        host_j = self._graph_readback(dev_trees, accs, host_j) if host_j is not None else None
                    assert not host_trees
                    if fault == "1":  # after a complete capture
                        raise RuntimeError("injected capture failure")
                    pool = g.pool()
                    # the collectives a replay issues (captured once, counted per replay)
                    coll = {k: self.comm.stats[k] - c0.get(k, 0) for k in self.comm.stats}
                    graphs.append((g, dev_trees, acc, acc_te, accs, nlc, coll, host_j))
            except Exception as e:
                err = e
            if self.comm.is_dist:
                # all ranks replay or none (a rank that fell back alone would still issue the
                # same collectives, but a failed capture is not worth the risk): one host vote
                ok = self.comm.allreduce_scalars([0.0 if err is not None else 1.0], op="min")[0] > 0.5
                if err is None and not ok:
                    err = RuntimeError("another rank could not capture its round")
            if err is not None:  # not capturable here: eager rounds, state as before
                (b.rows, b.rows_tmp, b.ghp, b.gh_tmp, b.tree_count, b.root_ready) = saved
                torch.cuda.synchronize(self.dev)
                self.comm.stats = stats0
                if self.comm.log is not None:
                    del self.comm.log[log0:]
                self.log.info(f"[GBDT] round capture failed ({type(err).__name__}: {err}); eager rounds")
                self._graphs = False
                return False
            self.comm.stats = stats0
            self._graphs = {"g": graphs, "n": 0}
        st = self._graphs
        self._bound_inflight()
        gs = st["g"]
        g, dev_trees, acc, acc_te, accs, nlc, coll, host_j = gs[st["n"] % len(gs)]
        g.replay()
        st["n"] += 1
        for k, v in coll.items():
            self.comm.stats[k] = self.comm.stats.get(k, 0) + v
        self._acc = (acc, acc_te)
        self.rounds_done = i + 1
        if host_j is not None:  # the graph copied the round into host_j: an event only
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self._inflight.append((i, dev_trees, host_j, ev, acc_te is not None, nlc, dev_trees[0].rv_off))
        else:
            self._readback_copy(i, dev_trees, accs, acc_te is not None, nlc)
        return True

    def _graph_readback(self, dev_trees, accs, host_buf):
        """(Inside a round capture) copy kernel of [snapshot | pad | round vector] into the
        graph's pinned buffer (host_buf = (tensor, device address)); None when the round has no
        such contiguous view (the host-launched copy then follows every replay)."""
        host, dptr = host_buf
        dt0 = dev_trees[0] if len(dev_trees) == 1 else None
        rv_off = getattr(dt0, "rv_off", None)
        if rv_off is None or accs.data_ptr() != dt0.snap.data_ptr() + rv_off:
            return None
        nb = (rv_off + 8 * accs.numel() + 15) // 16 * 16
        if nb > min(dt0.snap_full.numel(), host.numel()):
            return None
        self._graph_hosts.add(host.data_ptr())
        hip().copy_to_mapped(dptr, dt0.snap_full.data_ptr(), nb, torch.cuda.current_stream(self.dev).cuda_stream)
        return host

    def _graph_release(self):
        """Leave graph mode (an eager round follows): after an odd number of replays the
        engine's Python-side buffer assignment is one tree behind the device's."""
        st = self._graphs
        if isinstance(st, dict):
            if st["n"] & 1:
                self.builder.swap_ping_pong()
            self._graphs = None

    def _step_dev(self, i: int):
        """The device work of a round; returns (device trees, train acc, test acc, host trees)."""
        lr = 1.0 if self.rf else self.p.tree.learning_rate
        self.builder.p.learning_rate = lr
        arrays, raws, host_trees, dev_trees = [], [], [], []
        for k in range(self.K):
            if self.use_device_builder:
                if self.ghmax_fixed is not None:
                    dt = self.builder.build(self.gh[k], self.ghmax_fixed, ghmax_global=True)
                else:
                    dt = self.builder.build(self.gh[k], self.ghmax[k])
                if self.refiner is not None:  # l1: leaf values -> weighted residual medians, on device
                    self.refiner.refine_device(dt, self.builder, self.y[:, k],
                                               self.score[:, k] / self._score_div(i) + self.init_score[:, k], self.w,
                                               lr)
                dev_trees.append(dt)
                arrays.append(dt.bin_arrays)
                if self.test_data is not None:
                    raw = self.builder.raw_tree(self.cand_dev, self.coff_dev, self.fill_dev,
                                                self.p.split_type == "median")
                    raw["troot"], raw["tout"] = self._one_tree[k]
                    raws.append(raw)
            else:
                tree = self.builder.build(self.gh[k], self.ghmax_fixed if self.ghmax_fixed is not None
                                          else self.ghmax[k], ghmax_global=self.ghmax_fixed is not None)
                if self.refiner is not None:
                    self.refiner.refine(tree, self.builder, self.y[:, k], self.score[:, k] / self._score_div(i)
                                        + self.init_score[:, k], self.w, lr)
                host_trees.append(tree)
                arrays.append(None if self.exact else self._tree_to_dev(tree))
        if self.exact:
            # raw-threshold trees: the round's trees are walked on the filled raw features
            fl = GBDTModel(self.model.base_prediction, self.K, self.model.loss_name)
            fl.trees = host_trees
            gops.forest_predict(self.Xtr, {k: torch.from_numpy(v).to(self.dev) for k, v in fl.flatten().items()},
                                self.score, 1.0)
        if not self.use_device_builder:
            self.timer.mark("build_tree")
        # score update + train loss after this round + gradients for the next round
        self._rb_dev = None
        te_early = None
        if self.K == 1 and self.kernel_loss is not None and self.kernel_loss != "softmax":
            need_max = self.ghmax_fixed is None  # the global bound replaces the per-tree max
            if need_max:
                self.ghmax.zero_()
            want_lc = dev_trees and getattr(self.builder, "defer_leaf_counts", False) and self.builder.last_keep is None
            nlc = arrays[0][0].shape[0] if want_lc else 0
            root = self.builder.root_target() if (dev_trees and getattr(self.builder, "fuse_root", False)) else None
            # Round tail in two launches fewer: the test-set pass runs FIRST with its loss
            # partials left unfinished, the train pass's finish launch completes both, and
            # the (train, test) sums land next to the leaf counts in ONE vector
            # [train loss, weight | test loss, weight | leaf counts] -- the readback is one
            # copy with no stack / cat kernels.
            rb = acc_out = te_acc = None
            if (root is not None and self.test_data is not None and len(raws) == 1
                    and os.environ.get("YTK_FUSED_TEST_TAIL", "1") != "0"
                    and os.environ.get("YTK_ROUND_VECTOR", "1") != "0"):
                te = self.test_data
                rb = (self.builder.round_vector(4 + nlc) if hasattr(self.builder, "round_vector")
                      else torch.empty(4 + nlc, dtype=torch.float64, device=self.dev))
                part = gops.forest_predict_loss(self.Xte, raws[0], self.te_score, self.te_init, te.y, te.weight,
                                                self.kernel_loss, self._kparam(), self._score_div(i + 1),
                                                self.te_pred, finish=False)
                if part is None:
                    rb = None
                else:
                    acc_out, te_acc = rb[0:2], (part[0], part[1], rb[2:4])
                    te_early = rb[2:4]
            lc = None
            if want_lc:
                lc = rb[4:] if rb is not None else torch.empty(nlc, dtype=torch.float64, device=self.dev)
            acc = gops.tree_grad(self.bins, arrays[0], self.score, self.init_score, self.y, self.w,
                                 self.kernel_loss, self._kparam(), self._score_div(i + 1), self.pred, self.gh[0],
                                 True, self.ghmax[0] if need_max else None, leaf_counts=lc, root=root,
                                 acc_out=acc_out, te_acc=te_acc)
            if rb is not None:
                self._rb_dev = (rb, [nlc])
            if root is not None:
                self.builder.root_ready = root["done"]
            if lc is not None:
                dev_trees[0].leaf_counts = lc
        else:
            for k in range(self.K):
                if arrays[k] is not None:
                    gops.tree_add_bins(self.binsT, arrays[k], self.score, k)
            acc = self._loss_grad(self.score, self.init_score, self.y, self.w, self.pred, self.gh, i + 1)
        self.timer.mark("grad_and_score")
        # model conversion (slot -> raw threshold, names, default direction) for host trees,
        # before the test set is scored with their raw thresholds
        for tree in host_trees:
            self._convert(tree)
            self.model.trees.append(tree)
        acc_te = te_early
        if self.test_data is not None and acc_te is None:
            if host_trees:
                fl = GBDTModel(self.model.base_prediction, self.K, self.model.loss_name)
                fl.trees = host_trees
                raws = [{k: torch.from_numpy(v).to(self.dev) for k, v in fl.flatten().items()}]
            te = self.test_data
            if (dev_trees and len(raws) == 1 and self.K == 1 and self.kernel_loss not in (None, "softmax")
                    and os.environ.get("YTK_FUSED_TEST_TAIL", "1") != "0"):
                # the device builder's raw tree (root 0): scoring + loss in one pass
                acc_te = gops.forest_predict_loss(self.Xte, raws[0], self.te_score, self.te_init, te.y, te.weight,
                                                  self.kernel_loss, self._kparam(), self._score_div(i + 1),
                                                  self.te_pred)
            if acc_te is None:
                for raw in raws:
                    gops.forest_predict(self.Xte, raw, self.te_score, 1.0)
                acc_te = self._loss_grad(self.te_score, self.te_init, te.y, te.weight, self.te_pred, self.te_gh,
                                         i + 1, False)
            self.timer.mark("test_eval")
        return dev_trees, acc, acc_te, host_trees

    def _convert(self, tree: Tree):
        """convertModel (GBDTOptimizer.java:663-690): slot -> raw threshold, names, default
        direction -- vectorised per tree."""
        if self._names_arr is None:
            self._names_arr = np.asarray(self.feature_names, dtype=object)
        if self.mapper is not None:  # exact-greedy trees carry raw thresholds already
            if getattr(self, "_cand_tab", None) is None:  # float32 candidate table, built once
                self._cand_tab = CandTable(self.mapper.cands)
            tree.convert_split_values(self._cand_tab, self.p.split_type)
        tree.add_feature_names(self._names_arr)
        tree.add_default_direction(self.missing_fill)

    def materialize(self):
        """Land every in-flight round: device trees -> host model trees, losses -> log."""
        self._drain(0)

    # ------------------------------------------------------------------ report
    def _losses(self):
        acc, acc_te = self._acc
        if acc_te is not None:
            both = torch.stack([acc, acc_te]).cpu()
        else:
            both = acc.cpu()[None, :]
        if self.comm.is_dist:
            self.comm.allreduce_(both)
        tr = float(both[0, 0]) / max(self.train_wsum, 1e-300)
        te = float(both[1, 0]) / max(self.te_wsum, 1e-300) if acc_te is not None else None
        return tr, te

    @property
    def last_train_loss(self):
        return self._losses()[0]

    @property
    def last_test_loss(self):
        return self._losses()[1]

    def report(self) -> str:
        tr_loss, te_loss = self._losses()
        metric = getattr(self.log, "metric", None)
        if metric is not None:
            metric(model="gbdt", loss=self.loss.name, round=self.rounds_done, train_loss=tr_loss, test_loss=te_loss,
                   time_stats=dict(self.timer.last) if self.timer.enabled else None)
        out = [f"train loss = {jd(tr_loss)}\n"]
        if self.p.watch_train:
            out.append(self._eval_str(True))
        if te_loss is not None:
            out.append(f"test loss = {jd(te_loss)}\n")
            if self.p.watch_test:
                out.append(self._eval_str(False))
        return "".join(out)

    @property
    def last_report(self) -> str:
        return self.report()

    def _info(self):
        if self.loss.name == "sigmoid":
            return (2, False)
        if self.loss.name == "softmax":
            return (self.K, True)
        return None

    def _eval_str(self, train: bool) -> str:
        if train:
            wr = abs(self.train_wsum - self.train_real) > 1e-6
            return self.eval_train.eval(self.y, self.pred, self.w, "train", wr, self._info())
        te = self.test_data
        wr = abs(self.te_wsum - self.te_real) > 1e-6
        return self.eval_test.eval(te.y, self.te_pred, te.weight, "test", wr, self._info())

    def final_eval(self) -> str:
        s = self._eval_str(True)
        if self.test_data is not None:
            s += self._eval_str(False)
        return s

    def feature_importance(self):
        self.materialize()
        return self.model.feature_importance()
