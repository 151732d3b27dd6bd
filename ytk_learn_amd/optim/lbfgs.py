"""Distributed L-BFGS with OWL-QN, backtracking line search and hyper-parameter search.

Reference: ``J/optimizer/HoagOptimizer.java``
  lbfgs main loop           :306-811   (initial direction -g, step 1/|g|, then 1.0)
  calcLossAndGrad           :978-1065  (group-wise l2/l1 scaled by the weight sum,
                                        loss double[20] allreduce, grad allreduce,
                                        OWL-QN pseudo-gradient)
  lineSearch                :1068-1201 (orthant projection, Armijo c1, Wolfe c2,
                                        strong Wolfe, step incr/decr, abort codes)
  Hv two-loop               :904-929
  hyper search              :314-434 (grid), :813-902 (HOAG)

MI355X design: w, g, p and the (s, y) history are fp32 device tensors. With P > 1 ranks the
history is SHARDED like the reference's TwoLoop slices (HoagOptimizer.java:441-449): rank r
keeps [r * seg, (r + 1) * seg) of every s and y (seg = ceil(dim / P) rounded to 16 B), so
per-rank history memory and two-loop traffic drop by P. Each two-loop step's dot product is
a local fp64 partial summed over the ranks (one 8-byte all-reduce; the peer-memory exchange
on one node), the ys / yy pair rides one all-reduce, and the finished direction is
all-gathered ONCE (the reference gathers p twice, :904-929; the middle gather is redundant
because the scaling is element-wise). YTK_LBFGS_SHARD=0 keeps the full history on every
rank (redundant two-loop, no two-loop communication). The per-evaluation collectives are
the fp32 gradient all-reduce (RCCL over xGMI or the peer exchange) plus one small fp64 loss
vector. Dots/norms are computed in fp64 on the device; results are identical on every rank
because the all-reduced gradient and the all-reduced dot products are.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch

from ..config.params import HyperParams, LineSearchParams
from ..ops import blas
from ..utils.fault import fault_point
from ..utils.timestats import PhaseTimer, profiling_enabled
from ..utils.javafmt import java_double_str as jd


class ContinuousModel:
    """What the optimizer needs from a model (LinearHoagOptimizer & friends)."""

    name = "model"
    loss_name = "loss"

    def regular_groups(self) -> List[Tuple[int, int]]:  # [start, end) per regularization group
        raise NotImplementedError

    def pure_loss_grad(self, w: torch.Tensor, g: Optional[torch.Tensor]) -> float:
        """Local weighted pure loss; fills g (local gradient, overwritten) when given."""
        raise NotImplementedError

    def test_pure_loss_grad(self, w: torch.Tensor, g: Optional[torch.Tensor]) -> float:
        return float("nan")

    def has_test(self) -> bool:
        return False

    def train_eval(self) -> str:
        return ""

    def test_eval(self) -> str:
        return ""

    def precision(self, w: torch.Tensor, l2: Sequence[float], wsum: float) -> Optional[torch.Tensor]:
        return None

    def dump(self, w: torch.Tensor, precision: Optional[torch.Tensor]):
        pass

    def extra_info(self) -> str:
        return ""

    def other_train_info(self) -> str:
        return ""

    def other_test_info(self) -> str:
        return ""


def _dot(a: torch.Tensor, b: torch.Tensor) -> float:
    return blas.dot(a, b)


def _norm(a: torch.Tensor) -> float:
    return math.sqrt(blas.sum_sq(a))


@dataclass
class LbfgsResult:
    loss: float
    pure_loss: float
    status: int
    iters: int
    test_loss: Optional[float]
    best_l1: List[float]
    best_l2: List[float]


class HoagOptimizer:
    """L-BFGS/OWL-QN driver. ``wsum``/``test_wsum``: GLOBAL weight sums of train/test."""

    def __init__(self, model: ContinuousModel, ls: LineSearchParams, l1: Sequence[float], l2: Sequence[float],
                 comm, log, wsum: float, test_wsum: float = 0.0, hyper: Optional[HyperParams] = None,
                 just_evaluate: bool = False, dump_freq: int = -1):
        self.m = model
        self.ls = ls
        self.l1 = [float(v) for v in l1]
        self.l2 = [float(v) for v in l2]
        self.comm = comm
        self.log = log
        self.W = float(wsum)
        self.Wt = float(test_wsum)
        self.hp = hyper or HyperParams()
        self.just_evaluate = just_evaluate
        self.dump_freq = dump_freq
        self.groups = model.regular_groups()
        if len(self.groups) != len(self.l2):
            raise ValueError(f"{model.name}: {len(self.groups)} regularization groups but "
                             f"{len(self.l2)} l2 values")
        self.need_hyper = bool(self.hp.switch_on) and model.has_test()
        self.hoag = self.need_hyper and self.hp.mode == "hoag"
        self.grid = self.need_hyper and self.hp.mode == "grid"
        self.hyper_idx = 1
        self.loss_prev = 0.0
        self.pure_prev = 0.0
        dev = getattr(model, "device", None)
        self.timer = PhaseTimer(dev if isinstance(dev, torch.device) else None, profiling_enabled())

    # ------------------------------------------------------------------ logging
    def _info(self, it: int, msg: str):
        if self.need_hyper:
            head = f"[model={self.m.name}] [loss={self.m.loss_name}] [hyper={self.hyper_idx}] [iter={it}] "
        else:
            head = f"[model={self.m.name}] [loss={self.m.loss_name}] [iter={it}] "
        self.log.info(head + self.m.extra_info() + msg)

    def _metric(self, it: int, start: float, test_loss: Optional[float]):
        metric = getattr(self.log, "metric", None)
        if metric is not None:
            metric(model=self.m.name, loss=self.m.loss_name, iter=it, hyper=self.hyper_idx,
                   train_loss=self.pure_prev / self.W, regularized_loss=self.loss_prev / self.W,
                   test_loss=(test_loss / self.Wt) if (test_loss is not None and self.Wt > 0) else None,
                   elapsed=time.perf_counter() - start)

    def _verbose(self, it: int, msg: str):
        if getattr(self.log, "verbose", False):
            self._info(it, msg)

    # ------------------------------------------------------------------ loss / grad
    def loss_and_grad(self, w: torch.Tensor, g: torch.Tensor) -> Tuple[float, float]:
        """(pure loss, regularized loss), g = all-reduced (pseudo-)gradient (calcLossAndGrad)."""
        pure = self.m.pure_loss_grad(w, g)
        reg = 0.0
        for r, (s, e) in enumerate(self.groups):
            if e <= s:
                continue
            ws = w[s:e]
            if self.l2[r] > 0.0:
                reg += 0.5 * self.l2[r] * blas.sum_sq(ws)
            if self.l1[r] > 0.0:
                reg += self.l1[r] * blas.sum_abs(ws)
        # local pure loss is summed over ranks; the regularizer is added once with the global W
        tot = torch.tensor([pure], dtype=torch.float64)
        if self.comm is not None and self.comm.is_dist:
            self.comm.allreduce_(tot)
            self._grad_allreduce(g)
        pure = float(tot[0])
        allloss = pure + reg * self.W
        for r, (s, e) in enumerate(self.groups):
            if e <= s:
                continue
            ws, gs = w[s:e], g[s:e]
            if self.l2[r] > 0.0:
                gs.add_(ws, alpha=self.W * self.l2[r])
            if self.l1[r] > 0.0:
                lam = self.W * self.l1[r]
                sign = torch.sign(ws)
                sign[ws == 0] = 1.0
                gs.add_(sign, alpha=lam)
                # OWL-QN pseudo-gradient (HoagOptimizer.java:1040-1062)
                part_pos = gs.double()
                part_neg = torch.where(ws != 0, part_pos, part_pos - 2.0 * lam)
                newg = torch.where(part_neg > 0.0, part_neg, torch.where(part_pos < 0.0, part_pos,
                                                                         torch.zeros_like(part_pos)))
                gs.copy_(newg.float())
        self._peer_landed()
        return pure, allloss

    def _peer_landed(self):
        """Raise if the last peer gradient exchange failed (waits only for that exchange; the
        gradient post-processing above is already queued behind it)."""
        ev = getattr(self, "_peer_event", None)
        if ev is not None:
            self._peer_event = None
            ev.synchronize()
            self._peer.check()

    def test_loss(self, w: torch.Tensor, g: Optional[torch.Tensor] = None) -> float:
        t = torch.tensor([self.m.test_pure_loss_grad(w, g)], dtype=torch.float64)
        if self.comm is not None and self.comm.is_dist:
            self.comm.allreduce_(t)
            if g is not None:
                self._grad_allreduce(g)
                self._peer_landed()
        return float(t[0])

    def _grad_allreduce(self, g: torch.Tensor):
        """The dim-long gradient all-reduce (HoagOptimizer.java:1038, 68-628 MB for FM / FFM):
        the peer-memory two-shot exchange on one node (every xGMI link pulls its 1/P share, one
        kernel, fp32 sums in rank order), else the process group."""
        peer = getattr(self, "_peer", None)
        if peer is not None and peer.fits(g):
            peer.allreduce_(g)
            # a timed-out flag wait would leave g = stale peer sums (and every later exchange a
            # no-op): loss_and_grad checks the host-mapped error word once this exchange is done
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(g.device))
            self._peer_event = ev
        else:
            self.comm.allreduce_(g)

    # ------------------------------------------------------------------ line search
    def line_search(self, it: int, step: float, w, wprev, g, gprev, p) -> int:
        ls = self.ls
        prevloss, prevpure = self.loss_prev, self.pure_prev
        dginit = _dot(g, p)
        lsiter = 0
        while True:
            torch.add(wprev, p, alpha=step, out=w)
            for r, (s, e) in enumerate(self.groups):  # orthant projection
                if self.l1[r] > 0.0 and e > s:
                    wv, wp, gp = w[s:e], wprev[s:e], gprev[s:e]
                    kill = torch.where(wp != 0, wv * wp <= 0.0, wv * gp >= 0.0)
                    wv.masked_fill_(kill, 0.0)
            pure, loss = self.loss_and_grad(w, g)
            self.loss_prev, self.pure_prev = loss, pure
            self._verbose(it, f"----inner line search iter:{lsiter}, step:{jd(step)}, loss:{jd(loss)}, "
                              f"avg loss:{jd(loss / self.W)}, pure loss:{jd(pure)}")
            lsiter += 1
            dgtest = _dot(w - wprev, gprev)
            if loss > prevloss + ls.c1 * dgtest:
                factor = ls.step_decr
            else:
                if ls.mode == "sufficient_decrease":
                    return lsiter
                dg = _dot(p, g)
                if dg < ls.c2 * dginit:
                    factor = ls.step_incr
                else:
                    if ls.mode == "wolfe":
                        return lsiter
                    if dg > -ls.c2 * dginit:
                        factor = ls.step_decr
                    else:
                        return lsiter
            if step < ls.min_step:
                self.loss_prev, self.pure_prev = prevloss, prevpure
                self._info(it, f"----line search step is too small:{jd(step)}, optimizer will abort!")
                return -1
            if step > ls.max_step:
                self.loss_prev, self.pure_prev = prevloss, prevpure
                self._info(it, f"----line search step is too large:{jd(step)}, optimizer will abort!")
                return -2
            if ls.max_iter <= lsiter:
                self.loss_prev, self.pure_prev = prevloss, prevpure
                self._info(it, f"----line search iter >= max line search iter! step:{jd(step)}, "
                               "optimizer will abort!")
                return -3
            step *= factor

    # ------------------------------------------------------------------ history shards
    def setup_history(self, dim: int, dev) -> None:
        """Allocate the (s, y) history: this rank's slice [lo, hi) of every pair (the whole
        vector on one rank or with YTK_LBFGS_SHARD=0)."""
        m = self.ls.m
        P = self.comm.world if (self.comm is not None and self.comm.is_dist) else 1
        self.shard = P > 1 and os.environ.get("YTK_LBFGS_SHARD", "1") != "0"
        self.dim = dim
        if self.shard:
            seg = -(-dim // P)
            seg = -(-seg // 4) * 4  # whole 16-B units: equal all-gather segments
            r = self.comm.rank
            self.seg, self.lo, self.hi = seg, min(dim, r * seg), min(dim, (r + 1) * seg)
            self._gbuf = torch.zeros(P * seg, dtype=torch.float32, device=dev)  # all-gather buffer
            self.log.info(f"[lbfgs] (s, y) history sharded over {P} ranks: this rank keeps "
                          f"[{self.lo}, {self.hi}) of {dim}")
        else:
            self.seg, self.lo, self.hi = dim, 0, dim
            self._gbuf = None
        n = self.hi - self.lo
        self.S = torch.zeros((m, n), dtype=torch.float32, device=dev)
        self.Y = torch.zeros((m, n), dtype=torch.float32, device=dev)
        self.YS = [1.0] * m

    def _gsum(self, vals: List[float]) -> List[float]:
        """Sum per-rank fp64 partials of the sharded history over the ranks (one collective;
        the peer-memory exchange when the job has one); identity when not sharded."""
        if not getattr(self, "shard", False):
            return vals
        peer = getattr(self, "_peer", None)
        if peer is not None:
            t = torch.tensor(vals, dtype=torch.float64, device=self.S.device)
            peer.allreduce_(t)
            out = t.tolist()  # synchronises: the exchange has landed
            peer.check()
            return out
        return self.comm.allreduce_scalars(vals)

    def _gather_p(self, p: torch.Tensor):
        """p's slices [lo, hi) from every rank -> the whole p on every rank (one all-gather)."""
        P, r, seg = self.comm.world, self.comm.rank, self.seg
        buf = self._gbuf
        mine = buf[r * seg:(r + 1) * seg]
        n = self.hi - self.lo
        if n:
            mine[:n].copy_(p[self.lo:self.hi])
        peer = getattr(self, "_peer", None)
        if peer is not None and peer.fits_segments(buf):
            peer.allgather_(buf)
            p.copy_(buf[:self.dim])
            torch.cuda.current_stream(p.device).synchronize()
            peer.check()
        else:
            allp = self.comm.allgather(mine)
            p.copy_(allp[:self.dim])

    # ------------------------------------------------------------------ two loop
    def hv(self, p: torch.Tensor, cursor: int, loops: int, ys: float, yy: float):
        """p <- H p with the last ``loops`` pairs ending before ``cursor`` (Hv, :904-929)."""
        m = self.ls.m
        if getattr(self, "shard", False):
            self._hv_sharded(p, cursor, loops, ys, yy)
            return
        if loops > 0 and self._fused_two_loop(p):
            self._hv_fused(p, cursor, loops, ys, yy)
            return
        alphas = [0.0] * m
        c = cursor
        for _ in range(loops):
            c = (c + m - 1) % m
            a = _dot(self.S[c], p) / self.YS[c]
            alphas[c] = a
            p.add_(self.Y[c], alpha=-a)
        p.mul_(ys / yy)
        for _ in range(loops):
            b = _dot(self.Y[c], p) / self.YS[c]
            p.add_(self.S[c], alpha=alphas[c] - b)
            c = (c + 1) % m

    def _fused_two_loop(self, p: torch.Tensor) -> bool:
        # YTK_FUSED_TWO_LOOP=0: the unfused dot / axpy sequence
        return (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                and os.environ.get("YTK_FUSED_TWO_LOOP", "1") != "0")

    def _hv_fused(self, p: torch.Tensor, cursor: int, loops: int, ys: float, yy: float):
        """hv with every update fused with the next dot product (blas.axpy_dot): the same
        recursion, one pass over (p, update vector, next dot operand) per step."""
        m = self.ls.m
        alphas = [0.0] * m
        c = (cursor + m - 1) % m
        a = _dot(self.S[c], p) / self.YS[c]
        for k in range(loops):
            alphas[c] = a
            if k + 1 < loops:  # p -= a Y[c]; next: S[c - 1] . p
                nc = (c + m - 1) % m
                a = blas.axpy_dot(p, self.Y[c], -a, 1.0, self.S[nc]) / self.YS[nc]
                c = nc
            else:  # p = (p - a Y[c]) * ys / yy; the second loop starts at this c: Y[c] . p
                b = blas.axpy_dot(p, self.Y[c], -a, ys / yy, self.Y[c]) / self.YS[c]
        for k in range(loops):
            if k + 1 < loops:  # p += (alpha - b) S[c]; next: Y[c + 1] . p
                nc = (c + 1) % m
                b_next = blas.axpy_dot(p, self.S[c], alphas[c] - b, 1.0, self.Y[nc]) / self.YS[nc]
                c, b = nc, b_next
            else:
                p.add_(self.S[c], alpha=alphas[c] - b)

    def _hv_sharded(self, p: torch.Tensor, cursor: int, loops: int, ys: float, yy: float):
        """hv over this rank's history slice: every dot product is a local partial summed over
        the ranks (_gsum), every update touches only p[lo:hi]; one all-gather of p at the end.
        The update + next dot of a step are one pass (blas.axpy_dot) on the GPU."""
        m = self.ls.m
        pl = p[self.lo:self.hi]
        fused = self._fused_two_loop(p) and pl.numel() > 0

        def step(x, alpha, scale, d):  # pl <- (pl + alpha x) * scale; local d . pl
            if fused:
                return blas.axpy_dot(pl, x, alpha, scale, d)
            pl.add_(x, alpha=alpha)
            if scale != 1.0:
                pl.mul_(scale)
            return _dot(d, pl)

        if loops <= 0:
            p.mul_(ys / yy)
            return
        alphas = [0.0] * m
        c = (cursor + m - 1) % m
        a = self._gsum([_dot(self.S[c], pl)])[0] / self.YS[c]
        b = 0.0
        for k in range(loops):
            alphas[c] = a
            if k + 1 < loops:  # pl -= a Y[c]; next: S[c - 1] . p
                nc = (c + m - 1) % m
                a = self._gsum([step(self.Y[c], -a, 1.0, self.S[nc])])[0] / self.YS[nc]
                c = nc
            else:  # pl = (pl - a Y[c]) * ys / yy; the second loop starts at this c: Y[c] . p
                b = self._gsum([step(self.Y[c], -a, ys / yy, self.Y[c])])[0] / self.YS[c]
        for k in range(loops):
            if k + 1 < loops:  # pl += (alpha - b) S[c]; next: Y[c + 1] . p
                nc = (c + 1) % m
                b_next = self._gsum([step(self.S[c], alphas[c] - b, 1.0, self.Y[nc])])[0] / self.YS[nc]
                c, b = nc, b_next
            else:
                pl.add_(self.S[c], alpha=alphas[c] - b)
        self._gather_p(p)

    # ------------------------------------------------------------------ grid setup
    def _grid_points(self):
        hp = self.hp
        axes = []
        for arr, key in ((hp.grid_l1, "l1"), (hp.grid_l2, "l2")):
            for i, (a, b, n) in enumerate(arr):
                need = not (a <= 0.0 or b <= 0.0)
                num = int(n) + 1 if need else 1
                stepv = (b - a) / n if n else 0.0
                vals = [a + s * stepv if need else 0.0 for s in range(num)]
                self.log.info(f"{key}[{i}] search range: {vals}")
                axes.append(vals)
        combos = [[v] for v in axes[0]]
        for ax in axes[1:]:
            combos = [c + [v] for v in ax for c in combos]
        nl1 = len(hp.grid_l1)
        return [(c[:nl1], c[nl1:]) for c in combos]

    # ------------------------------------------------------------------ main loop
    def run(self, w: torch.Tensor) -> LbfgsResult:
        self._peer = None
        if self.comm is not None and self.comm.is_dist and w.is_cuda:
            from ..parallel import peer as peer_mod
            P = self.comm.world
            gather = P * (-(-(-(-w.numel() // P)) // 4) * 4)  # the sharded p all-gather buffer
            self._peer = peer_mod.make(self.comm, -(-max(w.numel(), gather) * 4 // 8))
        res = self._run(w)
        if self._peer is not None:  # collective: every rank leaves run() together
            self._peer.close()
            self._peer = None
        return res

    def _run(self, w: torch.Tensor) -> LbfgsResult:
        ls, m = self.ls, self.ls.m
        dev, dim = w.device, w.numel()
        start = time.perf_counter()
        has_test = self.m.has_test()
        best_test = float("inf")
        best_w = None
        best_l1, best_l2 = list(self.l1), list(self.l2)
        init_w = w.clone() if (self.need_hyper and self.hp.restart) else None
        grid = self._grid_points() if self.grid else None
        hoag_steps = [self.hp.init_step] * len(self.l2)
        hoag_grads: List[List[float]] = []
        hoag_deltas: List[float] = []
        t_old = 0.0
        g = torch.zeros(dim, dtype=torch.float32, device=dev)
        wprev, gprev = torch.empty_like(w), torch.empty_like(w)
        p = torch.empty_like(w)
        self.setup_history(dim, dev)
        lo, hi = self.lo, self.hi
        test_loss = None
        status, it, cursor = 0, 1, 0
        ys = yy = 1.0
        elapse = lambda: f"{jd((time.perf_counter() - start))} sec elapse\n"
        while True:
            it = 1
            if grid is not None:
                self.l1, self.l2 = list(grid[self.hyper_idx - 1][0]), list(grid[self.hyper_idx - 1][1])
            if self.need_hyper:
                self._info(it, f"hyper search new l1:{self.l1}, new l2:{self.l2}")
                if init_w is not None:
                    w.copy_(init_w)
            pure, loss = self.loss_and_grad(w, g)
            self.loss_prev, self.pure_prev = loss, pure
            msg = elapse() + f"train loss = {jd(pure / self.W)}\ntrain regularized loss = {jd(loss / self.W)}\n"
            msg += self.m.other_train_info() + self.m.train_eval()
            if has_test:
                test_loss = self.test_loss(w)
                if self.need_hyper and test_loss < best_test:
                    best_test, best_w = test_loss, w.clone()
                    best_l1, best_l2 = list(self.l1), list(self.l2)
                msg += f"test loss = {jd(test_loss / self.Wt)}\n" + self.m.other_test_info() + self.m.test_eval()
            self._info(0, msg)
            if self.just_evaluate:
                return LbfgsResult(loss, pure, 0, 0, test_loss, self.l1, self.l2)
            torch.neg(g, out=p)
            wnorm, gnorm = max(_norm(w), 1.0), _norm(g)
            if (not self.need_hyper or it >= 2 * m) and gnorm / wnorm <= ls.eps:
                self._info(0, "gnorm / wnorm <= lbfgsParams.convergence.eps, initial w meets converge condition, "
                              f"you can decrease eps to get more accurate result!gnorm:{jd(gnorm)}, "
                              f"wnorm:{jd(wnorm)}, eps:{jd(ls.eps)}")
                self._final_report(start, test_loss)
                return LbfgsResult(loss, pure, 1, 0, test_loss, self.l1, self.l2)
            step = 1.0 / gnorm if gnorm > 0 else 1.0
            cursor = 0
            while True:
                fault_point("lbfgs", it, getattr(self.comm, "rank", 0))
                self.timer.begin()
                wprev.copy_(w)
                gprev.copy_(g)
                self._verbose(it, "begin line search...")
                cnt = self.line_search(it, step, w, wprev, g, gprev, p)
                self.timer.mark("line_search_loss_grad")
                if cnt < 0:
                    self._verbose(it, "line search failed, move to prev point!")
                    w.copy_(wprev)
                    g.copy_(gprev)
                    status = 2
                    break
                msg = elapse() + (f"train loss = {jd(self.pure_prev / self.W)}\n"
                                  f"train regularized loss = {jd(self.loss_prev / self.W)}\n")
                msg += self.m.other_train_info() + self.m.train_eval()
                if has_test:
                    test_loss = self.test_loss(w)
                    if self.need_hyper and test_loss < best_test:
                        best_test, best_w = test_loss, w.clone()
                        best_l1, best_l2 = list(self.l1), list(self.l2)
                    msg += f"test loss = {jd(test_loss / self.Wt)}\n" + self.m.other_test_info() + \
                        self.m.test_eval()
                    self.timer.mark("test_eval")
                self._metric(it, start, test_loss)
                self._info(it, msg)
                wnorm, gnorm = _norm(w), _norm(g)
                wnorm = max(wnorm, 1.0)
                if (not self.need_hyper or it >= 2 * m) and gnorm / wnorm <= ls.eps:
                    self._info(it, f"gnorm / wnorm <= lbfgsParams.convergence.eps, converged!gnorm:{jd(gnorm)}, "
                                   f"wnorm:{jd(wnorm)}, eps:{jd(ls.eps)},  you can decrease eps to get more "
                                   "accurate result!")
                    status = 3
                    break
                if it >= ls.lbfgs_max_iter:
                    self._info(it, "max iter,  you can increase max iter to get more accurate result!")
                    status = 4
                    break
                if self.dump_freq > 0 and it % self.dump_freq == 0:
                    self._dump(w)
                torch.sub(w[lo:hi], wprev[lo:hi], out=self.S[cursor])
                torch.sub(g[lo:hi], gprev[lo:hi], out=self.Y[cursor])
                ys, yy = self._gsum([_dot(self.Y[cursor], self.S[cursor]), _dot(self.Y[cursor], self.Y[cursor])])
                if ys < 1.0e-60:
                    self._info(it, f"ys:{jd(ys)} is too small or is negtive(you may change to wolfe condition!), "
                                   "set to 0.01*yy!")
                    ys = yy * 0.01
                self.YS[cursor] = ys
                loops = min(m, it)
                cursor = (cursor + 1) % m
                torch.neg(g, out=p)
                self.hv(p, cursor, loops, ys, yy)
                for r, (s, e) in enumerate(self.groups):  # constrain the direction (l1)
                    if self.l1[r] > 0.0 and e > s:
                        p[s:e].masked_fill_(p[s:e] * g[s:e] >= 0.0, 0.0)
                self.timer.mark("two_loop")
                per = self.timer.end()
                if per:
                    self._info(it, f"time stats: {PhaseTimer.fmt(per)}")
                step = 1.0
                it += 1
            self._verbose(it, f"status:{status}")
            if not self.need_hyper:
                break
            self._info(it, f"[hyper search] until now, best test loss:{jd(best_test)}, best avg test loss:"
                           f"{jd(best_test / self.Wt)}, best l1:{best_l1}, best l2:{best_l2}")
            self._dump(w)
            if self.hoag:
                done, t_old = self._hoag_step(w, cursor, it, ys, yy, hoag_steps, hoag_grads, hoag_deltas, t_old)
                if done or self.hyper_idx >= self.hp.outer_iter:
                    break
            else:
                if self.hyper_idx >= len(grid):
                    break
            self.hyper_idx += 1
        if self.need_hyper and best_w is not None:
            w.copy_(best_w)
            self.l1, self.l2 = best_l1, best_l2
            test_loss = self.test_loss(w)
            pure, loss = self.loss_and_grad(w, g)
            self.loss_prev, self.pure_prev = loss, pure
        self._dump(w)
        self._final_report(start, test_loss, it)
        if self.timer.enabled:
            self._info(it, self.timer.report())
        return LbfgsResult(self.loss_prev, self.pure_prev, status, it, test_loss, self.l1, self.l2)

    def _final_report(self, start, test_loss, it=0):
        msg = (f"{jd(time.perf_counter() - start)} sec elapse\nfinal train loss = {jd(self.pure_prev / self.W)}\n"
               f"final train regularized loss = {jd(self.loss_prev / self.W)}\n")
        msg += self.m.other_train_info() + self.m.train_eval()
        if test_loss is not None and self.m.has_test():
            msg += f"final test loss = {jd(test_loss / self.Wt)}\n" + self.m.other_test_info() + self.m.test_eval()
        self._info(0, msg)

    def _dump(self, w):
        prec = self.m.precision(w, self.l2, self.W)
        if prec is not None and self.comm is not None and self.comm.is_dist:
            self.comm.allreduce_(prec)
        if prec is not None:
            # + l2 * W on regularized coordinates (LinearHoagOptimizer.calPrecision)
            for r, (s, e) in enumerate(self.groups):
                if self.l2[r] > 0.0 and e > s:
                    prec[s:e] += self.l2[r] * self.W
        self.m.dump(w, prec)  # every rank writes its own index range (model-%05d)

    def _hoag_step(self, w, cursor, k, ys, yy, steps, grads_hist, deltas, t_old):
        """One HOAG outer step (hyperHoagOptimization, :813-902). Returns (stop, new t_old)."""
        gtest = torch.zeros_like(w)
        tl = self.test_loss(w, gtest)
        gtest.mul_(1.0 / self.Wt)
        loops = min(self.ls.m, k)
        self.hv(gtest, cursor, loops, ys, yy)
        grads = [0.0] * len(self.l2)
        for r, (s, e) in enumerate(self.groups):
            if self.l2[r] > 0.0 and e > s:
                grads[r] = -self.l2[r] * self.W * _dot(w[s:e], gtest[s:e])
        grads_hist.append(grads)
        deltas.append((tl - t_old) / self.Wt)
        t_old = tl
        if len(grads_hist) >= 2:
            for r in range(len(self.l2)):
                if self.l2[r] > 0.0 and grads_hist[-2][r] * grads_hist[-1][r] < 0.0:
                    steps[r] *= self.hp.step_decr_factor
        if len(deltas) >= 3:
            avg = sum(abs(d) for d in deltas[-3:]) / 3
            if avg < self.hp.test_loss_reduce_limit:
                self._info(self.hyper_idx, f"[hoag] last 3 avg test reduce loss:{jd(avg)} < "
                                           f"{jd(self.hp.test_loss_reduce_limit)}, exit! final l2:{self.l2}")
                return True, t_old
        for r in range(len(self.l2)):
            if self.l2[r] > 0.0:
                lg = math.log(self.l2[r])
                lg = lg + steps[r] if -grads[r] >= 0 else lg - steps[r]
                self.l2[r] = math.exp(lg)
        self._info(self.hyper_idx, f"[hoag] l1:{self.l1}, new l2:{self.l2}")
        return False, t_old
