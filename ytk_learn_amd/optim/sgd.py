"""Mini-batch Hogwild!-style SGD for the linear, FM and FFM models.

An extension (``optimization.optimizer = "sgd"``): ytk-learn trains these models only
with full-batch L-BFGS (``J/param/CommonParams.java:55-60``), which stays the default.
SGD trades the L-BFGS convergence guarantees for cheap passes over data sets too large
to iterate many times.

Per mini-batch of rows (a contiguous row range of the rank's CSR shard, visited in a
seeded random order every epoch):
  1. forward on the batch rows (the training kernels read the CSR slice in place:
     ``fm_forward`` -- with k = 0 for the linear part -- and the FFM pair kernel);
  2. c_r = weight_r * dloss/dz (any loss of the framework, on the device);
  3. lock-free update: ``fm_sgd_update`` (csrc/hip/fm.hip) for the linear weights and
     FM latents, the FFM pair kernel with coefficient -lr * c_r written straight into V.
     Concurrent rows sharing a feature race exactly as in Hogwild! (Niu et al., 2011).
Regularization: l2 of the linear / latent groups is applied to the weights a sample
touches (sparse weight decay); l1 is not supported by this optimizer. FFM latents get no
decay (the pair kernel has none).
Step size (``optimization.sgd.average``): with ``feature`` (default) a weight's step is
the MEAN of the per-sample steps of the batch rows containing its feature (rows per
feature counted on the device before the update) -- rare features keep the per-sample
rate, hot ones (the bias is in every row) take one bounded step per batch. ``none`` applies
the sum, which for batches of thousands of rows diverges on hot features.

Multi-GPU: every rank runs SGD on its shard; weights are averaged across ranks with one
RCCL all-reduce every ``sync_every`` batches (0 = once per epoch) -- local SGD / model
averaging, so the per-step cost stays free of communication.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import List

import numpy as np
import torch

from ..ops.ffm import ffm_backward, ffm_forward
from ..ops.fm import fm_forward, fm_sgd_update, sgd_count
from ..utils.fault import fault_point
from ..utils.javafmt import java_double_str as jd

SUPPORTED = ("linear", "fm", "ffm")


@dataclass
class SGDParams:
    learning_rate: float = 0.05
    learning_rate_decay: float = 1.0  # multiplied into the rate after every epoch
    batch_size: int = 65536
    epochs: int = 10
    sync_every: int = 0               # batches between cross-rank weight averaging; 0 = per epoch
    seed: int = 1
    dtype: str = "fp32"               # "bf16": FM latents read from a bf16 working copy (fp32 master)
    average: str = "feature"          # "feature": a weight's step is the mean over the batch rows
    #                                   containing its feature; "none": the sum (per-sample steps)

    @classmethod
    def from_config(cls, c, prefix: str = "optimization.sgd.") -> "SGDParams":
        from ..config.params import check
        p = cls(learning_rate=c.get_double(prefix + "learning_rate", 0.05),
                learning_rate_decay=c.get_double(prefix + "learning_rate_decay", 1.0),
                batch_size=c.get_int(prefix + "batch_size", 65536), epochs=c.get_int(prefix + "epochs", 10),
                sync_every=c.get_int(prefix + "sync_every", 0), seed=c.get_int(prefix + "seed", 1),
                dtype=str(c.get_string(prefix + "dtype", "fp32")).lower(),
                average=str(c.get_string(prefix + "average", "feature")).lower())
        check(p.dtype in ("fp32", "bf16"), "%sdtype:%s must be fp32 or bf16", prefix, p.dtype)
        check(p.average in ("feature", "none"), "%saverage:%s must be feature or none", prefix, p.average)
        check(p.learning_rate > 0, "%slearning_rate:%f must > 0", prefix, p.learning_rate)
        check(0 < p.learning_rate_decay <= 1.0, "%slearning_rate_decay:%f must be in (0, 1]", prefix,
              p.learning_rate_decay)
        check(p.batch_size >= 1, "%sbatch_size:%d must >= 1", prefix, p.batch_size)
        check(p.epochs >= 1, "%sepochs:%d must >= 1", prefix, p.epochs)
        return p


class _Slice:
    """Row range [b, e) of a CSR matrix viewed in place (absolute offsets into the arrays)."""

    def __init__(self, X, b: int, e: int):
        self.indptr = X.indptr[b:e + 1]
        self.indices, self.values = X.indices, X.values
        self.n = e - b
        self.device = X.device


class SGDOptimizer:
    def __init__(self, model, sp: SGDParams, l1: List[float], l2: List[float], comm, log, W: float, Wt: float,
                 dump_freq: int = -1):
        if model.name not in SUPPORTED:
            from ..utils.errors import YtkLearnError
            raise YtkLearnError(f"optimization.optimizer = sgd supports {list(SUPPORTED)}, not {model.name}")
        if any(v > 0 for v in l1):
            log.info("[sgd] l1 regularization is ignored by the sgd optimizer")
        self.m, self.sp, self.comm, self.log = model, sp, comm, log
        self.W, self.Wt = W, Wt
        self.l2w = float(l2[0]) if len(l2) > 0 else 0.0
        self.l2v = float(l2[1]) if len(l2) > 1 else 0.0
        self.dump_freq = dump_freq
        self.dist = comm is not None and comm.is_dist
        # bf16 storage (BASELINE config 4, "FM k=16 ... bf16 SGD"): the FM latent matrix is
        # gathered from a bf16 working copy by the forward and gradient passes (half the
        # bytes of the dominant V-row gathers); updates land in the fp32 master, whose
        # touched entries re-round the copy; full re-sync after every weight averaging.
        # per-feature averaging (average = feature): rows per feature of the current batch,
        # counted before the update and cleared after it (zero between batches)
        self.cnt = (torch.zeros(model.F, dtype=torch.int32, device=model.w.device)
                    if sp.average == "feature" else None)
        self.Vb = None
        if sp.dtype == "bf16" and model.name == "fm" and getattr(model, "kk", 0) > 0:
            self.Vb = torch.empty((model.F, model.kk), dtype=torch.bfloat16, device=model.w.device)

    # ------------------------------------------------------------------ one batch
    def _step(self, w: torch.Tensor, b: int, e: int, lr: float):
        m = self.m
        d = m.data.train
        X = m.X
        F = m.F
        reg_skip = 0 if m.p.model.need_bias else -1
        upd_w = getattr(m, "need_first", True)
        sl = _Slice(X, b, e)
        w_lin = w[:F]
        # nnz range of the batch: only the CPU paths need it on the host (a device read
        # would synchronise every batch)
        o0, o1 = (int(X.indptr[b]), int(X.indptr[e])) if not w.is_cuda else (None, None)
        S = None
        if w.is_cuda and (m.name != "fm" or m.kk <= 64):
            # fused row pass (k = 0: linear score only): fx and S = X V of the batch
            kk = m.kk if m.name == "fm" else 0
            Vf = (self.Vb if self.Vb is not None else w[F:].view(F, kk)) if kk > 0 else w_lin.new_zeros((F, 0))
            fx, S = fm_forward(sl, w_lin, Vf)
            if kk == 0:
                S = None
        else:
            rows = X.rows_of_nnz[o0:o1] - b
            lin = w_lin[X.indices[o0:o1].long()] * X.values[o0:o1]
            fx = torch.zeros(e - b, dtype=torch.float64, device=w.device).index_add_(0, rows, lin.double())
            if m.name == "fm" and m.kk > 0:  # CPU: S = X V and the square term from index ops
                V = self.Vb.float() if self.Vb is not None else w[F:].view(F, m.kk)
                vx = V[X.indices[o0:o1].long()] * X.values[o0:o1, None]
                S = torch.zeros((e - b, m.kk), dtype=torch.float32).index_add_(0, rows, vx)
                Q = torch.zeros((e - b, m.kk), dtype=torch.float32).index_add_(0, rows, vx * vx)
                fx = fx + 0.5 * (S.double() ** 2 - Q.double()).sum(1)
        if m.name == "ffm" and m.stride > 0:
            fld = d.fields
            ip = sl.indptr if w.is_cuda else sl.indptr - o0
            idx = X.indices if w.is_cuda else X.indices[o0:o1]
            val = X.values if w.is_cuda else X.values[o0:o1]
            fl = fld if w.is_cuda else fld[o0:o1]
            fx = fx + ffm_forward(ip, idx, val, fl, w[F:], m.nf, m.kk, skip_feat=m._skip).double()
        y = d.y[b:e, 0].double()
        c = (d.weight[b:e].double() * m.loss.grad(fx, y)).float().contiguous()
        V = w[F:].view(F, m.kk) if (m.name == "fm" and m.kk > 0) else None
        cnt = self.cnt
        if cnt is not None:
            sgd_count(sl.indptr, X.indices, cnt, nnz_hint=(e - b) * max(1, X.nnz // max(1, X.n)))
        fm_sgd_update(sl.indptr, X.indices, X.values, w_lin, V, S, c, lr, self.l2w, self.l2v, reg_skip, upd_w,
                      bool(getattr(m, "bias_latent", False)), Vb=self.Vb, cnt=cnt)
        if m.name == "ffm" and m.stride > 0 and getattr(m, "need_second", True):
            ffm_backward(ip, idx, val, fl, w[F:], m.nf, m.kk, (-lr * c).contiguous(), w[F:], skip_feat=m._skip,
                         cnt=cnt)
        if cnt is not None:
            sgd_count(sl.indptr, X.indices, cnt, clear=True, nnz_hint=(e - b) * max(1, X.nnz // max(1, X.n)))

    def _average(self, w):
        if self.dist:
            self.comm.allreduce_(w)
            w.mul_(1.0 / self.comm.world)
        self._sync_copy(w)

    def _sync_copy(self, w):
        if self.Vb is not None:
            self.Vb.copy_(w[self.m.F:].view(self.m.F, self.m.kk))

    def _losses(self, w):
        t = torch.tensor([self.m.pure_loss_grad(w, None), self.m.test_pure_loss_grad(w, None)
                          if self.m.has_test() else 0.0], dtype=torch.float64)
        if self.dist:
            self.comm.allreduce_(t)
        return float(t[0]), float(t[1])

    def _info(self, it: int, msg: str):
        self.log.info(f"[model={self.m.name}] [loss={self.m.loss_name}] [iter={it}] " + msg)

    # ------------------------------------------------------------------ driver
    def run(self, w: torch.Tensor):
        sp = self.sp
        n = self.m.data.train.n
        bounds = [(b, min(b + sp.batch_size, n)) for b in range(0, n, sp.batch_size)]
        nb = len(bounds)
        nb_all = nb
        if self.dist:  # every rank runs the same number of steps (the sync points must match)
            nb_all = int(self.comm.allreduce_scalars([nb], op="max", dtype=torch.int64)[0])
        rng = np.random.default_rng(sp.seed + (self.comm.rank if self.comm is not None else 0))
        lr = sp.learning_rate
        self._sync_copy(w)
        start = time.perf_counter()
        train_loss = test_loss = float("nan")
        rank = self.comm.rank if self.comm is not None else 0
        for epoch in range(1, sp.epochs + 1):
            fault_point("sgd", epoch - 1, rank)
            order = rng.permutation(nb) if nb else np.zeros(0, np.int64)
            for step in range(nb_all):
                if step < nb:
                    b, e = bounds[int(order[step])]
                    self._step(w, b, e, lr)
                if self.dist and sp.sync_every > 0 and (step + 1) % sp.sync_every == 0:
                    self._average(w)
            if self.dist and (sp.sync_every <= 0 or nb_all % sp.sync_every != 0):
                self._average(w)
            pure, tl = self._losses(w)
            train_loss = pure / max(self.W, 1e-300)
            msg = (f"{jd(time.perf_counter() - start)} sec elapse\nlearning rate = {jd(lr)}\n"
                   f"train loss = {jd(train_loss)}\n" + self.m.train_eval())
            if self.m.has_test():
                test_loss = tl / max(self.Wt, 1e-300)
                msg += f"test loss = {jd(test_loss)}\n" + self.m.test_eval()
            self._info(epoch, msg)
            metric = getattr(self.log, "metric", None)
            if metric is not None:
                metric(model=self.m.name, loss=self.m.loss_name, iter=epoch, train_loss=train_loss,
                       test_loss=test_loss if self.m.has_test() else None, elapsed=time.perf_counter() - start)
            if self.dump_freq > 0 and epoch % self.dump_freq == 0:
                self.m.dump(w, None)
            lr *= sp.learning_rate_decay
        self.m.dump(w, None)
        self._info(0, f"{jd(time.perf_counter() - start)} sec elapse\nfinal train loss = {jd(train_loss)}\n"
                   + (f"final test loss = {jd(test_loss)}\n" if self.m.has_test() else ""))
        return train_loss, test_loss
