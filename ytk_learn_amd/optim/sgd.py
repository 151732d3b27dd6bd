"""Mini-batch SGD for the linear, FM and FFM models.

An extension (``optimization.optimizer = "sgd"``): ytk-learn trains these models only
with full-batch L-BFGS (``J/param/CommonParams.java:55-60``), which stays the default.
SGD trades the L-BFGS convergence guarantees for cheap passes over data sets too large
to iterate many times.

Batches are fixed contiguous row ranges of the rank's CSR shard, visited in a seeded random
order every epoch. On the GPU each batch's column order is built once at set-up
(:mod:`ytk_learn_amd.ops.sgd`) and a step is four kernels: the row pass (``fm_forward``;
FFM: + the pair forward), the fused row-loss pass (c_r = weight_r * dloss/dz), the
column pass over the batch CSC (FFM: + the streamed pair gradient) and ``sgd_apply``, where
every touched feature sums its chunk partials in order and updates its weights ONCE -- a
deterministic synchronous mini-batch step with no float atomics (round 4 ran per-entry
Hogwild! atomics: 42M per 65536-row FM batch, 409M for FFM). The CPU path applies the same
synchronous step with index ops (``fm_sgd_update`` / ``ffm_step_cpu``).
Regularization: l2 of the linear / latent groups (FFM latents too) is applied to the weights
a batch touches, once per batch entry holding the feature (sparse weight decay); l1 is not
supported by this optimizer.
Step size (``optimization.sgd.average``): with ``feature`` (default since round 4) a
weight's step is the MEAN of the per-sample steps of the batch entries holding its feature
(the batch CSC's column length) -- rare features keep the per-sample rate, hot ones (the bias
is in every row) take one bounded step per batch. ``none`` applies the sum, which for batches
of thousands of rows diverges on hot features. FFM: the count of V[i, f] is the entries of
feature i in the batch (not only those whose row also holds a field-f feature), so for rows
without every field such latents take a smaller step than a per-(feature, field) mean.
``optimization.sgd.dtype = bf16``: FM -- the row pass gathers the latents from a bf16 working
copy (half the bytes of its dominant V-row gathers); the fp32 master takes the updates and
``sgd_apply`` re-rounds the copy of every touched row. FFM (pair-term path: k = 4, fixed-layout
rows of <= 64 entries) -- the LDS-staged pair forward stages each row's latent rows from the
bf16 copy (half the bytes of its whole-row reads) and writes the pair terms E as bf16 (half the
bytes the chunk sums read back); dot products, sums and the fp32 master stay fp32, and both
update kernels re-round the copy of every slot they change.

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

from ..ops import sgd as sgd_ops
from ..ops.blas import row_loss
from ..ops.ffm import ffm_forward
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
    dtype: str = "fp32"               # "bf16": latents read from a bf16 working copy (fp32 master);
    #                                   FFM: the pair terms are bf16 too
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
        dev = model.w.device
        F = model.F
        self.kk = model.kk if model.name == "fm" else 0
        if dev.type == "cuda" and self.kk > 64:
            from ..utils.errors import YtkLearnError
            raise YtkLearnError("optimization.optimizer = sgd on the GPU supports fm k <= 64")
        # CPU: rows per feature of the current batch (count, step, clear); GPU: the batch CSC
        self.cnt = (torch.zeros(F, dtype=torch.int32, device=dev)
                    if sp.average == "feature" and dev.type != "cuda" else None)
        self.Vb = None
        if sp.dtype == "bf16" and model.name == "fm" and self.kk > 0:
            self.Vb = torch.empty((F, self.kk), dtype=torch.bfloat16, device=dev)
        if sp.dtype == "bf16" and model.name == "ffm" and dev.type != "cuda":
            # the CPU step's bf16 emulation of the GPU pair-term path (GPU: allocated by _setup)
            self.Vb = torch.empty((F, model.nf * model.kk), dtype=torch.bfloat16, device=dev)
        # FFM on the GPU: fixed-layout batches read the model's V directly (ffm_sgd_grad_kernel);
        # the general pair-gradient kernel reads a field-major copy ([nfield][F][k]) that
        # sgd_apply keeps current -- allocated only when some batch needs it (_setup)
        self.ffm = model.name == "ffm" and getattr(model, "stride", 0) > 0
        self.Vt = None
        self.E = None  # FFM pair terms written by the forward (ops/sgd.pair_terms_elems)
        self._batches = None

    # ------------------------------------------------------------------ one batch
    def _setup(self, bounds):
        m = self.m
        X = m.X
        if self._batches is None and X.device.type == "cuda":
            fld = m.data.train.fields if self.ffm else None
            self._batches = sgd_ops.build_batches(X, bounds, fld, m.nf if self.ffm else 0, getattr(m, "_skip", -1))
            bf = self.ffm and self.sp.dtype == "bf16"
            ne = sgd_ops.pair_terms_elems(self._batches, m.w[m.F:], m.kk, 2 if bf else 4) if self.ffm else 0
            if bf:
                from ..ops.ffm import lds_forward_ok
                mm = self._batches[0].lay[1] if (ne and self._batches[0].lay is not None) else 0
                if ne and lds_forward_ok(mm, m.nf, m.kk, m.w[m.F:]) and mm % 2 == 0 and m.nf % 2 == 0:
                    self.Vb = m.w[m.F:].view(m.F, -1).to(torch.bfloat16)  # run() re-syncs it from w
                else:
                    self.log.info("[sgd] dtype = bf16 needs the ffm pair-term path (k = 4, fixed-layout rows of "
                                  "<= 64 entries, even row length and field count): running fp32")
            if ne:
                self.E = torch.empty(ne, dtype=torch.bfloat16 if self.Vb is not None else torch.float32,
                                     device=X.device)
                for bt in self._batches:
                    sgd_ops.prepare_pair_terms(bt)
            else:
                for bt in self._batches:
                    bt.perm = None
            if self.ffm and sgd_ops.needs_transposed(self._batches, self.m.w[m.F:], m.kk):
                self.Vt = torch.empty((m.nf, m.F, m.kk), dtype=torch.float32, device=X.device)
                self._sync_copy(self.m.w)
        return self._batches

    def _step(self, w: torch.Tensor, b: int, e: int, lr: float, bt=None):
        if bt is not None:
            return self._step_gpu(w, bt, lr)
        return self._step_cpu(w, b, e, lr)

    def _coef(self, fx, y, wt, z1=None):
        fused = row_loss(self.m.loss, fx, y, wt, z1=z1, want_grad=True, want_loss=False)
        if fused is not None:
            return fused[2]
        z = fx.double() + (z1.double() if z1 is not None else 0.0)
        return (wt.double() * self.m.loss.grad(z, y.double())).float().contiguous()

    def _step_gpu(self, w: torch.Tensor, bt, lr: float):
        """Row pass -> c -> column pass -> one update per touched weight (ops/sgd.py)."""
        m, sp = self.m, self.sp
        d = m.data.train
        X, F = m.X, m.F
        b, e = bt.b, bt.e
        sl = _Slice(X, b, e)
        w_lin = w[:F]
        kk = self.kk
        reg_skip = 0 if m.p.model.need_bias else -1
        upd_w = getattr(m, "need_first", True)
        Vf = (self.Vb if self.Vb is not None else w[F:].view(F, kk)) if kk > 0 else w_lin.new_zeros((F, 0))
        fx, S = fm_forward(sl, w_lin, Vf)
        z1 = None
        use_e = self.E is not None and getattr(m, "need_second", True)
        if use_e:
            z1 = sgd_ops.ffm_forward_e(bt, sl.indptr, X.indices, X.values, d.fields, w[F:], m.nf, m._skip, self.E,
                                       Vb=self.Vb)
        elif self.ffm:
            z1 = ffm_forward(sl.indptr, X.indices, X.values, d.fields, w[F:], m.nf, m.kk, skip_feat=m._skip)
        c = self._coef(fx, d.y[b:e, 0], d.weight[b:e], z1)
        avg = sp.average == "feature"
        bias_latent = bool(getattr(m, "bias_latent", False))
        if use_e:  # single-chunk columns step inside ffm_sgd_ecol_kernel, the rest in sgd_apply
            lin, lat = sgd_ops.ffm_step_e(bt, c, self.E, w_lin, w[F:], m.nf, m.kk, lr, self.l2w, self.l2v, reg_skip,
                                          upd_w, bias_latent, avg, Vb=self.Vb)
            sgd_ops.apply_step(bt, lin, lat, m.stride, w_lin, w[F:], m.kk, lr, self.l2w, self.l2v, reg_skip, upd_w,
                               bias_latent, avg, Vb=self.Vb, multi=True)
            return
        part = sgd_ops.column_sums(bt, c, S if kk > 0 else None, kk)
        if self.ffm and getattr(m, "need_second", True):
            lat = sgd_ops.ffm_pair_sums(bt, c, w[F:], self.Vt, m.nf, m.kk, m._skip)
            sgd_ops.apply_step(bt, part, lat, m.stride, w_lin, w[F:], m.kk, lr, self.l2w, self.l2v, reg_skip, upd_w,
                               bool(getattr(m, "bias_latent", False)), avg, Vt=self.Vt)
        else:
            V = w[F:].view(F, kk) if kk > 0 else None
            sgd_ops.apply_step(bt, part, None, kk, w_lin, V, kk, lr, self.l2w, self.l2v, reg_skip, upd_w,
                               bool(getattr(m, "bias_latent", False)), avg, Vb=self.Vb)

    def _step_cpu(self, w: torch.Tensor, b: int, e: int, lr: float):
        """The same synchronous step with index ops (reference of the GPU kernels)."""
        m = self.m
        d = m.data.train
        X = m.X
        F = m.F
        reg_skip = 0 if m.p.model.need_bias else -1
        upd_w = getattr(m, "need_first", True)
        w_lin = w[:F]
        o0, o1 = int(X.indptr[b]), int(X.indptr[e])
        rows = X.rows_of_nnz[o0:o1] - b
        lin = w_lin[X.indices[o0:o1].long()] * X.values[o0:o1]
        fx = torch.zeros(e - b, dtype=torch.float64, device=w.device).index_add_(0, rows, lin.double())
        S = None
        if m.name == "fm" and m.kk > 0:  # S = X V and the square term from index ops
            V = self.Vb.float() if self.Vb is not None else w[F:].view(F, m.kk)
            vx = V[X.indices[o0:o1].long()] * X.values[o0:o1, None]
            S = torch.zeros((e - b, m.kk), dtype=torch.float32).index_add_(0, rows, vx)
            Q = torch.zeros((e - b, m.kk), dtype=torch.float32).index_add_(0, rows, vx * vx)
            fx = fx + 0.5 * (S.double() ** 2 - Q.double()).sum(1)
        sl_ip = X.indptr[b:e + 1]
        if self.ffm:
            Vf = self.Vb.float().view(-1) if self.Vb is not None else w[F:]
            fx = fx + ffm_forward(sl_ip - o0, X.indices[o0:o1], X.values[o0:o1], d.fields[o0:o1], Vf, m.nf,
                                  m.kk, skip_feat=m._skip).double()
        y = d.y[b:e, 0].double()
        c = (d.weight[b:e].double() * m.loss.grad(fx, y)).float().contiguous()
        cnt = self.cnt
        if cnt is not None:
            sgd_count(sl_ip, X.indices, cnt)
        if self.ffm:
            sgd_ops.ffm_step_cpu(sl_ip, X.indices, X.values, d.fields, w_lin,
                                 w[F:] if getattr(m, "need_second", True) else None, m.nf, m.kk, c, lr, self.l2w,
                                 self.l2v, reg_skip, upd_w, bool(getattr(m, "bias_latent", False)), cnt=cnt,
                                 skip_feat=m._skip, Vb=self.Vb)
            if self.Vb is not None:  # the GPU kernels re-round every slot they change
                self.Vb.copy_(w[F:].view(F, -1))
        else:
            V = w[F:].view(F, m.kk) if (m.name == "fm" and m.kk > 0) else None
            fm_sgd_update(sl_ip, X.indices, X.values, w_lin, V, S, c, lr, self.l2w, self.l2v, reg_skip, upd_w,
                          bool(getattr(m, "bias_latent", False)), Vb=self.Vb, cnt=cnt)
        if cnt is not None:
            sgd_count(sl_ip, X.indices, cnt, clear=True)

    def _average(self, w):
        if self.dist:
            self.comm.allreduce_(w)
            w.mul_(1.0 / self.comm.world)
        self._sync_copy(w)

    def _sync_copy(self, w):
        F = self.m.F
        if self.Vb is not None:
            self.Vb.copy_(w[F:].view(F, -1))
        if self.Vt is not None:
            self.Vt.copy_(w[F:].view(F, self.m.nf, self.m.kk).transpose(0, 1))

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
        batches = self._setup(bounds)
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
                    j = int(order[step])
                    b, e = bounds[j]
                    self._step(w, b, e, lr, batches[j] if batches is not None else None)
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
