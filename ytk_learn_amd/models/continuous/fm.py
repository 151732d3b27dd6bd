"""Factorization machine: fx = w.x + 1/2 sum_f [(sum_i v_if x_i)^2 - sum_i (v_if x_i)^2].

Reference: ``J/optimizer/FMHoagOptimizer.java:60-160`` (two regularization groups:
linear [bias?1:0, F) and latent [F, dim); g_w += c x, g_v_if += c (s_f - v_if x_i) x_i;
gradient blocks zeroed when k[0] < 1 / k[1] < 1 / the bias has no latent factor) and
``J/dataflow/FMModelDataFlow.java`` (dim = (1+k1) F, latents ~ java.util.Random
N(mean, std) or U(a, b) with the configured seed, bias latent = 0; dump
``name,%f(w),v_1..v_k``).

Device path (deterministic, ``csrc/hip/fm.hip``): one fused pass over the rows gives
  fx = X w + 1/2 sum_f [S^2 - (X∘X)(V∘V)],  S = X V
and one fused pass over the CSC chunks gives
  g_w = X^T c,  G_V = X^T (c∘S) - V ∘ ((X∘X)^T c)
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ...ops._ext import native
from ...ops.blas import row_loss
from ...ops.fm import fm_backward, fm_forward
from .base import ContinuousModelBase, fmt_f, jfloat
from ...utils.javafmt import java_double_str


def random_init(params, n: int, seed_offset: int = 0) -> np.ndarray:
    """java.util.Random stream of RandomParamsUtils.next() (normal or uniform)."""
    rp = params.random
    if rp is None:
        return np.random.default_rng(111111).normal(0.0, 0.01, n).astype(np.float32)
    seed = rp.seed + seed_offset
    if rp.mode == "normal":
        v = native().java_random(seed, n, 0, rp.mean, rp.std)
    else:
        v = native().java_random(seed, n, 1, rp.range_start, rp.range_end)
    return v.astype(np.float32)


class FMModel(ContinuousModelBase):
    name = "fm"
    ngroups = 2

    def __init__(self, params, data, comm, log, fs=None):
        super().__init__(params, data, comm, log, fs)
        k = params.extra.get("k", [1, 8])
        self.k0, self.k1 = int(k[0]), int(k[1])
        self.need_first = self.k0 >= 1
        self.need_second = self.k1 >= 1
        self.bias_latent = bool(params.extra.get("bias_need_latent_factor", False))
        self.kk = max(self.k1, 0)
        self.dim = (1 + self.kk) * self.F
        w = np.zeros(self.dim, np.float32)
        if self.kk > 0:
            w[self.F:] = random_init(params, self.dim - self.F)
            if params.model.need_bias:
                w[self.F:self.F + self.kk] = 0.0
        rows = self.load_model_rows()
        for n, cols in rows.items():
            i = data.name2idx.get(n)
            if i is None:
                continue
            w[i] = float(cols[0])
            if self.kk > 0:
                w[self.F + i * self.kk:self.F + (i + 1) * self.kk] = [float(c) for c in cols[1:1 + self.kk]]
        self.w = torch.from_numpy(w).to(self.device)
        log.info(f"K:[{self.k0}, {self.k1}], bias_need_latent_factor:{self.bias_latent}, "
                 f"need_first_order:{self.need_first}, need_second_order:{self.need_second}")

    def regular_groups(self) -> List[Tuple[int, int]]:
        return [(self.bias_delta, self.F), (self.F, self.dim)]

    def _fx(self, X, w):
        if self.kk > 0:
            return fm_forward(X, w[:self.F], w[self.F:].view(self.F, self.kk))
        return X.matmul(w[:self.F]).double(), None

    def _forward(self, X, d, w, g):
        fx, S = self._fx(X, w)
        fused = row_loss(self.loss, fx, d.y[:, 0], d.weight, want_grad=g is not None)
        if fused is not None:  # one fused row pass (sigmoid / l2 on the GPU)
            lsum, pred, c = fused
        else:
            y = d.y[:, 0].double()
            wt = d.weight.double()
            lsum = float((wt * self.loss.loss(fx, y)).sum())
            pred = self.loss.predict(fx).float()
            c = (wt * self.loss.grad(fx, y)).float() if g is not None else None
        if g is not None:
            if self.kk > 0:
                fm_backward(X, c, S, w[self.F:].view(self.F, self.kk), g[:self.F], g[self.F:].view(self.F, self.kk))
            else:
                X.t_matmul(c, out=g[:self.F])
            if not self.need_first:
                g[self.bias_delta:self.F] = 0.0
            if not self.need_second:
                g[self.F:] = 0.0
            if not self.bias_latent and self.need_second and self.p.model.need_bias and self.kk > 0:
                g[self.F:self.F + self.kk] = 0.0
        return lsum, pred

    def pure_loss_grad(self, w, g):
        loss, pred = self._forward(self.X, self.data.train, w, g)
        self.pred = pred[:, None]
        return loss

    def test_pure_loss_grad(self, w, g):
        if self.data.test is None:
            return 0.0
        if g is not None and self.Xt._csc is None:
            self.Xt._build_csc()
        loss, pred = self._forward(self.Xt, self.data.test, w, g)
        self.pred_test = pred[:, None]
        return loss

    def dump(self, w, precision):
        wn = w.detach().cpu().numpy()
        V = wn[self.F:].reshape(self.F, self.kk) if self.kk > 0 else np.zeros((self.F, 0), np.float32)
        start, end = self.index_range(self.F)
        delim = self.p.model.delim
        lines, dict_lines = [], []
        for i in range(start, end):
            n = self.data.names[i]
            vs = delim.join(jfloat(v) for v in V[i])
            if self.p.model.need_bias and i == 0:
                lines.append(f"{n}{delim}{java_double_str(float(wn[i]))}{delim}{vs}")
                continue
            lines.append(f"{n}{delim}{fmt_f(wn[i])}{delim}{vs}")
            dict_lines.append(n)
        self.write_parts(lines, dict_lines)
