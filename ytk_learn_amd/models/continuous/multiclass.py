"""Multiclass linear model: K-1 free weight vectors, the last class score fixed at 0.

Reference: ``J/optimizer/MulticlassLinearHoagOptimizer.java:56-149`` (W is F x (K-1),
row-major per feature; scores wx[0..K-2] = X W, wx[K-1] = 0; ``loss.all`` gives loss,
prediction and d1; g[f, p] += weight * d1[p] * x; regularization group starts at the bias
row, i.e. index K-1) and ``J/dataflow/MulticlassLinearModelDataFlow.java`` (labels are a
class id or a K-vector summing to 1; dump ``name,w_0,...,w_{K-2}`` with Float.toString).
Device path: S = X W and G = X^T D as the segmented SpMM kernel (J = K-1 columns); the
per-row loss / prediction / D epilogue is one fused HIP pass (``ops.blas.multiclass_row_loss``,
every multiclass loss, K <= 64) and fp64 torch otherwise.
Note: y_sampling keys on the first label value (a class id line); K-vector label lines are
not sampled by class.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ...ops.blas import multiclass_row_loss
from .base import ContinuousModelBase, jfloat


class MulticlassLinearModel(ContinuousModelBase):
    name = "multiclass_linear"

    def __init__(self, params, data, comm, log, fs=None):
        super().__init__(params, data, comm, log, fs)
        self.K = int(params.extra.get("k", data.train.y.shape[1]))
        if self.K < 2:
            raise ValueError("multiclass_linear needs k >= 2")
        if not self.loss.multi:
            raise ValueError(f"multiclass_linear needs a multi-class loss, got {self.loss.name}")
        self.S = self.K - 1
        self.dim = self.F * self.S
        self.w = torch.zeros(self.dim, dtype=torch.float32, device=self.device)
        rows = self.load_model_rows()
        if rows:
            w = np.zeros((self.F, self.S), np.float32)
            for n, cols in rows.items():
                i = data.name2idx.get(n)
                if i is not None:
                    w[i] = [float(c) for c in cols[:self.S]]
            self.w.copy_(torch.from_numpy(w.reshape(-1)))

    def regular_groups(self) -> List[Tuple[int, int]]:
        return [(self.S if self.p.model.need_bias else 0, self.dim)]

    def _eval_info(self):
        return (self.K, True)

    def _forward(self, X, d, w, g):
        W = w.view(self.F, self.S)
        s32 = X.matmul(W)
        fused = multiclass_row_loss(self.loss, s32, d.y, d.weight, want_grad=g is not None)
        if fused is not None:  # one fused row pass on the GPU
            loss, pred, D = fused
            if g is not None:
                X.t_matmul(D, out=g.view(self.F, self.S))
            return loss, pred
        z = torch.zeros((X.n, self.K), dtype=torch.float64, device=self.device)
        z[:, :self.S] = s32.double()
        y = d.y.double()
        lv, pred, d1 = self.loss.all(z, y)
        wt = d.weight.double()
        if g is not None:
            D = (d1[:, :self.S] * wt[:, None]).float().contiguous()
            X.t_matmul(D, out=g.view(self.F, self.S))
        return float((wt * lv).sum()), pred.float()

    def pure_loss_grad(self, w, g):
        loss, self.pred = self._forward(self.X, self.data.train, w, g)
        return loss

    def test_pure_loss_grad(self, w, g):
        if self.data.test is None:
            return 0.0
        if g is not None and self.Xt._csc is None:
            self.Xt._build_csc()
        loss, self.pred_test = self._forward(self.Xt, self.data.test, w, g)
        return loss

    def dump(self, w, precision):
        W = w.detach().cpu().numpy().reshape(self.F, self.S)
        start, end = self.index_range(self.F)
        delim = self.p.model.delim
        lines, dict_lines = [], []
        for i in range(start, end):
            n = self.data.names[i]
            lines.append(n + delim + delim.join(jfloat(v) for v in W[i]))
            dict_lines.append(n)
        self.write_parts(lines, dict_lines)
