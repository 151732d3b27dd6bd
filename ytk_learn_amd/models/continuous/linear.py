"""Linear model (logistic / least squares / any binary or regression loss) with L-BFGS.

Reference: ``J/optimizer/LinearHoagOptimizer.java`` (z = Xw :76-87, loss/pred/D/l' per
row :127-147, g = X^T(weight*l') :89-106, Laplace precision diag(X^T D X) + l2*W without
the intercept :179-206) and ``J/dataflow/LinearModelDataFlow.java`` (zero init, continue
train by name :67-121, dump ``name,w,precision`` with ``%f`` and ``_bias_,w,null``).

Device path: z and g are the deterministic segmented SpMV kernels of
``csrc/hip/sparse.hip``; the per-row fp64 loss math is one fused pass (``ops.blas.row_loss``)
for sigmoid / l2 and fp64 torch otherwise.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...ops.blas import row_loss
from .base import ContinuousModelBase, fmt_f, jfloat


class LinearModel(ContinuousModelBase):
    name = "linear"

    def __init__(self, params, data, comm, log, fs=None):
        super().__init__(params, data, comm, log, fs)
        if self.loss.multi:
            raise ValueError(f"linear model needs a single-output loss, got {self.loss.name}")
        self.dim = self.F
        self.w = torch.zeros(self.dim, dtype=torch.float32, device=self.device)
        rows = self.load_model_rows()
        if rows:
            w = np.zeros(self.dim, np.float32)
            for n, cols in rows.items():
                i = data.name2idx.get(n)
                if i is not None:
                    w[i] = float(cols[0])
            self.w.copy_(torch.from_numpy(w))
        self.D = None

    def regular_groups(self) -> List[Tuple[int, int]]:
        return [(self.bias_delta, self.dim)]

    def _forward(self, X, d, w, g):
        z32 = X.matmul(w)
        fused = row_loss(self.loss, z32, d.y[:, 0], d.weight, want_grad=g is not None)
        if fused is not None:  # one fused row pass (sigmoid / l2 on the GPU)
            loss, pred, c = fused
            if g is not None:
                X.t_matmul(c, out=g)
            return loss, pred
        z = z32.double()
        y = d.y[:, 0].double()
        wt = d.weight.double()
        lv = self.loss.loss(z, y)
        pred = self.loss.predict(z).float()
        if g is not None:
            d1 = self.loss.grad(z, y)
            X.t_matmul((wt * d1).float(), out=g)
        return float((wt * lv).sum()), pred

    def pure_loss_grad(self, w, g):
        loss, pred = self._forward(self.X, self.data.train, w, g)
        self.pred = pred[:, None]
        return loss

    def test_pure_loss_grad(self, w, g):
        d = self.data.test
        if d is None:
            return 0.0
        if g is not None and self.Xt._csc is None:
            self.Xt._build_csc()
        loss, pred = self._forward(self.Xt, d, w, g)
        self.pred_test = pred[:, None]
        return loss

    def precision(self, w, l2: Sequence[float], wsum: float) -> Optional[torch.Tensor]:
        """diag(X^T diag(weight*l'') X) without the intercept (the optimizer adds l2*W)."""
        d = self.data.train
        z = self.X.matmul(w).double()
        D = (self.loss.hess(z, d.y[:, 0].double()) * d.weight.double()).float()
        prec = self.X.t_matmul(D, square=True)
        if self.p.model.need_bias:
            # the bias column is every row's intercept: excluded like the reference
            prec[0] = 0.0
        return prec

    def dump(self, w, precision):
        wn = w.detach().cpu().numpy()
        pn = precision.detach().cpu().numpy() if precision is not None else np.zeros_like(wn)
        start, end = self.index_range(self.dim)
        delim = self.p.model.delim
        lines, dict_lines = [], []
        bias = self.p.model.bias_feature_name
        nz = int(np.count_nonzero(wn))
        for i in range(start, end):
            n = self.data.names[i]
            if self.p.model.need_bias and i == 0:
                lines.append(f"{n}{delim}{jfloat(wn[i])}{delim}null")
                continue
            if wn[i] == 0.0:
                continue
            lines.append(f"{n}{delim}{fmt_f(wn[i])}{delim}{fmt_f(pn[i])}")
            dict_lines.append(n)
        self.write_parts(lines, dict_lines)
        self.log.info(f"all nonzero num:{nz}, dim:{self.dim}, prop:{nz / max(self.dim, 1)}")
