"""Evaluation metrics: bucketed distributed AUC, confusion matrix, mae, rmse.

Reference: ``J/eval/AucEvaluator.java:61-120`` (1e5 prediction slots, weighted and
unweighted pos/neg histograms all-reduced, high->low sweep with 1/2 credit for
ties), ``J/eval/ConfusionMatrixEvaluator.java:80-212``,
``J/eval/PointWiseEvaluator.java:51-89``, ``J/eval/EvaluatorFactory.java:52-64``
(accepted names: auc[@...], rmse, mae, confusion_matrix[@thr]).

The histograms are built on the data's device (``slot_sums``: sort + segmented sums on
the GPU, deterministic and free of hot-slot atomics; torch.bincount on the CPU) and the
all-reduce is one collective per evaluator (weighted+unweighted stacked).
Output strings keep the reference's log grammar (users grep them).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..parallel.comm import Comm
from ..utils.segsum import slot_sums  # noqa: F401 (re-exported)

AUC_SLOTS = 100000


def _jd(x: float) -> str:
    """Java String.valueOf(double)."""
    from ..utils.javafmt import java_double_str
    return java_double_str(x)


class Evaluator:
    def __init__(self, name: str):
        self.name = name

    def eval(self, y, pred, w, comm: Comm, prefix: str, weight_and_real: bool, info=None) -> str:
        raise NotImplementedError


class AucEvaluator(Evaluator):
    def __init__(self, name: str):
        super().__init__(name)
        self.slots = AUC_SLOTS
        if "@" in name:
            try:
                self.slots = int(name.split("@")[1])
            except ValueError:
                pass

    def compute(self, y, pred, w, comm: Comm):
        S = self.slots
        p = pred[:, 0] if pred.dim() == 2 else pred
        yy = y[:, 0] if y.dim() == 2 else y
        idx = (p.float() * float(S)).to(torch.int64).clamp(0, S - 1)
        pos = yy == 1.0
        slot = idx * 2 + (~pos).to(torch.int64)
        ww = w.double() if w is not None else torch.ones_like(p, dtype=torch.float64)
        h = slot_sums(slot, ww, 2 * S)
        if comm.is_dist:
            comm.allreduce_(h)
        res = []
        for k in range(2):
            pc = h[k, 0::2].flip(0)
            nc = h[k, 1::2].flip(0)
            pos_before = torch.cumsum(pc, 0) - pc
            pair = (nc * (pos_before + pc * 0.5)).sum()
            res.append(float(pair / (pc.sum() * nc.sum())))
        return res

    def eval(self, y, pred, w, comm, prefix, weight_and_real, info=None):
        a_w, a_r = self.compute(y, pred, w, comm)
        if weight_and_real:
            return (f"{prefix} {self.name}(weighted) = {_jd(a_w)}\n"
                    f"{prefix} {self.name}(real) = {_jd(a_r)}")
        return f"{prefix} {self.name} = {_jd(a_w)}"


class PointWiseEvaluator(Evaluator):
    def compute(self, y, pred, w, comm: Comm):
        p = pred[:, 0] if pred.dim() == 2 else pred
        yy = y[:, 0] if y.dim() == 2 else y
        d = (yy.float() - p.float()).double()
        row = d * d if self.name == "rmse" else d.abs()
        ww = w.double() if w is not None else torch.ones_like(row)
        t = torch.stack([(row * ww).sum(), ww.sum(), row.sum(), torch.tensor(float(row.numel()),
                                                                             dtype=torch.float64,
                                                                             device=row.device)])
        if comm.is_dist:
            comm.allreduce_(t)
        t = t.tolist()
        f = (lambda s, c: (s / c) ** 0.5) if self.name == "rmse" else (lambda s, c: s / c)
        return f(t[0], t[1]), f(t[2], t[3])

    def eval(self, y, pred, w, comm, prefix, weight_and_real, info=None):
        a_w, a_r = self.compute(y, pred, w, comm)
        if weight_and_real:
            return (f"{prefix} {self.name}(weighted) = {_jd(a_w)}\n"
                    f"{prefix} {self.name}(real) = {_jd(a_r)}")
        return f"{prefix} {self.name} = {_jd(a_w)}"


class ConfusionMatrixEvaluator(Evaluator):
    def __init__(self, name: str):
        super().__init__(name)
        self.thr = 0.5
        if "@" in name:
            self.thr = float(name.split("@")[1])

    def matrix(self, y, pred, w, comm: Comm, K: int, softmax: bool):
        if softmax:
            K = y.shape[1]
            idx = torch.arange(K, device=y.device).expand_as(y)
            target = torch.where(y == 1.0, idx, torch.full_like(idx, -1000000)).max(1).values
            # first max wins (strict >)
            pr = torch.argmax(pred.float(), dim=1)
        else:
            target = (y[:, 0] if y.dim() == 2 else y).to(torch.int64)
            p = pred[:, 0] if pred.dim() == 2 else pred
            pr = (p >= self.thr).to(torch.int64)
        cell = (target * K + pr).clamp(0, K * K - 1)
        ww = w.double() if w is not None else torch.ones(cell.shape[0], dtype=torch.float64, device=cell.device)
        m = slot_sums(cell, ww, K * K)
        if comm.is_dist:
            comm.allreduce_(m)
        return m.cpu().view(2, K, K)

    @staticmethod
    def _table(mat, K, prefix):
        line = "+" + ("-" * 15 + "+") * (K + 1)
        out = [line, "|" + "%16s" % "|" + "".join("%16s" % f"pred c{i} |" for i in range(K)), line]
        for i in range(K):
            out.append("|" + "%16s" % f"actual c{i} |" + "".join("%14.1f |" % float(mat[i, j]) for j in range(K)))
            out.append(line)
        col = mat.sum(0)
        row = mat.sum(1)
        for i in range(K):
            out.append(f"{prefix} class = {i}, precision = {_jd(float(mat[i, i] / col[i]) if col[i] else float('nan'))}"
                       f", recall = {_jd(float(mat[i, i] / row[i]) if row[i] else float('nan'))}")
        tot = float(mat.sum())
        out.append(f"{prefix} accuracy = {_jd(float(mat.diag().sum()) / tot if tot else float('nan'))}")
        return "\n".join(out)

    def eval(self, y, pred, w, comm, prefix, weight_and_real, info=None):
        K, softmax = info if info is not None else (2, False)
        m = self.matrix(y, pred, w, comm, K, softmax)
        Kk = m.shape[1]
        if weight_and_real:
            return (f"{prefix} {self.name}(weighted) = \n{self._table(m[0], Kk, prefix)}\n"
                    f"{prefix} {self.name}(real) = \n{self._table(m[1], Kk, prefix)}")
        return f"{prefix} {self.name} = \n{self._table(m[0], Kk, prefix)}"


def create_evaluator(name: str) -> Evaluator:
    n = name.strip()
    if n.startswith("auc"):
        return AucEvaluator(n)
    if n in ("rmse", "mae"):
        return PointWiseEvaluator(n)
    if n.startswith("confusion_matrix"):
        return ConfusionMatrixEvaluator(n)
    raise ValueError(f"unknown evaluation metric type:{name}")


class EvalSet:
    def __init__(self, names: List[str], comm: Comm):
        self.evals = [create_evaluator(n) for n in names]
        self.comm = comm

    def eval(self, y, pred, w, prefix, weight_and_real, info=None) -> str:
        return "".join(e.eval(y, pred, w, self.comm, prefix, weight_and_real, info) + "\n" for e in self.evals)
