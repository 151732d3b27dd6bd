"""Field-aware factorization machine.

Reference: ``J/optimizer/FFMHoagOptimizer.java`` (pairwise field-aware interactions,
two regularization groups, gradient masks as FM) and ``J/dataflow/FFMModelDataFlow.java``
(field = feature-name prefix before ``field_delim``; the field dict file is required and
maps bias -> field 0 when need_bias; dim = F + F*nfield*k1; latent init from
java.util.Random; dump ``name,%f(w),[nfield*k values]``).

Device path: linear part on the deterministic SpMV kernels, pair part on
``csrc/hip/ffm.hip`` (forward: one wave per row, k-wide gathers; backward: column-ordered
gather over the CSC chunks with an LDS accumulator per chunk, no global atomics).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from ...data.dataflow import read_dict_files
from ...ops.blas import row_loss
from ...ops.ffm import ffm_backward_csc, ffm_forward, ffm_pairs_cpu
from ...utils.errors import YtkLearnError
from ...utils.javafmt import java_double_str
from .base import ContinuousModelBase, fmt_f, jfloat
from .fm import random_init


def load_field_dict(fs, params) -> List[str]:
    path = params.model.field_dict_path
    if not path or not fs.exists(path):
        raise YtkLearnError("ffm model must contain field dict, set model.field_dict_path")
    fields = [params.model.bias_feature_name] if params.model.need_bias else []
    seen = set(fields)
    for f in read_dict_files(fs, path):
        if f not in seen:
            seen.add(f)
            fields.append(f)
    return fields


class FFMModel(ContinuousModelBase):
    name = "ffm"
    ngroups = 2

    def __init__(self, params, data, comm, log, fs=None):
        super().__init__(params, data, comm, log, fs)
        k = params.extra.get("k", [1, 4])
        self.k0, self.k1 = int(k[0]), int(k[1])
        self.need_first = self.k0 >= 1
        self.need_second = self.k1 >= 1
        self.bias_latent = bool(params.extra.get("bias_need_latent_factor", False))
        self.fields = data.fields or []
        self.nf = len(self.fields)
        self.kk = max(self.k1, 0)
        self.stride = self.nf * self.kk
        self.dim = self.F + self.F * self.stride
        w = np.zeros(self.dim, np.float32)
        if self.stride > 0:
            w[self.F:] = random_init(params, self.dim - self.F)
            if params.model.need_bias:
                w[self.F:self.F + self.stride] = 0.0
        for n, cols in self.load_model_rows().items():
            i = data.name2idx.get(n)
            if i is None:
                continue
            w[i] = float(cols[0])
            if self.stride > 0:
                w[self.F + i * self.stride:self.F + (i + 1) * self.stride] = [float(c) for c in
                                                                              cols[1:1 + self.stride]]
        self.w = torch.from_numpy(w).to(self.device)
        self._cache = {}
        # the bias without a latent factor keeps an all-zero latent block: skip its pairs
        self._skip = 0 if (params.model.need_bias and not self.bias_latent) else -1
        log.info(f"field dict size:{self.nf}, K:[{self.k0}, {self.k1}], dim:{self.dim}")

    def regular_groups(self) -> List[Tuple[int, int]]:
        return [(self.bias_delta, self.F), (self.F, self.dim)]

    def _max_m(self, key, d) -> int:
        """Entries of the longest row (GPU; the LDS-staged pair forward needs it), cached."""
        from ...ops.ffm import LDS_FWD_FULL
        if not d.indptr.is_cuda or not LDS_FWD_FULL:
            return 0
        ck = ("max_m", key)
        if ck not in self._cache:
            n = d.indptr.shape[0] - 1
            self._cache[ck] = int((d.indptr[1:] - d.indptr[:-1]).max()) if n > 0 else 0
        return self._cache[ck]

    def _pairs(self, key, d):
        if d.indptr.is_cuda:
            return None
        if key not in self._cache:
            self._cache[key] = ffm_pairs_cpu(d.indptr, d.indices, d.values, self._skip)
        return self._cache[key]

    def _forward(self, X, d, w, g, key):
        z_lin = X.matmul(w[:self.F])
        V = w[self.F:]
        cache = self._pairs(key, d)
        z_pair = None
        if self.stride > 0:
            z_pair = ffm_forward(d.indptr, d.indices, d.values, d.fields, V, self.nf, self.kk, cache=cache,
                                 skip_feat=self._skip, max_m=self._max_m(key, d))
        fused = row_loss(self.loss, z_lin, d.y[:, 0], d.weight, z1=z_pair, want_grad=g is not None)
        if fused is not None:  # one fused row pass (sigmoid / l2 on the GPU)
            lsum, pred, c = fused
        else:
            fx = z_lin.double() + (z_pair.double() if z_pair is not None else 0.0)
            y = d.y[:, 0].double()
            wt = d.weight.double()
            lsum = float((wt * self.loss.loss(fx, y)).sum())
            pred = self.loss.predict(fx).float()
            c = (wt * self.loss.grad(fx, y)).float().contiguous() if g is not None else None
        if g is not None:
            X.t_matmul(c, out=g[:self.F])
            if self.stride > 0:
                gv = g[self.F:]
                gv.zero_()
                ffm_backward_csc(X, d.fields, V, self.nf, self.kk, c, gv, skip_feat=self._skip, cache=cache)
            if not self.need_first:
                g[self.bias_delta:self.F] = 0.0
            if not self.need_second:
                g[self.F:] = 0.0
            if not self.bias_latent and self.need_second and self.p.model.need_bias and self.stride > 0:
                g[self.F:self.F + self.stride] = 0.0
        return lsum, pred

    def pure_loss_grad(self, w, g):
        loss, pred = self._forward(self.X, self.data.train, w, g, "train")
        self.pred = pred[:, None]
        return loss

    def test_pure_loss_grad(self, w, g):
        if self.data.test is None:
            return 0.0
        if g is not None and self.Xt._csc is None:
            self.Xt._build_csc()
        loss, pred = self._forward(self.Xt, self.data.test, w, g, "test")
        self.pred_test = pred[:, None]
        return loss

    def dump(self, w, precision):
        wn = w.detach().cpu().numpy()
        V = wn[self.F:].reshape(self.F, self.stride) if self.stride > 0 else np.zeros((self.F, 0), np.float32)
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
