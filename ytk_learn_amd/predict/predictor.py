"""Online (per-sample) and batch (files) predictors for every model family.

Reference: ``J/predictor/OnlinePredictor.java`` (ResultSaveMode PREDICT_RESULT_ONLY /
LABEL_AND_PREDICT / PREDICT_AS_FEATURE, PredictType value / leafid),
``ContinuousOnlinePredictor.java:66-421`` (feature hash + transform-stat replay, batch
predict from files with loss + evaluation), ``LinearOnlinePredictor.java`` (Thompson
sampling), ``MulticlassLinearOnlinePredictor``, ``FMOnlinePredictor``, ``FFMOnlinePredictor``,
``GBDTOnlinePredictor.java:100-486`` (first round_num rounds, RF averaging, base + init
prediction, leaf indexes), ``GBMLROnlinePredictor.java`` & friends (gating values as leaves),
``ITreePredictor.java`` (``tree_leaf_i:v`` features).

MI355X design: a batch file is parsed once by the native multithreaded parser, mapped to
the model's feature index space, and scored as ONE device batch (segmented SpMV/SpMM
kernels for the continuous models and soft trees, the forest kernel for GBDT) instead of
a per-line map walk. The per-sample API builds a one-row batch through the same path.
Deviation (documented): soft-tree predictors use pred2score(uniform_base_prediction) as
the bias, like training; the reference predictor adds the raw prediction value.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..config.hocon import Config, parse_file
from ..config.params import Delim, FeatureParams
from ..data.dataflow import (RawShard, TRANSFORM_STAT_SUFFIX, TransformNode, labels_matrix, load_transform_fn,
                             parse_paths, read_transform_stats)
from ..io.fs import create_fs
from ..losses import create_loss
from ..metrics.evaluators import EvalSet
from ..ops._ext import native
from ..ops.sparse import SparseMatrix
from ..parallel.comm import Comm
from ..utils.errors import YtkLearnError
from ..utils.javafmt import java_double_str as jd
from ..utils.logging import get_logger

SAVE_MODES = ("PREDICT_RESULT_ONLY", "LABEL_AND_PREDICT", "PREDICT_AS_FEATURE")


class PredBatch:
    """Rows mapped into the model's feature space (CSR) + labels/weights/init."""

    def __init__(self, indptr, indices, values, n, weight, raw: RawShard, fields=None):
        self.indptr, self.indices, self.values, self.n = indptr, indices, values, n
        self.weight = weight
        self.raw = raw
        self.fields = fields


class OnlinePredictor:
    model_name = "base"

    def __init__(self, conf: Union[str, Config], device: str = "cpu", log=None):
        self.cfg = parse_file(conf) if isinstance(conf, str) else conf
        self.device = torch.device(device)
        self.fs = create_fs(self.cfg.get_string("fs_scheme", "local"))
        self.log = log or get_logger(None)
        self.delim = Delim.from_config(self.cfg, "data.delim.")

    # ------------------------------------------------------------------ to override
    @property
    def K(self) -> int:
        return 1

    def feature_index(self) -> Dict[str, int]:
        raise NotImplementedError

    def batch_scores(self, b: PredBatch, other: Optional[torch.Tensor]) -> torch.Tensor:
        """fp64 [n, K] scores (margins)."""
        raise NotImplementedError

    def batch_leaf(self, b: PredBatch) -> torch.Tensor:
        raise YtkLearnError(f"{self.model_name} do not support predict type:leafid")

    def parse_options(self) -> dict:
        d = self.delim
        return {"x_delim": d.x_delim, "y_delim": d.y_delim, "features_delim": d.features_delim,
                "feature_name_val_delim": d.feature_name_val_delim, "field_delim": d.field_delim}

    def transforms(self) -> Dict[str, TransformNode]:
        return {}

    def need_bias(self) -> bool:
        return False

    def field_map(self) -> Optional[Dict[str, int]]:
        return None

    def init_width(self) -> int:
        return 0

    # ------------------------------------------------------------------ batching
    def _to_batch(self, raw: RawShard) -> PredBatch:
        idx = self.feature_index()
        lut = np.array([idx.get(n, -1) for n in raw.names], np.int64) if raw.names else np.zeros(0, np.int64)
        gid = lut[raw.feat.astype(np.int64)] if raw.feat.size else np.zeros(0, np.int64)
        rows = np.repeat(np.arange(raw.n_rows, dtype=np.int64), np.diff(raw.indptr))
        val = raw.val.astype(np.float32).copy()
        tr = self.transforms()
        if tr:
            names = np.array(raw.names, dtype=object)
            for n, node in tr.items():
                loc = [i for i, x in enumerate(raw.names) if x == n]
                if loc:
                    m = raw.feat == loc[0]
                    val[m] = node.apply(val[m])
        keep = gid >= 0
        if self.need_bias():
            keep &= gid != 0
        fld = None
        fm = self.field_map()
        if fm is not None:
            flut = np.array([fm.get(f, -1) for f in raw.fields], np.int64) if raw.fields else np.zeros(0, np.int64)
            fld = flut[raw.field.astype(np.int64)] if raw.field.size else np.zeros(0, np.int64)
            keep &= fld >= 0
            fld = fld[keep]
        rows, gid, val = rows[keep], gid[keep], val[keep]
        if self.need_bias():
            n = raw.n_rows
            rows = np.concatenate([rows, np.arange(n)])
            gid = np.concatenate([gid, np.zeros(n, np.int64)])
            val = np.concatenate([val, np.ones(n, np.float32)])
            if fld is not None:
                fld = np.concatenate([fld, np.zeros(n, np.int64)])
        order = np.argsort(rows, kind="stable")
        rows, gid, val = rows[order], gid[order], val[order]
        indptr = np.zeros(raw.n_rows + 1, np.int64)
        np.cumsum(np.bincount(rows, minlength=raw.n_rows), out=indptr[1:])
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dtype=dt, device=self.device)
        return PredBatch(t(indptr, torch.int64), t(gid, torch.int32), t(val, torch.float32), raw.n_rows,
                         t(raw.weight, torch.float32), raw,
                         t(fld[order], torch.int32) if fld is not None else None)

    def _raw_from_features(self, features: Dict[str, float], other=None) -> RawShard:
        names = list(features.keys())
        init = np.zeros(0, np.float32)
        init_ptr = np.array([0, 0], np.int64)
        if other is not None:
            o = np.atleast_1d(np.asarray(other, np.float32))
            init, init_ptr = o, np.array([0, o.size], np.int64)
        fields, field = [], np.zeros(0, np.int32)
        if self.field_map() is not None:
            fdel = self.delim.field_delim
            fl = [n.split(fdel)[0] if fdel in n else n for n in names]
            fields = sorted(set(fl))
            fi = {f: i for i, f in enumerate(fields)}
            field = np.array([fi[f] for f in fl], np.int32)
        return RawShard(1, np.ones(1, np.float32), np.array([0, 0], np.int64), np.zeros(0, np.float32), init_ptr,
                        init, np.array([0, len(names)], np.int64), np.arange(len(names), dtype=np.int32),
                        np.array([float(features[n]) for n in names], np.float32), field, names,
                        np.ones(len(names), np.int64), None, fields)

    def _prepare_features(self, features: Dict[str, float]) -> Dict[str, float]:
        return dict(features)

    # ------------------------------------------------------------------ per-sample API
    def scores(self, features: Dict[str, float], other=None) -> np.ndarray:
        raw = self._raw_from_features(self._prepare_features(features), other)
        b = self._to_batch(raw)
        o = None
        if other is not None:
            o = torch.tensor(np.atleast_1d(np.asarray(other, np.float64))[None, :], device=self.device)
        return self.batch_scores(b, o)[0].cpu().numpy()

    def score(self, features: Dict[str, float], other=None) -> float:
        return float(self.scores(features, other)[0])

    def predicts(self, features: Dict[str, float], other=None) -> np.ndarray:
        s = torch.from_numpy(self.scores(features, other))[None, :]
        return self._pred(s)[0].numpy()

    def predict(self, features: Dict[str, float], other=None) -> float:
        return float(self.predicts(features, other)[0])

    def loss(self, features: Dict[str, float], label, other=None) -> float:
        s = torch.from_numpy(self.scores(features, other))[None, :]
        y = torch.tensor(np.atleast_1d(np.asarray(label, np.float64))[None, :])
        return float(self._loss(s, y)[0])

    def predict_leaf(self, features: Dict[str, float]) -> np.ndarray:
        raw = self._raw_from_features(self._prepare_features(features))
        return self.batch_leaf(self._to_batch(raw))[0].cpu().numpy()

    def leaf_features(self, features: Dict[str, float], features_delim=None, kv_delim=None) -> str:
        fd = features_delim or self.delim.features_delim
        kv = kv_delim or self.delim.feature_name_val_delim
        return fd.join(f"tree_leaf_{i}{kv}{jd(float(v))}" for i, v in enumerate(self.predict_leaf(features)))

    # ------------------------------------------------------------------ shared math
    def _pred(self, s: torch.Tensor) -> torch.Tensor:
        return self.loss_fn.predict(s) if self.loss_fn.multi else self.loss_fn.predict(s[:, 0])[:, None]

    def _loss(self, s: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if self.loss_fn.multi:
            return self.loss_fn.loss(s, y)
        return self.loss_fn.loss(s[:, 0], y[:, 0])

    def _eval_info(self):
        if self.loss_fn.name == "sigmoid":
            return (2, False)
        if self.loss_fn.multi:
            return (self.K, True)
        return None

    # ------------------------------------------------------------------ batch files
    def batch_predict_from_files(self, file_dir: str, transform_script: Optional[str] = None,
                                 save_mode: str = "PREDICT_RESULT_ONLY", suffix: Optional[str] = None,
                                 max_error_tol: int = 100, eval_metric: str = "", predict_type: str = "value"):
        """Predict every file under ``file_dir`` into ``<file><suffix>``; returns avg loss or NaN."""
        save_mode = save_mode.upper()
        if save_mode not in SAVE_MODES:
            raise YtkLearnError(f"unknown result save mode {save_mode}, only support {SAVE_MODES}")
        predict_type = predict_type.lower()
        if predict_type not in ("value", "leafid"):
            raise YtkLearnError(f"unknown predict type {predict_type}")
        suffix = suffix if suffix is not None else f"_{self.model_name}_{save_mode}"
        transform = load_transform_fn(transform_script)
        d = self.delim
        tot_loss, tot_w, tot_n, errors = 0.0, 0.0, 0, 0
        has_label = False
        ys, ps, ws = [], [], []
        for path in self.fs.recur_get_paths([file_dir]):
            out_path = path + suffix
            self.log.info(f"predict path:{path}")
            self.log.info(f"predict result path:{out_path}")
            lines: List[str] = []
            with self.fs.open_read(path) as f:
                for raw_line in f:
                    raw_line = raw_line.rstrip("\n").rstrip("\r")
                    if transform is not None:
                        lines.extend(x if isinstance(x, str) else bytes(x).decode("utf-8")
                                     for x in (transform(raw_line.encode("utf-8")) or []))
                    else:
                        lines.append(raw_line)
            opts = self.parse_options()
            opts["max_error_tol"] = int(max_error_tol)
            buf = ("\n".join(lines) + "\n").encode("utf-8")
            r = native().parse_buffer(buf, opts)
            raw = RawShard.from_native(r, False)
            errors += raw.n_errors
            row_line = r["row_line"]
            b = self._to_batch(raw)
            lab_cnt = np.diff(raw.label_ptr)
            file_has_label = bool((lab_cnt > 0).any())
            has_label |= file_has_label
            if not file_has_label and save_mode != "PREDICT_RESULT_ONLY":
                raise YtkLearnError(f"sample has no label: {lines[row_line[0]] if raw.n_rows else ''}")
            other = None
            if self.init_width() > 0:
                iw = np.diff(raw.init_ptr)
                if (iw != self.init_width()).any():
                    raise YtkLearnError(f"sample dependent base prediction must have {self.init_width()} values")
                other = torch.from_numpy(raw.init.reshape(-1, self.init_width()).astype(np.float64)).to(self.device)
            s = self.batch_scores(b, other) if raw.n_rows else torch.zeros((0, self.K), dtype=torch.float64)
            pred = self._pred(s)
            if predict_type == "leafid":
                outv = self.batch_leaf(b).double()
            else:
                outv = pred
            outn = outv.cpu().numpy()
            if file_has_label:
                y = torch.from_numpy(labels_matrix(raw, self.K if self.loss_fn.multi else 1,
                                                   class_ids=self.loss_fn.multi)).double().to(s.device)
                w = b.weight.double().to(s.device)
                tot_loss += float((w * self._loss(s, y)).sum())
                tot_w += float(w.sum())
                tot_n += raw.n_rows
                ys.append(y.float().cpu())
                ps.append(pred.float().cpu())
                ws.append(b.weight.cpu())
            with self.fs.open_write(out_path) as fo:
                for i in range(raw.n_rows):
                    src = lines[int(row_line[i])].strip()
                    xs = src.split(d.x_delim)
                    vals = outn[i]
                    if save_mode == "PREDICT_RESULT_ONLY":
                        fo.write(d.y_delim.join(jd(float(v)) for v in vals) + "\n")
                    elif save_mode == "LABEL_AND_PREDICT":
                        fo.write(xs[1] + d.x_delim + d.y_delim.join(jd(float(v)) for v in vals) + "\n")
                    else:
                        head = xs[0] + d.x_delim + xs[1] + d.x_delim + (xs[2] if len(xs) > 2 else "")
                        if predict_type == "leafid":
                            feat = d.features_delim.join(f"tree_leaf_{j}{d.feature_name_val_delim}{jd(float(v))}"
                                                         for j, v in enumerate(vals))
                        elif len(vals) == 1 and not self.loss_fn.multi and self.model_name != "gbdt":
                            feat = f"{self.model_name}_label_{d.feature_name_val_delim}{jd(float(vals[0]))}"
                        else:
                            feat = d.features_delim.join(f"{self.model_name}_label_{j}{d.feature_name_val_delim}"
                                                         f"{jd(float(v))}" for j, v in enumerate(vals))
                        fo.write(head + d.features_delim + feat + "\n")
        self.log.info(f"error data format line number:{errors}")
        if not has_label:
            self.log.info("predict complete!")
            return float("nan")
        avg = tot_loss / tot_w if tot_w else float("nan")
        self.log.info(f"loss:{jd(avg)}, sample number:{tot_n}, sample weight sum:{jd(tot_w)}")
        metrics = [m for m in (eval_metric or "").split(",") if m.strip()]
        if metrics:
            y, p, w = torch.cat(ys), torch.cat(ps), torch.cat(ws)
            weighted = abs(float(w.double().sum()) - float(w.shape[0])) > 1e-6
            self.log.info("evaluation results:\n" + EvalSet(metrics, Comm.local()).eval(y, p, w, "", weighted,
                                                                                         self._eval_info()))
        self.log.info("predict complete!")
        return avg


# ---------------------------------------------------------------------------
# continuous models
# ---------------------------------------------------------------------------
class ContinuousPredictor(OnlinePredictor):
    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        c = self.cfg
        self.fp = FeatureParams.from_config(c)
        self.loss_fn = create_loss(c.get_string("loss.loss_function"))
        self.model_path = c.get_string("model.data_path")
        self.model_delim = c.get_string("model.delim", ",")
        self._need_bias = c.get_bool("model.need_bias", True)
        self.bias_name = c.get_string("model.bias_feature_name", "_bias_")
        self._tr_nodes: Dict[str, TransformNode] = {}
        if self.fp.transform.switch_on:
            self._tr_nodes = read_transform_stats(self.fs, self.model_path + TRANSFORM_STAT_SUFFIX)
        self.names: List[str] = []
        self._idx: Dict[str, int] = {}

    def parse_options(self):
        o = super().parse_options()
        fh = self.fp.feature_hash
        if fh.need_feature_hash:
            o.update(feature_hash=True, hash_bucket=int(fh.bucket_size), hash_seed=int(fh.seed) & 0xffffffff,
                     hash_prefix=fh.feature_prefix)
        return o

    def _prepare_features(self, features):
        feats = {k: v for k, v in features.items() if k != self.bias_name}
        fh = self.fp.feature_hash
        if not fh.need_feature_hash:
            return feats
        nat = native()
        out: Dict[str, float] = {}
        for n, v in feats.items():
            h = nat.murmur3_128_aslong(n, int(fh.seed) & 0xffffffff)
            bucket = (h & 0x7fffffff) % fh.bucket_size
            sign = 2.0 * ((h & 0x10000000000) >> 40) - 1.0
            hn = f"{fh.feature_prefix}{bucket}"
            out[hn] = float(np.float32(out.get(hn, 0.0) + sign * v))
        return out

    def transforms(self):
        return self._tr_nodes

    def need_bias(self):
        return self._need_bias

    def feature_index(self):
        return self._idx

    def _read_rows(self) -> Dict[str, List[str]]:
        if not self.fs.exists(self.model_path):
            raise YtkLearnError(f"{self.model_name} model doesn't exist! path:{self.model_path}")
        rows: Dict[str, List[str]] = {}
        for f in sorted(self.fs.recur_get_paths([self.model_path])):
            for line in self.fs.read_lines(f):
                s = line.strip()
                if not s:
                    continue
                info = s.split(self.model_delim)
                if len(info) < 2:
                    continue
                rows[info[0]] = info[1:]
        return rows

    def _index(self, rows: Dict[str, List[str]]):
        names = [self.bias_name] if self._need_bias else []
        names += [n for n in rows if n != self.bias_name]
        self.names = names
        self._idx = {n: i for i, n in enumerate(names)}


class LinearPredictor(ContinuousPredictor):
    model_name = "linear"

    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        rows = self._read_rows()
        self._index(rows)
        w = np.zeros(len(self.names), np.float32)
        prec = np.zeros(len(self.names), np.float32)
        for n, cols in rows.items():
            i = self._idx[n]
            w[i] = float(cols[0])
            if len(cols) > 1 and cols[1] != "null":
                prec[i] = float(cols[1])
        self.w = torch.from_numpy(w).to(self.device)
        with np.errstate(divide="ignore"):
            std = np.where(prec > 0, np.sqrt(1.0 / np.maximum(prec, 1e-30)), 0.0).astype(np.float32)
        self.std = torch.from_numpy(std).to(self.device)
        self.log.info(f"linear model loaded, feature num:{len(self.names)}")

    def batch_scores(self, b, other):
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        s = X.matmul(self.w).double()
        if other is not None:
            s = s + self.loss_fn.pred2score(other[:, 0])
        return s[:, None]

    def thompson_sampling_predict(self, features: Dict[str, float], alpha: float, seed: Optional[int] = None) -> float:
        """sigmoid(sum (w + alpha * std * N(0,1)) x)  (LinearOnlinePredictor.java:141-165)."""
        raw = self._raw_from_features(self._prepare_features(features))
        b = self._to_batch(raw)
        g = torch.Generator(device="cpu")
        if seed is not None:
            g.manual_seed(seed)
        noise = torch.randn(len(self.names), generator=g).to(self.device)
        ws = self.w + float(alpha) * self.std * noise
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        z = X.matmul(ws.float()).double()
        return float(torch.sigmoid(z)[0])


class MulticlassLinearPredictor(ContinuousPredictor):
    model_name = "multiclass_linear"

    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        self._K = self.cfg.get_int("k")
        rows = self._read_rows()
        self._index(rows)
        W = np.zeros((len(self.names), self._K - 1), np.float32)
        for n, cols in rows.items():
            W[self._idx[n]] = [float(v) for v in cols[:self._K - 1]]
        self.W = torch.from_numpy(W).to(self.device)

    @property
    def K(self):
        return self._K

    def batch_scores(self, b, other):
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        s = torch.zeros((b.n, self._K), dtype=torch.float64, device=self.device)
        s[:, :self._K - 1] = X.matmul(self.W).double()
        return s


class FMPredictor(ContinuousPredictor):
    model_name = "fm"

    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        k = self.cfg.get_list("k")
        self.kk = max(int(k[1]), 0)
        rows = self._read_rows()
        self._index(rows)
        F = len(self.names)
        w = np.zeros(F, np.float32)
        V = np.zeros((F, self.kk), np.float32)
        for n, cols in rows.items():
            i = self._idx[n]
            w[i] = float(cols[0])
            if self.kk:
                V[i] = [float(v) for v in cols[1:1 + self.kk]]
        self.w = torch.from_numpy(w).to(self.device)
        self.V = torch.from_numpy(V).to(self.device)

    def batch_scores(self, b, other):
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        fx = X.matmul(self.w).double()
        if self.kk:
            S = X.matmul(self.V).double()
            Q = X.matmul((self.V * self.V).contiguous(), square=True).double()
            fx = fx + 0.5 * (S * S - Q).sum(1)
        return fx[:, None]


class FFMPredictor(ContinuousPredictor):
    model_name = "ffm"

    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        from ..data.dataflow import read_dict_files
        k = self.cfg.get_list("k")
        self.kk = max(int(k[1]), 0)
        fpath = self.cfg.get_string("model.field_dict_path")
        fields = [self.bias_name] if self._need_bias else []
        for f in read_dict_files(self.fs, fpath):
            if f not in fields:
                fields.append(f)
        self.fields = fields
        self._fmap = {f: i for i, f in enumerate(fields)}
        self.nf = len(fields)
        rows = self._read_rows()
        self._index(rows)
        F = len(self.names)
        w = np.zeros(F, np.float32)
        V = np.zeros((F, self.nf * self.kk), np.float32)
        for n, cols in rows.items():
            i = self._idx[n]
            w[i] = float(cols[0])
            V[i] = [float(v) for v in cols[1:1 + self.nf * self.kk]]
        self.w = torch.from_numpy(w).to(self.device)
        self.V = torch.from_numpy(V.reshape(-1)).to(self.device)

    def parse_options(self):
        o = super().parse_options()
        o["split_field"] = True
        return o

    def field_map(self):
        return self._fmap

    def batch_scores(self, b, other):
        from ..ops.ffm import ffm_forward
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        fx = X.matmul(self.w).double()
        if self.kk:
            fx = fx + ffm_forward(b.indptr, b.indices, b.values, b.fields, self.V, self.nf, self.kk).double()
        return fx[:, None]


class GBSTPredictor(ContinuousPredictor):
    """gbmlr / gbsdt / gbhmlr / gbhsdt: sum over trees of lr * mixture(x) + base."""

    def __init__(self, model_name: str, conf, device="cpu", log=None):
        from ..models.gbst.model import VARIANTS
        self.model_name = model_name
        super().__init__(conf, device, log)
        c = self.cfg
        self.gate_kind, self.expert_kind = VARIANTS[model_name]
        self._Kg = c.get_int("k")
        self.rf = c.get_string("type", "gradient_boosting").lower() == "random_forest"
        self.lr = 1.0 if self.rf else c.get_double("learning_rate", 1.0)
        self.sample_dep = c.get_bool("sample_dependent_base_prediction", False)
        base_pred = c.get_double("uniform_base_prediction", 0.5)
        self.base = float(np.float32(self.loss_fn.pred2score(base_pred)))
        info_path = os.path.join(self.model_path, "tree-info")
        if not self.fs.exists(info_path):
            raise YtkLearnError(f"have no {model_name} model info data, old model doesn't exist! path:{info_path}")
        lines = [l.strip() for l in self.fs.read_lines(info_path) if l.strip()]
        if len(lines) != 4:
            raise YtkLearnError("model info must have 4 lines!")
        if int(lines[0].split(":")[1]) != self._Kg:
            raise YtkLearnError("model info K != param K")
        finished = int(lines[2].split(":")[1])
        self.tree_num = min(c.get_int("tree_num", finished), finished)
        K = self._Kg
        self.stride = 2 * K - 1 if self.expert_kind == "linear" else K - 1
        per_tree: List[Tuple[Dict[str, List[float]], Optional[List[float]]]] = []
        all_names = set()
        for t in range(self.tree_num):
            d = os.path.join(self.model_path, "tree-%05d" % t)
            rows: Dict[str, List[float]] = {}
            leaves = None
            for f in sorted(self.fs.recur_get_paths([d])):
                it = iter(self.fs.read_lines(f))
                head = next(it, "")
                if int(head.split(":")[1]) != K:
                    raise YtkLearnError(f"old model k != config's K = {K}")
                if self.expert_kind == "scalar":
                    leaves = [float(v) for v in next(it, "").strip().split(self.model_delim) if v != ""]
                for line in it:
                    s = line.strip()
                    if not s:
                        continue
                    info = s.split(self.model_delim)
                    rows[info[0]] = [float(v) for v in info[1:] if v != ""][:self.stride]
            per_tree.append((rows, leaves))
            all_names.update(rows)
        self._index({n: [] for n in sorted(all_names)})
        F = len(self.names)
        self.Ws, self.leaves = [], []
        for rows, leaves in per_tree:
            W = np.zeros((F, self.stride), np.float32)
            for n, v in rows.items():
                W[self._idx[n], :len(v)] = v
            self.Ws.append(torch.from_numpy(W).to(self.device))
            self.leaves.append(torch.tensor(leaves, dtype=torch.float32, device=self.device) if leaves else None)

    def init_width(self):
        return 1 if self.sample_dep else 0

    def _mixtures(self, b):
        from ..models.gbst.model import gbst_mixture
        X = SparseMatrix(b.indptr, b.indices, b.values, len(self.names), build_csc=False)
        for W, leaves in zip(self.Ws, self.leaves):
            A = X.matmul(W).double()
            yield gbst_mixture(A, self._Kg, self.gate_kind, self.expert_kind, leaves)

    def batch_scores(self, b, other):
        fx = torch.zeros(b.n, dtype=torch.float64, device=self.device)
        for g, H, mu, _ in self._mixtures(b):
            fx += self.lr * ((g * H).sum(1) if mu is None else mu[:, 1])
        if self.rf and self.tree_num > 0:
            fx /= self.tree_num
        fx += self.base
        if other is not None:
            fx = fx + self.loss_fn.pred2score(other[:, 0])
        return fx[:, None]

    def batch_leaf(self, b):
        return torch.cat([g for g, _, _, _ in self._mixtures(b)], dim=1)


# ---------------------------------------------------------------------------
# GBDT
# ---------------------------------------------------------------------------
class GBDTPredictor(OnlinePredictor):
    model_name = "gbdt"

    def __init__(self, conf, device="cpu", log=None):
        super().__init__(conf, device, log)
        from ..models.gbdt.tree import GBDTModel
        c = self.cfg
        path = c.get_string("model.data_path")
        if not self.fs.exists(path):
            raise YtkLearnError(f"gbdt model doesn't exist! path:{path}")
        with self.fs.open_read(path) as f:
            self.model = GBDTModel.loads(f.read())
        self.sample_dep = c.get_bool("optimization.sample_dependent_base_prediction", False)
        self.rf = c.get_string("type", "gradient_boosting").lower() == "random_forest"
        self.loss_fn = create_loss(self.model.loss_name)
        self.base = float(np.float32(self.loss_fn.pred2score(self.model.base_prediction)))
        nk = self.model.class_num
        rounds = len(self.model.trees) // nk
        if len(self.model.trees) == 0 or len(self.model.trees) % nk:
            raise YtkLearnError(f"[GBDT] model error, treeNum={len(self.model.trees)}, numClass={nk}")
        use = c.get_int("optimization.round_num", -1)
        self.use_rounds = rounds if use <= 0 else use
        if self.use_rounds > rounds:
            raise YtkLearnError(f"[GBDT] param error, use round num={self.use_rounds}, but tree only has {rounds} round")
        self._idx = self.model.feature_dict()
        for t in self.model.trees:
            t.update_feature_index(self._idx)
        self.forest = {k: torch.from_numpy(v).to(self.device) for k, v in self.model.flatten(self.use_rounds).items()}
        self.log.info(f"numClass={nk}, useRoundNum={self.use_rounds}, totalRoundNum={len(self.model.trees)}")

    @property
    def K(self):
        return self.model.class_num

    def feature_index(self):
        return self._idx

    def init_width(self):
        return self.K if self.sample_dep else 0

    def _dense(self, b):
        F = max(len(self._idx), 1)
        X = torch.full((b.n, F), float("nan"), dtype=torch.float32, device=self.device)
        rows = torch.repeat_interleave(torch.arange(b.n, device=self.device), b.indptr[1:] - b.indptr[:-1])
        X[rows, b.indices.long()] = b.values
        return X

    def batch_scores(self, b, other):
        from ..ops import gbdt as gops
        out = torch.zeros((b.n, self.K), dtype=torch.float32, device=self.device)
        if b.n:
            gops.forest_predict(self._dense(b), self.forest, out, 1.0)
        s = out.double()
        if self.rf:
            s = s / self.use_rounds
        s = s + self.base
        if other is not None:
            s = s + self.loss_fn.pred2score(other)
        return s

    def batch_leaf(self, b):
        from ..ops import gbdt as gops
        T = int(self.forest["troot"].shape[0])
        leaf = torch.zeros((b.n, T), dtype=torch.int32, device=self.device)
        if b.n:
            gops.forest_predict(self._dense(b), self.forest, None, 1.0, leaf_out=leaf)
        # leaf node id within each tree (Tree.getLeafIndex)
        return leaf


def create_predictor(model_name: str, conf, device: str = "cpu", log=None) -> OnlinePredictor:
    """OnlinePredictorFactory (``J/predictor/OnlinePredictorFactory.java:33-79``)."""
    m = model_name.lower()
    if m == "linear":
        return LinearPredictor(conf, device, log)
    if m == "multiclass_linear":
        return MulticlassLinearPredictor(conf, device, log)
    if m == "fm":
        return FMPredictor(conf, device, log)
    if m == "ffm":
        return FFMPredictor(conf, device, log)
    if m == "gbdt":
        return GBDTPredictor(conf, device, log)
    if m in ("gbmlr", "gbsdt", "gbhmlr", "gbhsdt"):
        return GBSTPredictor(m, conf, device, log)
    raise YtkLearnError(f"unknown model {model_name}")
