"""Shared plumbing of the L-BFGS model family (linear, multiclass_linear, fm, ffm, gb*).

Reference: ``J/dataflow/ContinuousDataFlow.java`` (params, weight vectors),
``J/dataflow/DataFlow.java`` (loadFlow), the per-model ``*ModelDataFlow`` load/dump
(``model-%05d`` + ``_dict/dict-%05d`` written by each rank for its index range,
``LinearModelDataFlow.java:129-204``) and ``J/optimizer/*HoagOptimizer.java``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...config.params import CommonParams
from ...data.dataflow import (RawShard, SparseData, TRANSFORM_STAT_SUFFIX, assigned_paths, build_dictionary,
                              make_transform_nodes, merge_stats, parse_options, parse_paths, read_dict_files,
                              to_sparse_data, write_transform_stats)
from ...io.fs import FileSystem, create_fs
from ...losses import create_loss
from ...metrics.evaluators import EvalSet
from ...ops.sparse import SparseMatrix
from ...optim.lbfgs import ContinuousModel
from ...utils.errors import YtkLearnError
from ...utils.javafmt import java_float_str


@dataclass
class LoadedData:
    train: SparseData
    test: Optional[SparseData]
    names: List[str]                 # global index -> feature name
    name2idx: Dict[str, int]
    fields: Optional[List[str]] = None


class ContinuousDataLoader:
    """loadFlow for continuous models: parse train/test, dictionary, transforms, CSR on device."""

    def __init__(self, params: CommonParams, comm, device, fs: Optional[FileSystem] = None, log=None,
                 transform_fn=None, threads: int = 0):
        self.p = params
        self.comm = comm
        self.device = torch.device(device)
        self.fs = fs or create_fs(params.fs_scheme)
        self.log = log
        self.transform_fn = transform_fn
        self.threads = threads

    def _info(self, msg):
        if self.log is not None:
            self.log.info(msg)

    def _parse(self, path: str, max_err: int, y_sampling, split_field, want_stats) -> RawShard:
        rank = self.comm.rank if self.comm is not None else 0
        world = self.comm.world if self.comm is not None else 1
        paths, mod, rem = assigned_paths(self.fs, path, self.p.data, rank, world)
        opts = parse_options(self.p.data, self.p.feature, max_error_tol=max_err, y_sampling=y_sampling,
                             split_field=split_field, want_stats=want_stats, seed=rank * 1000003 + 7,
                             threads=self.threads)
        return RawShard.from_native(parse_paths(self.fs, paths, opts, self.transform_fn, mod, rem), want_stats)

    def user_dict(self) -> Optional[List[str]]:
        mp = self.p.model
        model_dict = mp.data_path + "_dict"
        if self.p.loss.just_evaluate:
            self._info(f"just evaluation, so load this model's dict, path:{model_dict}")
            return read_dict_files(self.fs, model_dict)
        if mp.need_dict:
            return read_dict_files(self.fs, mp.dict_path)
        if mp.continue_train and self.fs.exists(model_dict):
            self._info(f"continue_train=true && model dict path exist={model_dict}, will be loaded!")
            return read_dict_files(self.fs, model_dict)
        return None

    def load(self, ylen: int, class_ids: bool = False, split_field: bool = False, init_width: int = 0,
             field_names: Optional[List[str]] = None, bias_field: int = 0) -> LoadedData:
        p = self.p
        need_transform = p.feature.transform.switch_on
        raw = self._parse(p.data.train_path, p.data.train_max_error_tol, p.data.y_sampling_map(), split_field,
                          need_transform)
        self._info(f"[train data] read lines:{raw.n_lines}, rows:{raw.n_rows}, errors:{raw.n_errors}")
        user = self.user_dict()
        name2idx, names = build_dictionary(raw, self.comm, p.feature.filter_threshold, p.model.need_bias,
                                           p.model.bias_feature_name, user)
        if len(names) == 0:
            raise YtkLearnError("feature dim(0) <= 0 is invalid! may be cased by no data or filter all feature")
        self._info(f"feature name to index map! size:{len(names)}")
        transforms = None
        if need_transform:
            stats = merge_stats(raw, self.comm)
            nodes = make_transform_nodes(stats, names, p.feature, p.model.need_bias, p.model.bias_feature_name)
            if self.comm is None or self.comm.is_master:
                write_transform_stats(self.fs, p.model.data_path + TRANSFORM_STAT_SUFFIX, nodes)
            transforms = {name2idx[n]: t for n, t in nodes.items() if n in name2idx}
        fmap = {f: i for i, f in enumerate(field_names)} if field_names is not None else None
        train = to_sparse_data(raw, name2idx, p.model.need_bias, ylen, self.device, self.comm, class_ids=class_ids,
                               init_width=init_width, transforms=transforms, field_map=fmap, bias_field=bias_field)
        del raw
        test = None
        if p.data.test_path:
            rt = self._parse(p.data.test_path, p.data.test_max_error_tol, None, split_field, False)
            self._info(f"[test data] read lines:{rt.n_lines}, rows:{rt.n_rows}, errors:{rt.n_errors}")
            test = to_sparse_data(rt, name2idx, p.model.need_bias, ylen, self.device, self.comm, class_ids=class_ids,
                                  init_width=init_width, transforms=transforms, field_map=fmap,
                                  bias_field=bias_field)
        return LoadedData(train, test, names, name2idx, field_names)


def read_model_lines(fs: FileSystem, path: str, delim: str) -> Dict[str, List[str]]:
    """name -> remaining columns, from every model part file under ``path``."""
    out: Dict[str, List[str]] = {}
    if not fs.exists(path):
        return out
    for f in sorted(fs.recur_get_paths([path])):
        for line in fs.read_lines(f):
            s = line.strip()
            if not s:
                continue
            info = s.split(delim)
            if len(info) < 2:
                continue
            out[info[0]] = info[1:]
    return out


class ContinuousModelBase(ContinuousModel):
    """Common state: params, data matrices, loss, evaluators, sharded dump."""

    name = "continuous"
    ngroups = 1

    def __init__(self, params: CommonParams, data: LoadedData, comm, log, fs: Optional[FileSystem] = None):
        self.p = params
        self.data = data
        self.comm = comm
        self.log = log
        self.fs = fs or create_fs(params.fs_scheme)
        self.device = data.train.values.device
        self.loss = create_loss(params.loss.loss_function)
        self.loss_name = self.loss.name
        self.F = len(data.names)
        self.X = SparseMatrix(data.train.indptr, data.train.indices, data.train.values, self.F)
        self.Xt = None
        if data.test is not None and data.test.n >= 0:
            self.Xt = SparseMatrix(data.test.indptr, data.test.indices, data.test.values, self.F, build_csc=False)
        self.eval_train = EvalSet(params.loss.evaluate_metric, comm)
        self.eval_test = EvalSet(params.loss.evaluate_metric, comm)
        self.pred = None
        self.pred_test = None

    # ---------------------------------------------------------------- helpers
    @property
    def bias_delta(self) -> int:
        return 1 if self.p.model.need_bias else 0

    def has_test(self) -> bool:
        return self.data.test is not None

    def _eval_info(self):
        if self.loss.name == "sigmoid":
            return (2, False)
        if self.loss.multi:
            return (self.data.train.y.shape[1], True)
        return None

    def _weighted(self, d: SparseData) -> bool:
        return abs(d.weight_sum - d.real_num) > 1e-6

    def train_eval(self) -> str:
        if not self.p.loss.evaluate_metric or self.pred is None:
            return ""
        d = self.data.train
        return self.eval_train.eval(d.y, self.pred, d.weight, "train", self._weighted(d), self._eval_info())

    def test_eval(self) -> str:
        if not self.p.loss.evaluate_metric or self.pred_test is None:
            return ""
        d = self.data.test
        return self.eval_test.eval(d.y, self.pred_test, d.weight, "test", self._weighted(d), self._eval_info())

    # ---------------------------------------------------------------- dump
    def index_range(self, dim: int) -> Tuple[int, int]:
        """This rank's feature range for the sharded dump (LinearModelDataFlow.java:133-140)."""
        world = self.comm.world if self.comm is not None else 1
        rank = self.comm.rank if self.comm is not None else 0
        avg = dim // world
        start = rank * avg
        end = dim if rank == world - 1 else (rank + 1) * avg
        return start, end

    def write_parts(self, model_lines: List[str], dict_lines: List[str]):
        rank = self.comm.rank if self.comm is not None else 0
        path = self.p.model.data_path
        mpath = os.path.join(path, "model-%05d" % rank)
        dpath = os.path.join(path + "_dict", "dict-%05d" % rank)
        with self.fs.open_write(mpath) as f:
            for line in model_lines:
                f.write(line + "\n")
        with self.fs.open_write(dpath) as f:
            for line in dict_lines:
                f.write(line + "\n")
        self.log.info(f"model is written to {mpath}")
        self.log.info(f"model-dict is written to {dpath}")

    def load_model_rows(self) -> Dict[str, List[str]]:
        if not (self.p.model.continue_train or self.p.loss.just_evaluate):
            return {}
        rows = read_model_lines(self.fs, self.p.model.data_path, self.p.model.delim)
        if not rows:
            self.log.info("old model doesn't exist, new model...")
        else:
            self.log.info(f"load model finished, old model feature cnt:{len(rows)}")
        return rows


def fmt_f(x: float) -> str:
    """Java String.format("%f")."""
    return "%f" % x


def jfloat(x: float) -> str:
    return java_float_str(x)
