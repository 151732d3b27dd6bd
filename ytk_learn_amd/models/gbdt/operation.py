"""GBDT operation: config -> data -> train / evaluate -> model + feature importance files.

Reference: ``J/operation/GBDTOperation.java``, ``J/optimizer/GBDTOptimizer.java:174-480``
(operate: train or just_evaluate), ``J/dataflow/GBDTDataFlow.java`` (dense feature matrix
with ``max_feature_dim`` columns, user dict or count-filtered sorted dict, model load with
objective / base prediction / class_num consistency checks :302-372, dumpModel :376-398,
dumpFeatureImportance :400-420) and ``J/dataflow/GBDTCoreData.java`` (labels: one value, or
a class id / K-vector for softmax; optional init prediction in the 4th field).

``tree_maker = "feature"`` (the reference's single-machine exact greedy maker,
``FeatureParallelTreeMakerByLevel.java``) runs ``exact.ExactGreedyBuilder``: presorted raw
columns, node-segmented orders kept by stable re-partitioning, every distinct value a
candidate (any cardinality). ``YTK_EXACT_BINNED=1`` selects the older emulation on the
histogram engine with ``no_sample`` bins (neighbouring values closer than
``MIN_FEA_SPLIT_GAP`` share one bin, ``binning.merge_split_gap``; <= 65,536 values).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch

from ...config.params import DataParams, gbdt_params_from_config
from ...data.dataflow import (RawShard, assigned_paths, build_dictionary, init_matrix, labels_matrix,
                              parse_options, parse_paths, read_dict_files)
from ...io.fs import FileSystem, create_fs
from ...utils.errors import YtkLearnError
from ...utils.javafmt import java_double_str
from .tree import GBDTModel
from .trainer import GBDTData, GBDTTrainer


def _dense(raw: RawShard, name2idx, F: int, device) -> torch.Tensor:
    """CSR shard -> dense [N, F] (NaN = absent) with the native multithreaded scatter
    (csr_to_dense), then one host->device copy from pinned memory."""
    from ...ops._ext import native
    lut = np.array([name2idx.get(n, -1) for n in raw.names], np.int64) if raw.names else np.zeros(0, np.int64)
    Xh = torch.from_numpy(native().csr_to_dense(raw.indptr, raw.feat, raw.val, lut, F, 0))
    dev = torch.device(device)
    if dev.type != "cuda":
        return Xh
    return Xh.pin_memory().to(dev, non_blocking=True)


class GBDTLoader:
    def __init__(self, cfg, comm, device, log, fs: Optional[FileSystem] = None, transform_fn=None, threads=0):
        self.cfg = cfg
        self.gp, self.dp, self.mp = gbdt_params_from_config(cfg)
        self.comm = comm
        self.device = torch.device(device)
        self.log = log
        self.fs = fs or create_fs(cfg.get_string("fs_scheme", "local"))
        self.transform_fn = transform_fn
        self.threads = threads

    def _parse(self, path, max_err, y_sampling):
        rank = self.comm.rank if self.comm is not None else 0
        world = self.comm.world if self.comm is not None else 1
        paths, mod, rem = assigned_paths(self.fs, path, self.dp, rank, world)
        opts = parse_options(self.dp, None, max_error_tol=max_err, y_sampling=y_sampling,
                             seed=rank * 1000003 + 11, threads=self.threads)
        return RawShard.from_native(parse_paths(self.fs, paths, opts, self.transform_fn, mod, rem), False)

    def _data(self, raw, name2idx, F, K, softmax):
        y = labels_matrix(raw, K, class_ids=softmax, allow_empty=False)
        w = raw.weight.astype(np.float32)
        init = init_matrix(raw, K) if self.gp.sample_dependent_base_prediction else None
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        return GBDTData(_dense(raw, name2idx, F, self.device), t(y), t(w), t(init) if init is not None else None)

    def load(self, model: Optional[GBDTModel] = None):
        gp, dp, mp = self.gp, self.dp, self.mp
        softmax = gp.loss_function.startswith("softmax")
        K = gp.class_num
        ys = dp.y_sampling_map() if dp.y_sampling else None
        raw = self._parse(dp.train_path, dp.train_max_error_tol, ys)
        self.log.info(f"[train data] read lines:{raw.n_lines}, rows:{raw.n_rows}, errors:{raw.n_errors}")
        if gp.just_evaluate and model is not None:
            names = list(model.feature_dict().keys())
            name2idx = {n: i for i, n in enumerate(names)}
        else:
            user = read_dict_files(self.fs, mp.dict_path) if mp.need_dict else None
            name2idx, names = build_dictionary(raw, self.comm, gp.filter_threshold, False, "", user)
        F = len(names)
        if F == 0:
            raise YtkLearnError("feature dim(0) <= 0 is invalid! may be cased by no data or filter all feature")
        if dp.max_feature_dim > 0 and F > dp.max_feature_dim:
            raise YtkLearnError(f"feature number {F} > data.max_feature_dim {dp.max_feature_dim}")
        train = self._data(raw, name2idx, F, K, softmax)
        del raw
        test = None
        if dp.test_path:
            rt = self._parse(dp.test_path, dp.test_max_error_tol, None)
            self.log.info(f"[test data] read lines:{rt.n_lines}, rows:{rt.n_rows}, errors:{rt.n_errors}")
            test = self._data(rt, name2idx, F, K, softmax)
        return train, test, names


def load_gbdt_model(fs: FileSystem, path: str) -> GBDTModel:
    with fs.open_read(path) as f:
        return GBDTModel.loads(f.read())


def run_gbdt(cfg, comm, log, transform_fn=None, threads=0, profile: bool = False):
    t0 = time.perf_counter()
    loader = GBDTLoader(cfg, comm, comm.device, log, None, transform_fn, threads)
    gp, mp, fs = loader.gp, loader.mp, loader.fs
    if gp.tree_maker == "feature":
        if comm.is_dist:
            raise YtkLearnError("[GBDT] feature parallel only support single machine")
        if gp.tree.grow_policy != "level":
            raise YtkLearnError("[GBDT] feature parallel tree maker grows level-wise (tree_grow_policy = level)")
        if os.environ.get("YTK_EXACT_BINNED", "0") == "1":
            # emulation on the histogram path: every distinct value a bin, runs closer than
            # MIN_FEA_SPLIT_GAP merged (<= 65,536 distinct values per feature)
            gp.approximate = [{"cols": "default", "type": "no_sample", "min_split_gap": 1e-16}]
    model = None
    if mp.continue_train or gp.just_evaluate:
        if mp.continue_train and not fs.exists(mp.data_path):
            raise YtkLearnError("GBDT: set continue_train=true, but old model doesn't exist")
        model = load_gbdt_model(fs, mp.data_path)
        if model.loss_name != gp.loss_function:
            raise YtkLearnError(f"GBDT: params inconsistent! objective is {model.loss_name} in old model, "
                                f"but {gp.loss_function} in gbdt.conf")
        if abs(model.base_prediction - gp.uniform_base_prediction) >= 1e-6:
            raise YtkLearnError("GBDT: params inconsistent! uniform_base_prediction differs")
        if model.class_num != gp.class_num:
            raise YtkLearnError("GBDT: params inconsistent! class_num differs")
        if len(model.trees) % gp.class_num != 0:
            raise YtkLearnError("GBDT: model error! tree number is not a multiple of class_num")
        cur = len(model.trees) // gp.class_num
        if mp.continue_train and cur >= gp.round_num:
            raise YtkLearnError(f"GBDT: old model round_num({cur}) >= target round_num({gp.round_num}), "
                                "no need to train, exit!")
        if gp.just_evaluate and cur < gp.round_num:
            raise YtkLearnError(f"GBDT: model round_num({cur}) < use round_num({gp.round_num}), exit!")
        log.info(f"load model finished, old model round_num={cur}, target round_num={gp.round_num}, "
                 f"num_tree_in_group={gp.class_num}")
    train, test, names = loader.load(model)
    log.info(f"LoadDataFlow cost:{time.perf_counter() - t0:.3f}s")
    if gp.just_evaluate:
        return evaluate_gbdt(model, gp, train, test, names, comm, log)
    tr = GBDTTrainer(gp, train, test, comm, names, model, log=log, profile=profile)

    def dump_cb(i):
        dump_gbdt(tr, fs, mp, comm, log)

    tr.train(dump_cb=dump_cb)
    tr.close()  # collective: frees the peer-memory group once every rank has drained
    dump_gbdt(tr, fs, mp, comm, log)
    dump_feature_importance(tr, fs, mp, comm, log)
    return tr


def dump_gbdt(tr: GBDTTrainer, fs, mp, comm, log):
    if comm is not None and not comm.is_master:
        return
    path = mp.data_path
    if not path or not path.strip():
        return
    tr.materialize()
    with fs.open_write(path) as f:
        f.write(tr.model.dumps(True))
    log.info(f"GBDT model is saved in {path}")


def dump_feature_importance(tr: GBDTTrainer, fs, mp, comm, log):
    if comm is not None and not comm.is_master:
        return
    path = mp.feature_importance_path
    if not path or not path.strip() or path == "???":
        return
    imp = tr.feature_importance()
    with fs.open_write(path) as f:
        f.write("feature_name\tsum_split_count\tsum_gain\n")
        for n, (cnt, gain) in imp.items():
            f.write(f"{n}\t{int(cnt)}\t{java_double_str(gain)}\n")
    log.info(f"GBDT feature importance is saved in {path}")


def evaluate_gbdt(model: GBDTModel, gp, train, test, names, comm, log):
    """just_evaluate: score the loaded model's first round_num rounds on train/test."""
    from ...losses import create_loss
    from ...metrics.evaluators import EvalSet
    from ...ops import gbdt as gops
    loss = create_loss(gp.loss_function)
    name2idx = {n: i for i, n in enumerate(names)}
    for t in model.trees:
        t.update_feature_index(name2idx)
    dev = train.X.device
    fl = {k: torch.from_numpy(v).to(dev) for k, v in model.flatten(gp.round_num).items()}
    out = []
    for tag, d in (("train", train), ("test", test)):
        if d is None:
            continue
        K = gp.class_num
        score = torch.zeros((d.n, K), dtype=torch.float32, device=dev)
        gops.forest_predict(d.X.contiguous(), fl, score, 1.0)
        if gp.type == "random_forest":
            score /= max(gp.round_num, 1)
        z = score.double() + float(np.float32(loss.pred2score(model.base_prediction)))
        if d.init_pred is not None and gp.sample_dependent_base_prediction:
            z = z + loss.pred2score(d.init_pred.double())
        y = d.y.double()
        w = d.weight.double() if d.weight is not None else torch.ones(d.n, dtype=torch.float64, device=dev)
        lv = loss.loss(z, y) if loss.multi else loss.loss(z[:, 0], y[:, 0])
        pred = loss.predict(z).float()
        t = torch.tensor([float((w * lv.reshape(d.n, -1).sum(1)).sum()), float(w.sum()), float(d.n)],
                         dtype=torch.float64)
        if comm.is_dist:
            comm.allreduce_(t)
        msg = f"{tag} loss = {java_double_str(float(t[0] / t[1]))}\n"
        info = (2, False) if loss.name == "sigmoid" else ((K, True) if loss.multi else None)
        msg += EvalSet(gp.eval_metric, comm).eval(d.y, pred, d.weight, tag, abs(float(t[1]) - float(t[2])) > 1e-6,
                                                  info)
        log.info(msg)
        out.append(float(t[0] / t[1]))
    return out
