"""Training entry point for every model family.

Reference: ``J/worker/TrainWorker.java:54-239`` (parse config + overrides, create the
communicator, DataFlow init/loadFlow, run the operation per worker, report load vs train
time), ``J/operation/TrainOperationFactory.java:34-54`` (model -> operation) and
``J/optimizer/OptimizerFactory.java``.

One process per GPU: launch with ``python -m torch.distributed.run --nproc-per-node N
-m ytk_learn_amd.cli.train ...`` (or ``bin/local_optimizer.sh``); rank/world come from
the environment and collectives go over RCCL (device tensors) / gloo (host objects).
"""
from __future__ import annotations

import os
import time
from typing import Any, Dict, Optional, Union

import torch

from .config.hocon import Config, parse_file
from .config.params import CommonParams
from .data.dataflow import load_transform_fn
from .io.fs import create_fs
from .parallel.comm import Comm
from .utils.errors import YtkLearnError
from .utils.logging import get_logger

CONTINUOUS = ("linear", "multiclass_linear", "fm", "ffm")
GBST = ("gbmlr", "gbsdt", "gbhmlr", "gbhsdt")
MODELS = CONTINUOUS + ("gbdt",) + GBST


def load_config(conf: Union[str, Config], overrides: Optional[Dict[str, Any]] = None) -> Config:
    c = parse_file(conf) if isinstance(conf, str) else conf
    if overrides:
        c = c.with_overrides(overrides)
    return c


def build_continuous_model(model_name: str, params: CommonParams, comm, device, log, transform_fn=None,
                           threads: int = 0):
    """(model, loaded data) for linear / multiclass_linear / fm / ffm."""
    from .models.continuous.base import ContinuousDataLoader
    fs = create_fs(params.fs_scheme)
    loader = ContinuousDataLoader(params, comm, device, fs, log, transform_fn, threads)
    if model_name == "linear":
        from .models.continuous.linear import LinearModel
        data = loader.load(1)
        return LinearModel(params, data, comm, log, fs)
    if model_name == "multiclass_linear":
        from .models.continuous.multiclass import MulticlassLinearModel
        K = int(params.extra.get("k", 2))
        data = loader.load(K, class_ids=True)
        return MulticlassLinearModel(params, data, comm, log, fs)
    if model_name == "fm":
        from .models.continuous.fm import FMModel
        data = loader.load(1)
        return FMModel(params, data, comm, log, fs)
    if model_name == "ffm":
        from .models.continuous.ffm import FFMModel, load_field_dict
        fields = load_field_dict(fs, params)
        data = loader.load(1, split_field=True, field_names=fields, bias_field=0)
        return FFMModel(params, data, comm, log, fs)
    raise YtkLearnError(f"unknown continuous model {model_name}")


def train(model_name: str, conf: Union[str, Config], overrides: Optional[Dict[str, Any]] = None,
          transform_script: Optional[str] = None, device: Optional[str] = None, comm: Optional[Comm] = None,
          threads: int = 0, log=None):
    """Train ``model_name`` with config ``conf``. Returns the optimizer/trainer result."""
    model_name = model_name.lower()
    if model_name not in MODELS:
        raise YtkLearnError(f"unknown model {model_name}, only support {list(MODELS)}")
    cfg = load_config(conf, overrides)
    comm = comm or Comm.from_env(device)
    dev = comm.device
    verbose = cfg.get_bool("verbose", False)
    log = log or get_logger(comm, verbose=verbose, jsonl_path=os.environ.get("YTK_METRICS_JSONL") or None)
    log.info(f"model:{model_name}, world:{comm.world}, device:{dev}")
    transform_fn = load_transform_fn(transform_script)
    t0 = time.perf_counter()
    if model_name in CONTINUOUS:
        params = CommonParams.from_config(cfg, model_name)
        model = build_continuous_model(model_name, params, comm, dev, log, transform_fn, threads)
        t_load = time.perf_counter() - t0
        log.info(f"LoadDataFlow cost:{t_load:.3f}s")
        if params.optimizer == "sgd":  # extension: mini-batch Hogwild!-style SGD (optim/sgd.py)
            from .optim.sgd import SGDOptimizer
            opt = SGDOptimizer(model, params.sgd, params.loss.l1, params.loss.l2, comm, log,
                               model.data.train.weight_sum,
                               model.data.test.weight_sum if model.data.test is not None else 0.0,
                               params.model.dump_freq)
            res = opt.run(model.w)
            log.info(f"Train cost details: LoadDataFlow:{t_load:.3f}s, PreprocessAndTrain:"
                     f"{time.perf_counter() - t0 - t_load:.3f}s")
            return res
        from .optim.lbfgs import HoagOptimizer
        opt = HoagOptimizer(model, params.line_search, params.loss.l1, params.loss.l2, comm, log,
                            model.data.train.weight_sum,
                            model.data.test.weight_sum if model.data.test is not None else 0.0,
                            params.hyper, params.loss.just_evaluate, params.model.dump_freq)
        res = opt.run(model.w)
        log.info(f"Train cost details: LoadDataFlow:{t_load:.3f}s, PreprocessAndTrain:"
                 f"{time.perf_counter() - t0 - t_load:.3f}s")
        return res
    if model_name == "gbdt":
        from .models.gbdt.operation import run_gbdt
        return run_gbdt(cfg, comm, log, transform_fn, threads)
    from .models.gbst.operation import run_gbst
    return run_gbst(model_name, cfg, comm, log, transform_fn, threads)
