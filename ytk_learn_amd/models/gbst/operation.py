"""Boosting loop for soft trees (reference: ``J/operation/GBMLROperation.java:37-115``)."""
from __future__ import annotations

from ...config.params import CommonParams
from ...io.fs import create_fs
from ...optim.lbfgs import HoagOptimizer
from ...utils.fault import fault_point
from ..continuous.base import ContinuousDataLoader
from .model import GBSTModel


def build_gbst(model_name, cfg, comm, log, transform_fn=None, threads=0):
    params = CommonParams.from_config(cfg, model_name)
    fs = create_fs(params.fs_scheme)
    loader = ContinuousDataLoader(params, comm, comm.device, fs, log, transform_fn, threads)
    init_width = 1 if params.extra.get("sample_dependent_base_prediction", False) else 0
    data = loader.load(1, init_width=init_width)
    return GBSTModel(model_name, params, data, comm, log, fs), params


def run_gbst(model_name, cfg, comm, log, transform_fn=None, threads=0):
    model, params = build_gbst(model_name, cfg, comm, log, transform_fn, threads)
    if not model.load_or_init():
        return None
    just_eval = params.loss.just_evaluate
    tree = model.finished
    prev = float("inf")
    res = None
    while True:
        fault_point("gbst", tree, comm.rank)
        log.info(f"finished tree num:{model.finished}, now constructing treeid:{tree}")
        opt = HoagOptimizer(model, params.line_search, params.loss.l1, params.loss.l2, comm, log,
                            model.data.train.weight_sum,
                            model.data.test.weight_sum if model.data.test is not None else 0.0,
                            params.hyper, just_eval, params.model.dump_freq)
        res = opt.run(model.w)
        if just_eval:
            log.info("just evalate, return!")
            return res
        log.info(f"gradient boost cur loss:{res.loss}, prev loss:{prev}, will construct next tree!")
        log.info(f"accumulate tree:{tree}...")
        model.accumulate(model.X, model.z, model.w, model.fmask)
        if model.Xt is not None:
            model.accumulate(model.Xt, model.z_test, model.w, model.fmask)
        log.info(f"constructing treeid:{tree} finished!")
        model.finished += 1
        log.info(f"finished num:{model.finished}")
        model.dump_info()
        tree += 1
        if tree >= model.tree_num:
            break
        prev = res.loss
        model.init_w()
        model.next_sample(model.rate, model.frate)
    return res
