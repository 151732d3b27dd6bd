#!/usr/bin/env python3
"""Generate the demo configs and run scripts (reference: ``demo/**``, 17 configs, 9 models).

Each demo config is this repo's ``config/model/<model>.conf`` with the demo's settings
applied (data paths, loss, tree settings...), so the demo files stay in the same flat
dotted-key style as the model configs. Run from the repo root:

    python demo/build_demos.py          # (re)writes demo/<model>/<task>/{<model>.conf,run.sh}

The datasets (agaricus, dermatology, machine: the public LibSVM files the reference ships
under demo/data/libsvm) are not vendored; ``demo/prepare_data.sh`` converts them from
``$YTK_DEMO_DATA`` (default ``demo/data/libsvm``) into ``demo/data/ytklearn``.
"""
from __future__ import annotations

import json
import os
import stat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = "demo/data/ytklearn"

BIN = {"data.train.data_path": f"{DATA}/agaricus.train.ytklearn",
       "data.test.data_path": f"{DATA}/agaricus.test.ytklearn"}
REG = {"data.train.data_path": f"{DATA}/machine.train.ytklearn",
       "data.test.data_path": f"{DATA}/machine.test.ytklearn",
       "loss.loss_function": "l2", "loss.evaluate_metric": ["rmse"]}
MULTI = {"data.train.data_path": f"{DATA}/dermatology.train.ytklearn",
         "data.test.data_path": f"{DATA}/dermatology.test.ytklearn"}
NO_SAMPLE = [{"cols": "default", "type": "no_sample"}]

# (model, task dir, settings, predict metrics)
DEMOS = [
    ("linear", "linear/binary_classification", dict(BIN), "auc"),
    ("linear", "linear/regression", dict(REG), "rmse"),
    ("multiclass_linear", "multiclass_linear", dict(MULTI, k=6), "confusion_matrix"),
    ("fm", "fm/binary_classification", dict(BIN), "auc"),
    ("fm", "fm/regression", dict(REG), "rmse"),
    ("ffm", "ffm/binary_classification", dict(BIN, **{"model.field_dict_path": f"{DATA}/agaricus.field.dict"}),
     "auc"),
    ("ffm", "ffm/regression", dict(REG, **{"model.field_dict_path": f"{DATA}/machine.field.dict"}), "rmse"),
    ("gbmlr", "gbmlr/binary_classification", dict(BIN), "auc"),
    ("gbmlr", "gbmlr/regression", dict(REG), "rmse"),
    ("gbsdt", "gbsdt/binary_classification", dict(BIN), "auc"),
    ("gbsdt", "gbsdt/regression", dict(REG), "rmse"),
    ("gbhmlr", "gbhmlr/binary_classification", dict(BIN), "auc"),
    ("gbhmlr", "gbhmlr/regression", dict(REG), "rmse"),
    ("gbhsdt", "gbhsdt/binary_classification", dict(BIN), "auc"),
    ("gbhsdt", "gbhsdt/regression", dict(REG), "rmse"),
    # GBDT: loss-wise growth, 3 rounds (the README of this demo publishes the losses)
    ("gbdt", "gbdt/binary_classification", {
        **BIN, "data.max_feature_dim": 117, "model.dict_path": f"{DATA}/agaricus.feat_dict",
        "model.feature_importance_path": "demo/gbdt/binary_classification/feature_importance",
        "optimization.tree_grow_policy": "loss", "optimization.round_num": 3,
        "optimization.min_child_hessian_sum": 1, "optimization.min_split_samples": -1,
        "optimization.max_leaf_cnt": 16, "optimization.regularization.learning_rate": 0.5,
        "optimization.eval_metric": ["confusion_matrix", "auc"], "optimization.silent": 1,
        "feature.approximate": NO_SAMPLE}, "auc"),
    ("gbdt", "gbdt/multiclass_classification", {
        **MULTI, "data.max_feature_dim": 33, "model.need_dict": True,
        "model.dict_path": f"{DATA}/dermatology.feat_dict",
        "model.feature_importance_path": "demo/gbdt/multiclass_classification/feature_importance",
        "optimization.round_num": 5, "optimization.max_depth": 6, "optimization.min_split_samples": -1,
        "optimization.loss_function": "softmax", "optimization.regularization.learning_rate": 0.1,
        "optimization.uniform_base_prediction": 0.0, "optimization.class_num": 6,
        "optimization.eval_metric": ["confusion_matrix"], "feature.approximate": NO_SAMPLE,
        "feature.missing_value": "quantile@0.5"}, "confusion_matrix"),
    # exact greedy (feature-parallel maker) on the raw LibSVM lines through a transform hook
    ("gbdt", "gbdt/regression_l2", {
        "data.train.data_path": "demo/data/libsvm/machine.train.libsvm",
        "data.test.data_path": "demo/data/libsvm/machine.test.libsvm", "data.max_feature_dim": 35,
        "model.dict_path": f"{DATA}/machine.feat_dict",
        "model.feature_importance_path": "demo/gbdt/regression_l2/feature_importance",
        "optimization.tree_maker": "feature", "optimization.round_num": 2, "optimization.max_depth": 3,
        "optimization.min_split_samples": -1, "optimization.loss_function": "l2",
        "optimization.regularization.learning_rate": 1.0, "optimization.uniform_base_prediction": 0.0,
        "optimization.eval_metric": ["rmse"], "optimization.silent": 1, "optimization.watch_train": True,
        "optimization.watch_test": True, "feature.approximate": NO_SAMPLE, "feature.missing_value": "quantile"},
     "rmse"),
]
TRANSFORM = {"gbdt/regression_l2": "demo/gbdt/regression_l2/transform.py"}


def render(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, list) and v and isinstance(v[0], dict):
        items = ", ".join("{" + ", ".join(f"{k} = {render(x)}" for k, x in d.items()) + "}" for d in v)
        return f"[{items}]"
    return json.dumps(v)


def apply(base_text: str, settings: dict) -> str:
    """Replace the values of ``settings`` keys in the flat config text; append new keys."""
    out, skip_depth, done = [], 0, set()
    for line in base_text.splitlines():
        if skip_depth > 0:  # inside a replaced multi-line value
            skip_depth += line.count("[") + line.count("{") - line.count("]") - line.count("}")
            continue
        key = line.split("=", 1)[0].strip() if "=" in line and not line.lstrip().startswith("#") else None
        if key in settings:
            rhs = line.split("=", 1)[1].split("#", 1)[0]
            depth = rhs.count("[") + rhs.count("{") - rhs.count("]") - rhs.count("}")
            out.append(f"{key} = {render(settings[key])}")
            done.add(key)
            skip_depth = depth
            continue
        out.append(line)
    extra = [k for k in settings if k not in done]
    if extra:
        out.append("")
        out.append("# demo settings")
        out.extend(f"{k} = {render(settings[k])}" for k in extra)
    return "\n".join(out) + "\n"


RUN = """#!/usr/bin/env bash
# demo: {task} ({model}). Run from anywhere; paths are relative to the repo root.
set -euo pipefail
cd "$(dirname "$0")/{up}"
bash demo/prepare_data.sh
bash bin/local_optimizer.sh {model} demo/{task}/{model}.conf 1 {transform}
bash bin/predict.sh {model} {test} demo/{task}/{model}.conf LABEL_AND_PREDICT value {metrics} {transform}
"""


def main():
    for model, task, settings, metrics in DEMOS:
        settings = dict(settings)
        settings.setdefault("model.data_path", f"demo/{task}/{model}.model")
        base = open(os.path.join(ROOT, "config", "model", f"{model}.conf")).read()
        d = os.path.join(ROOT, "demo", task)
        os.makedirs(d, exist_ok=True)
        head = f"# demo {task}: generated by demo/build_demos.py from config/model/{model}.conf\n"
        with open(os.path.join(d, f"{model}.conf"), "w") as f:
            f.write(head + apply(base, settings))
        up = "/".join([".."] * (task.count("/") + 2))
        run = os.path.join(d, "run.sh")
        with open(run, "w") as f:
            f.write(RUN.format(task=task, model=model, up=up, transform=TRANSFORM.get(task, ""),
                               test=settings["data.test.data_path"], metrics=metrics))
        os.chmod(run, os.stat(run).st_mode | stat.S_IXUSR | stat.S_IXGRP | stat.S_IXOTH)
        print("wrote", os.path.relpath(d, ROOT))


if __name__ == "__main__":
    main()
