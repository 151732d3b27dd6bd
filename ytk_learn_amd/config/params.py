"""Typed, validated parameter objects built from a HOCON :class:`Config`.

Mirrors the reference's ``J/param`` classes (keys, defaults on missing keys,
CheckUtils validations):
  DataParams        J/param/DataParams.java:41-158
  FeatureParams     J/param/FeatureParams.java, FeatureHashParams.java, TransformParams.java
  ModelParams       J/param/ModelParams.java:39-57
  LossParams        J/param/LossParams.java:42-78
  LineSearchParams  J/param/LineSearchParams.java:43-139
  HyperParams       J/param/HyperParams.java:41-150
  RandomParams      J/param/RandomParams.java:41-101
  GBDT              J/param/gbdt/GBDT*Params.java (GBDTOptimizationParams.java:108-238)
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set

from .hocon import Config, ConfigError, ConfigMissing

EVAL_NAMES = ("auc", "confusion_matrix", "mae", "rmse")


def check(cond: bool, msg: str, *args):
    """CheckUtils.check: raise YtkLearnError(msg % args) when cond is false."""
    if not cond:
        from ..utils.errors import YtkLearnError
        raise YtkLearnError(msg % args if args else msg)


def _mode(name: str, allowed, key: str) -> str:
    n = str(name).lower()
    check(n in allowed, "unknown %s:%s, only support:%s", key, name, list(allowed))
    return n


# ---------------------------------------------------------------------------
@dataclass
class Delim:
    x_delim: str = "###"
    y_delim: str = ","
    features_delim: str = ","
    feature_name_val_delim: str = ":"
    field_delim: str = "@"  # ffm only

    @classmethod
    def from_config(cls, c: Config, prefix: str) -> "Delim":
        d = cls(c.get_string(prefix + "x_delim"), c.get_string(prefix + "y_delim"),
                c.get_string(prefix + "features_delim"), c.get_string(prefix + "feature_name_val_delim"),
                c.get_string(prefix + "field_delim", "@"))
        check(d.x_delim != d.y_delim, "%sx_delim:%s must be different with %sy_delim:%s!", prefix, d.x_delim,
              prefix, d.y_delim)
        check(d.x_delim != d.features_delim, "%sx_delim:%s must be different with %sfeatures_delim:%s!", prefix,
              d.x_delim, prefix, d.features_delim)
        check(d.x_delim != d.feature_name_val_delim,
              "%sx_delim:%s must be different with %sfeature_name_val_delim:%s!", prefix, d.x_delim, prefix,
              d.feature_name_val_delim)
        check(d.features_delim != d.feature_name_val_delim,
              "%sfeatures_delim:%s must be different with %sfeature_name_val_delim:%s!", prefix, d.features_delim,
              prefix, d.feature_name_val_delim)
        return d


@dataclass
class DataParams:
    train_path: str = ""
    train_max_error_tol: int = 0
    test_path: str = ""
    test_max_error_tol: int = 0
    delim: Delim = field(default_factory=Delim)
    y_sampling: List[str] = field(default_factory=list)
    assigned: bool = False
    unassigned_mode: str = "lines_avg"
    max_feature_dim: int = -1  # gbdt only

    @classmethod
    def from_config(cls, c: Config, prefix: str = "", gbdt: bool = False) -> "DataParams":
        k = prefix + "data."
        p = cls()
        p.train_path = c.get_string(k + "train.data_path")
        p.train_max_error_tol = c.get_int(k + "train.max_error_tol")
        p.test_path = c.get_string(k + "test.data_path", "")
        if p.test_path == "???":
            p.test_path = ""
        p.test_max_error_tol = c.get_int(k + "test.max_error_tol", 0)
        p.delim = Delim.from_config(c, k + "delim.")
        p.y_sampling = c.get_string_list(k + "y_sampling", [])
        p.assigned = c.get_bool(k + "assigned", False)
        p.unassigned_mode = str(c.get_string(k + "unassigned_mode", "lines_avg")).lower()
        for s in p.y_sampling:
            check(re.fullmatch(r"\d+@(-?\d+)(\.\d+)?", s) is not None,
                  "%sy_sampling:%s must be the format of labelindex@rate. e.g 0@#0.1", k, s)
        check(p.unassigned_mode in ("files_avg", "lines_avg"),
              "unknown %sunassigned_mode:%s, only support:%s", k, p.unassigned_mode, ["files_avg", "lines_avg"])
        if gbdt:
            p.max_feature_dim = c.get_int(k + "max_feature_dim")
        return p

    def y_sampling_map(self) -> Dict[int, float]:
        out = {}
        for s in self.y_sampling:
            a, b = s.split("@")
            out[int(a)] = float(b)
        return out


@dataclass
class FeatureHashParams:
    need_feature_hash: bool = False
    bucket_size: int = 1000000
    seed: int = 39916801
    feature_prefix: str = "hash_"


@dataclass
class TransformParams:
    switch_on: bool = False
    mode: str = "standardization"
    scale_min: float = -1.0
    scale_max: float = 1.0
    include: Set[str] = field(default_factory=set)
    exclude: Set[str] = field(default_factory=set)


@dataclass
class FeatureParams:
    feature_hash: FeatureHashParams = field(default_factory=FeatureHashParams)
    transform: TransformParams = field(default_factory=TransformParams)
    filter_threshold: int = 0

    @classmethod
    def from_config(cls, c: Config, prefix: str = "") -> "FeatureParams":
        k = prefix + "feature."
        fh = FeatureHashParams(
            c.get_bool(k + "feature_hash.need_feature_hash", False),
            c.get_int(k + "feature_hash.bucket_size", 1000000),
            c.get_int(k + "feature_hash.seed", 39916801),
            c.get_string(k + "feature_hash.feature_prefix", "hash_"))
        tp = TransformParams(
            c.get_bool(k + "transform.switch_on", False),
            str(c.get_string(k + "transform.mode", "standardization")).lower(),
            c.get_double(k + "transform.scale_range.min", -1.0),
            c.get_double(k + "transform.scale_range.max", 1.0),
            set(c.get_string_list(k + "transform.include_features", [])),
            set(c.get_string_list(k + "transform.exclude_features", [])))
        if tp.switch_on:
            _mode(tp.mode, ("standardization", "scale_range"), k + "transform.mode")
        return cls(fh, tp, c.get_int(k + "filter_threshold", 0))


@dataclass
class ModelParams:
    data_path: str = ""
    delim: str = ","
    need_dict: bool = False
    dict_path: str = ""
    dump_freq: int = -1
    need_bias: bool = True
    bias_feature_name: str = "_bias_"
    continue_train: bool = False
    field_dict_path: str = ""           # ffm
    feature_importance_path: str = ""   # gbdt

    @classmethod
    def from_config(cls, c: Config, prefix: str = "", gbdt: bool = False) -> "ModelParams":
        k = prefix + "model."
        p = cls()
        p.data_path = c.get_string(k + "data_path")
        p.need_dict = c.get_bool(k + "need_dict")
        p.dict_path = c.get_string(k + "dict_path", "")
        p.dump_freq = c.get_int(k + "dump_freq", -1)
        p.continue_train = c.get_bool(k + "continue_train", False)
        if gbdt:
            p.feature_importance_path = c.get_string(k + "feature_importance_path", "")
            p.need_bias = False
        else:
            p.delim = c.get_string(k + "delim", ",")
            p.need_bias = c.get_bool(k + "need_bias", True)
            p.bias_feature_name = c.get_string(k + "bias_feature_name", "_bias_")
            p.field_dict_path = c.get_string(k + "field_dict_path", "")
        return p


def check_eval_names(names: List[str], key: str):
    for m in names:
        base = m.split("@")[0]
        check(base in EVAL_NAMES or any(m.startswith(e) for e in EVAL_NAMES),
              "%s:%s, only support:%s", key, m, list(EVAL_NAMES))


@dataclass
class LossParams:
    loss_function: str = "sigmoid"
    evaluate_metric: List[str] = field(default_factory=list)
    just_evaluate: bool = False
    l1: List[float] = field(default_factory=lambda: [0.0])
    l2: List[float] = field(default_factory=lambda: [0.0])

    @classmethod
    def from_config(cls, c: Config, prefix: str = "") -> "LossParams":
        k = prefix + "loss."
        p = cls(c.get_string(k + "loss_function"), c.get_string_list(k + "evaluate_metric", []),
                c.get_bool(k + "just_evaluate", False), c.get_double_list(k + "regularization.l1"),
                c.get_double_list(k + "regularization.l2"))
        check(len(p.l1) == len(p.l2), "%sregularization.l1 lenght must be equal to %sregularization.l2 lenght", k, k)
        check_eval_names(p.evaluate_metric, k + "evaluate_metric")
        return p


@dataclass
class LineSearchParams:
    mode: str = "wolfe"
    step_decr: float = 0.5
    step_incr: float = 2.1
    max_iter: int = 55
    min_step: float = 1e-16
    max_step: float = 1e18
    c1: float = 1e-4
    c2: float = 0.9
    m: int = 8
    lbfgs_max_iter: int = 60
    eps: float = 1e-3

    @classmethod
    def from_config(cls, c: Config, prefix: str = "optimization.") -> "LineSearchParams":
        k = prefix + "line_search."
        opt = c.get_string(prefix + "optimizer", "line_search")
        # "sgd" is this framework's extension (optim/sgd.py); ytk-learn only has line_search
        check(opt in ("line_search", "sgd"), "optimization.optimizer:%s, only support line_search or sgd", opt)
        if opt == "sgd" and not c.has(k.rstrip(".")):
            return cls()
        b = k + "backtracking."
        p = cls(mode=_mode(c.get_string(k + "mode"), ("sufficient_decrease", "wolfe", "strong_wolfe"), k + "mode"),
                step_decr=c.get_double(b + "step_decr"), step_incr=c.get_double(b + "step_incr"),
                max_iter=c.get_int(b + "max_iter"), min_step=c.get_double(b + "min_step"),
                max_step=c.get_double(b + "max_step"), c1=c.get_double(b + "c1"), c2=c.get_double(b + "c2"),
                m=c.get_int(k + "lbfgs.m"), lbfgs_max_iter=c.get_int(k + "lbfgs.convergence.max_iter"),
                eps=c.get_double(k + "lbfgs.convergence.eps"))
        check(p.step_decr < 1.0, "%sstep_decr:%f must < 1.0", b, p.step_decr)
        check(p.step_incr > 1.0, "%sstep_incr:%f must > 1.0", b, p.step_incr)
        check(0.0 < p.c1 < 1.0, "%sc1:%f must be in range(0, 1)", b, p.c1)
        check(p.c2 > p.c1 and p.c1 < 1.0, "%sc2:%f must be in range(c1, 1)", b, p.c2)
        check(p.m >= 1, "%slbfgs.m:%d must >= 1", k, p.m)
        return p


@dataclass
class HyperParams:
    switch_on: bool = False
    restart: bool = False
    mode: str = "hoag"
    init_step: float = 1.0
    step_decr_factor: float = 0.7
    test_loss_reduce_limit: float = 1e-5
    outer_iter: int = 10
    hoag_l1: List[float] = field(default_factory=list)
    hoag_l2: List[float] = field(default_factory=list)
    grid_l1: List[List[float]] = field(default_factory=list)  # per group [start, end, count]
    grid_l2: List[List[float]] = field(default_factory=list)

    @classmethod
    def from_config(cls, c: Config, prefix: str = "") -> "HyperParams":
        k = prefix + "hyper."
        if not c.has(k.rstrip(".")):
            return cls()
        p = cls(switch_on=c.get_bool(k + "switch_on", False), restart=c.get_bool(k + "restart", False),
                mode=_mode(c.get_string(k + "mode", "hoag"), ("hoag", "grid"), k + "mode"))
        h = k + "hoag."
        p.init_step = c.get_double(h + "init_step", 1.0)
        p.step_decr_factor = c.get_double(h + "step_decr_factor", 0.7)
        p.test_loss_reduce_limit = c.get_double(h + "test_loss_reduce_limit", 1e-5)
        p.outer_iter = c.get_int(h + "outer_iter", 10)
        p.hoag_l1 = c.get_double_list(h + "l1", [])
        p.hoag_l2 = c.get_double_list(h + "l2", [])
        check(p.step_decr_factor < 1.0, "%sstep_decr_factor:%f must < 1.0", h, p.step_decr_factor)
        check(len(p.hoag_l1) == len(p.hoag_l2), "%sl1 lenght must be equal to %sl2 lenght", h, h)
        g = k + "grid."
        l1 = c.get_double_list(g + "l1", [])
        l2 = c.get_double_list(g + "l2", [])
        check(len(l1) == len(l2), "%sl1 length must be equal to %sl2 length", g, g)
        check(len(l1) % 3 == 0, "%sl1 length must be 3 * regularization groups", g)
        p.grid_l1 = [l1[i:i + 3] for i in range(0, len(l1), 3)]
        p.grid_l2 = [l2[i:i + 3] for i in range(0, len(l2), 3)]
        return p


@dataclass
class RandomParams:
    mode: str = "normal"
    seed: int = 111111
    mean: float = 0.0
    std: float = 0.01
    range_start: float = -0.01
    range_end: float = 0.01

    @classmethod
    def from_config(cls, c: Config, prefix: str = "") -> "RandomParams":
        k = prefix + "random."
        return cls(mode=_mode(c.get_string(k + "mode"), ("normal", "uniform"), k + "mode"),
                   seed=c.get_int(k + "seed"), mean=c.get_double(k + "normal.mean"),
                   std=c.get_double(k + "normal.std"), range_start=c.get_double(k + "uniform.range_start"),
                   range_end=c.get_double(k + "uniform.range_end"))


# ---------------------------------------------------------------------------
@dataclass
class CommonParams:
    """Everything a continuous (L-BFGS) model needs (CommonParams.java:39-63)."""
    fs_scheme: str = "local"
    verbose: bool = False
    data: DataParams = field(default_factory=DataParams)
    feature: FeatureParams = field(default_factory=FeatureParams)
    model: ModelParams = field(default_factory=ModelParams)
    loss: LossParams = field(default_factory=LossParams)
    line_search: LineSearchParams = field(default_factory=LineSearchParams)
    hyper: HyperParams = field(default_factory=HyperParams)
    optimizer: str = "line_search"
    sgd: Optional[object] = None  # optim.sgd.SGDParams when optimizer == "sgd"
    random: Optional[RandomParams] = None
    extra: Dict[str, object] = field(default_factory=dict)  # model-specific keys (k, tree_num, ...)

    @classmethod
    def from_config(cls, c: Config, model_name: str = "linear") -> "CommonParams":
        p = cls()
        p.fs_scheme = c.get_string("fs_scheme", "local")
        p.verbose = c.get_bool("verbose", False)
        p.data = DataParams.from_config(c)
        p.feature = FeatureParams.from_config(c)
        p.model = ModelParams.from_config(c)
        p.loss = LossParams.from_config(c)
        p.line_search = LineSearchParams.from_config(c)
        p.optimizer = str(c.get_string("optimization.optimizer", "line_search")).lower()
        if p.optimizer == "sgd":
            from ..optim.sgd import SGDParams
            p.sgd = SGDParams.from_config(c)
        p.hyper = HyperParams.from_config(c)
        if c.has("random"):
            p.random = RandomParams.from_config(c)
        groups = len(p.loss.l2)
        if p.hyper.switch_on:
            if p.hyper.mode == "hoag":
                check(len(p.hyper.hoag_l2) == groups, "hyper.hoag.l2 length must equal loss.regularization.l2 length")
            else:
                check(len(p.hyper.grid_l2) == groups,
                      "hyper.grid.l2 length must be 3 * loss.regularization.l2 length")
        for key in ("k", "bias_need_latent_factor", "instance_sample_rate", "feature_sample_rate",
                    "uniform_base_prediction", "sample_dependent_base_prediction", "tree_num",
                    "learning_rate", "type", "leaf_random_init_range"):
            if c.has(key):
                p.extra[key] = c.get(key)
        return p


# ---------------------------------------------------------------------------
def gbdt_params_from_config(c: Config):
    """(GBDTParams, DataParams, ModelParams, extras) with the reference's derivations.

    GBDTOptimizationParams.java:108-238: min_split_loss default 1e-5 when missing,
    min_split_samples default -1, max_abs_leaf_val default -1, RF forces lr=1,
    data-parallel max_leaf_cnt = min(max_leaf_cnt, 2^max_depth), feature-parallel
    max_depth = 32 when max_leaf_cnt > 0 and max_depth < 0, class_num only for softmax.
    """
    from ..models.gbdt.builder import TreeParams
    from ..models.gbdt.trainer import GBDTParams

    k = "optimization."
    learn_type = str(c.get_string("type", "gradient_boosting")).lower()
    check(learn_type in ("gradient_boosting", "random_forest"), "[GBDT] learn type(%s) invalid", learn_type)
    round_num = c.get_int(k + "round_num")
    mcw = c.get_double(k + "min_child_hessian_sum")
    max_depth = c.get_int(k + "max_depth")
    max_leaf = c.get_int(k + "max_leaf_cnt")
    objective = c.get_string(k + "loss_function")
    min_split_loss = c.get_double(k + "min_split_loss", 1e-5)
    min_split_samples = c.get_int(k + "min_split_samples", -1)
    max_abs_leaf = c.get_double(k + "max_abs_leaf_val", -1.0)
    l1 = c.get_double(k + "regularization.l1")
    l2 = c.get_double(k + "regularization.l2")
    lr = c.get_double(k + "regularization.learning_rate")
    if learn_type == "random_forest":
        lr = 1.0
    maker = str(c.get_string(k + "tree_maker", "data")).lower()
    check(maker in ("data", "feature"), "[GBDT] tree maker type(%s) invalid, data or feature", maker)
    hist_pool = -1.0
    if maker == "data":
        policy = str(c.get_string(k + "tree_grow_policy")).lower()
        check(policy in ("level", "loss"), "[GBDT] tree_grow_policy (%s) invalid, loss or level", policy)
        if max_depth > 0:
            max_leaf = (1 << max_depth) if max_leaf < 0 else min(max_leaf, 1 << max_depth)
        hist_pool = c.get_double(k + "histogram_pool_capacity", -1.0)
    else:
        policy = "level"
        if max_leaf > 0 and max_depth < 0:
            max_depth = 32
    base = c.get_double(k + "uniform_base_prediction")
    class_num = c.get_int(k + "class_num") if objective.startswith("softmax") else 1
    zmax = c.get_double(k + "sigmoid_zmax", 0.0) if objective.lower() == "sigmoid" else 0.0
    lad_appr = c.get_bool(k + "lad_refine_appr", True) if objective.lower() == "l1" else True
    verbose = c.get_bool(k + "verbose", c.get_bool("verbose", False))
    tp = TreeParams(max_depth=max_depth, max_leaf_cnt=max_leaf, min_child_hessian_sum=mcw,
                    max_abs_leaf_val=max_abs_leaf, min_split_loss=min_split_loss,
                    min_split_samples=min_split_samples, learning_rate=lr, l1=l1, l2=l2, grow_policy=policy,
                    instance_sample_rate=c.get_double(k + "instance_sample_rate"),
                    feature_sample_rate=c.get_double(k + "feature_sample_rate"),
                    seed=c.get_int(k + "seed", 2018),
                    hist_sync=str(c.get_string(k + "hist_sync", "auto")).lower())
    check(tp.hist_sync in ("auto", "allreduce", "owner"), "[GBDT] hist_sync (%s) invalid: auto, allreduce or owner",
          tp.hist_sync)
    f = "feature."
    approx = c.get_list(f + "approximate", [{"cols": "default", "type": "no_sample"}])
    gp = GBDTParams(round_num=round_num, loss_function=objective, class_num=class_num, type=learn_type,
                    uniform_base_prediction=base,
                    sample_dependent_base_prediction=c.get_bool(k + "sample_dependent_base_prediction"),
                    sigmoid_zmax=zmax, lad_refine_appr=lad_appr, eval_metric=c.get_string_list(k + "eval_metric"),
                    watch_train=c.get_bool(k + "watch_train"), watch_test=c.get_bool(k + "watch_test"),
                    split_type=str(c.get_string(f + "split_type", "mean")).lower(),
                    missing_value=c.get_string(f + "missing_value", "value"), approximate=approx,
                    dump_freq=c.get_int("model.dump_freq", -1), verbose=verbose, tree=tp)
    gp.tree_maker = maker
    gp.histogram_pool_capacity = hist_pool
    gp.just_evaluate = c.get_bool(k + "just_evaluate", False)
    gp.filter_threshold = c.get_int(f + "filter_threshold", 0)
    # checkParams (GBDTOptimizationParams.java:208-238)
    check(round_num >= 1, "[GBDT] round_num(%d) should >=1", round_num)
    check(class_num >= 1, "[GBDT] class_num(%d) should >= 1", class_num)
    check(min_split_loss >= 0, "[GBDT] min_split_loss(%f) should >= 0", min_split_loss)
    check(min_split_samples >= 2 or min_split_samples < 0, "[GBDT] min_split_samples(%d) should >=2 or < 0",
          min_split_samples)
    check(max_leaf != 0, "[GBDT] max_leaf_cnt(%d) should not be 0", max_leaf)
    check(not (max_leaf < 0 and max_depth < 0),
          "[GBDT] max_leaf_cnt(%d) and max_depth(%d) should not be both negative", max_leaf, max_depth)
    check(not (objective == "sigmoid" and not (0.0 < base < 1.0)),
          "[GBDT] uniform_base_prediction(%f) for sigmoid should between (0, 1)", base)
    check(0.0 < tp.instance_sample_rate <= 1.0, "instance_sample_rate(%f) should belong to (0, 1]",
          tp.instance_sample_rate)
    check(0.0 < tp.feature_sample_rate <= 1.0, "feature_sample_rate(%f) should belong to (0, 1]",
          tp.feature_sample_rate)
    check(zmax >= 0.0, "sigmoid_zmax(%f) for sigmoid should >=0, recommend [2, 4]", zmax)
    for m in gp.eval_metric:
        check(m.split("@")[0] in EVAL_NAMES, "[GBDT] eval name %s invalid", m.split("@")[0])
    data = DataParams.from_config(c, gbdt=True)
    model = ModelParams.from_config(c, gbdt=True)
    return gp, data, model
