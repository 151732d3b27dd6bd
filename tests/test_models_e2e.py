"""End-to-end training of every model family through the HOCON configs and the CLI-facing
``train()`` API, on synthetic ytk-format files (and the reference demo data when present).

Parity anchors: the reference's demo README for GBDT binary classification publishes
train/test losses for rounds 2 and 3 (demo/gbdt/binary_classification/README.md:42-49);
``test_gbdt_demo_matches_reference_readme`` reproduces them.
"""
import os

import numpy as np
import pytest
import torch

from ytk_learn_amd.config.hocon import parse_file
from ytk_learn_amd.parallel.comm import Comm
from ytk_learn_amd.train import train

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONF = os.path.join(ROOT, "config", "model")
REF = "/root/reference"


def write_binary(path, n, F=40, seed=0, fields=False, label_noise=0.05):
    w = np.random.default_rng(1234).normal(size=F)  # same ground truth for train and test
    g = np.random.default_rng(seed)
    lines = []
    for _ in range(n):
        k = int(g.integers(3, 9))
        idx = np.unique(g.integers(0, F, size=k))
        val = g.random(len(idx)) * 2.0
        z = float((w[idx] * val).sum())
        y = int(z > 0) if g.random() > label_noise else int(z <= 0)
        names = [f"f{i % 5}@x{i}" if fields else f"x{i}" for i in idx]
        lines.append("1###%d###%s" % (y, ",".join(f"{nm}:{v:.4f}" for nm, v in zip(names, val))))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def write_multiclass(path, n, K=4, F=20, seed=0):
    W = np.random.default_rng(4321).normal(size=(F, K))
    g = np.random.default_rng(seed)
    lines = []
    for _ in range(n):
        x = g.random(F)
        y = int(np.argmax(x @ W + 0.1 * g.normal(size=K)))
        lines.append("1###%d###%s" % (y, ",".join(f"{i}:{x[i]:.4f}" for i in range(F))))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def _cfg(model, tmp, train_path, test_path, **kw):
    c = parse_file(os.path.join(CONF, f"{model}.conf"))
    ov = {"data.train.data_path": train_path, "data.test.data_path": test_path,
          "model.data_path": os.path.join(tmp, f"{model}.model")}
    ov.update(kw)
    return c.with_overrides(ov)


def _local(dev="cpu"):
    return Comm.local(dev)


@pytest.fixture(scope="module")
def bin_data(tmp_path_factory):
    d = tmp_path_factory.mktemp("bin")
    write_binary(str(d / "train.txt"), 3000, seed=1)
    write_binary(str(d / "test.txt"), 800, seed=2)
    write_binary(str(d / "ftrain.txt"), 3000, seed=3, fields=True)
    write_binary(str(d / "ftest.txt"), 500, seed=4, fields=True)
    with open(d / "fields.dict", "w") as f:
        f.write("\n".join(f"f{i}" for i in range(5)) + "\n")
    return d


@pytest.mark.parametrize("model,kw", [
    ("linear", {}),
    ("fm", {"k": [1, 4]}),
    ("gbmlr", {"k": 4, "tree_num": 2}),
    ("gbsdt", {"k": 4, "tree_num": 2}),
    ("gbhmlr", {"k": 4, "tree_num": 2}),
    ("gbhsdt", {"k": 4, "tree_num": 2}),
])
def test_continuous_models_learn(bin_data, tmp_path, model, kw):
    cfg = _cfg(model, str(tmp_path), str(bin_data / "train.txt"), str(bin_data / "test.txt"),
               **{"optimization.line_search.lbfgs.convergence.max_iter": 30}, **kw)
    res = train(model, cfg, comm=_local())
    assert res.test_loss is not None
    # weighted avg test log-loss clearly below the 0.693 of a constant predictor (the
    # mixtures overfit 3000 rows a little, hence the looser bound)
    assert res.test_loss / 800 < (0.45 if model in ("linear", "fm") else 0.62), res
    files = os.listdir(tmp_path / f"{model}.model")
    assert files, "model was not dumped"


def test_ffm_learns(bin_data, tmp_path):
    cfg = _cfg("ffm", str(tmp_path), str(bin_data / "ftrain.txt"), str(bin_data / "ftest.txt"),
               **{"model.field_dict_path": str(bin_data / "fields.dict"), "k": [1, 2],
                  "optimization.line_search.lbfgs.convergence.max_iter": 15})
    res = train("ffm", cfg, comm=_local())
    assert res.test_loss / 500 < 0.6, res


def test_multiclass_linear_learns(tmp_path):
    write_multiclass(str(tmp_path / "tr.txt"), 2000, seed=1)
    write_multiclass(str(tmp_path / "te.txt"), 500, seed=2)
    cfg = _cfg("multiclass_linear", str(tmp_path), str(tmp_path / "tr.txt"), str(tmp_path / "te.txt"), k=4)
    res = train("multiclass_linear", cfg, comm=_local())
    assert res.test_loss / 500 < 0.8


def test_linear_continue_train_and_predict(bin_data, tmp_path):
    from ytk_learn_amd.predict.predictor import create_predictor
    cfg = _cfg("linear", str(tmp_path), str(bin_data / "train.txt"), str(bin_data / "test.txt"),
               **{"optimization.line_search.lbfgs.convergence.max_iter": 5})
    r1 = train("linear", cfg, comm=_local())
    r2 = train("linear", cfg.with_value("model.continue_train", True), comm=_local())
    assert r2.loss <= r1.loss * 1.0001
    p = create_predictor("linear", cfg)
    data = tmp_path / "pred.txt"
    data.write_text(open(bin_data / "test.txt").read())
    loss = p.batch_predict_from_files(str(data), None, "LABEL_AND_PREDICT", None, 10, "auc", "value")
    np.testing.assert_allclose(loss * 800, r2.test_loss, rtol=1e-4)
    out = open(str(data) + "_linear_LABEL_AND_PREDICT").read().splitlines()
    assert len(out) == 800 and "###" in out[0]


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "demo/data/libsvm/agaricus.train.libsvm")),
                    reason="reference demo data not available")
def test_gbdt_demo_matches_reference_readme(tmp_path):
    """demo/gbdt/binary_classification: loss-wise, 3 rounds, sigmoid on agaricus (libsvm converted)."""
    from ytk_learn_amd.tools.libsvm_convert import convert
    for part in ("train", "test"):
        convert("binary_classification@0,1", "###", ",", ",", ":", "local",
                os.path.join(REF, f"demo/data/libsvm/agaricus.{part}.libsvm"), str(tmp_path / f"{part}.ytk"),
                log=lambda *_: None)
    cfg = parse_file(os.path.join(REF, "demo/gbdt/binary_classification/local_gbdt.conf")).with_overrides({
        "data.train.data_path": str(tmp_path / "train.ytk"), "data.test.data_path": str(tmp_path / "test.ytk"),
        "model.data_path": str(tmp_path / "gbdt.model"), "model.feature_importance_path": str(tmp_path / "fi")})
    losses = []

    class Log:
        verbose = False

        def info(self, msg, all_ranks=False):
            for line in msg.splitlines():
                if line.startswith("train loss = ") or line.startswith("test loss = "):
                    losses.append(float(line.split("=")[1]))

        def enabled_for_round(self, i):
            return True

        def error(self, msg):
            pass

    train("gbdt", cfg, comm=_local(), log=Log())
    # README: iter 2: train 0.17249267375913763 test 0.17219528385526198; iter 3: 0.09960066518065772 / 0.09943817574378232
    np.testing.assert_allclose(losses[2:6], [0.17249267375913763, 0.17219528385526198, 0.09960066518065772,
                                             0.09943817574378232], rtol=1e-12)
    txt = open(tmp_path / "gbdt.model").read()
    assert txt.startswith("uniform_base_prediction=0.5\nclass_num=1\nloss_function=sigmoid\ntree_num=3\n")


def test_gbdt_multiclass_and_feature_maker(tmp_path):
    write_multiclass(str(tmp_path / "tr.txt"), 1500, K=3, F=10, seed=5)
    write_multiclass(str(tmp_path / "te.txt"), 300, K=3, F=10, seed=6)
    cfg = parse_file(os.path.join(CONF, "gbdt.conf")).with_overrides({
        "data.train.data_path": str(tmp_path / "tr.txt"), "data.test.data_path": str(tmp_path / "te.txt"),
        "data.max_feature_dim": 10, "model.data_path": str(tmp_path / "m"), "optimization.round_num": 8,
        "optimization.loss_function": "softmax", "optimization.class_num": 3, "optimization.max_depth": 4,
        "optimization.eval_metric": ["confusion_matrix"]})
    tr = train("gbdt", cfg, comm=_local())
    assert tr.last_test_loss < 0.9
    cfg2 = cfg.with_overrides({"optimization.tree_maker": "feature", "optimization.round_num": 3,
                               "model.data_path": str(tmp_path / "m2")})
    tr2 = train("gbdt", cfg2, comm=_local())
    assert tr2.last_test_loss < 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("model,kw", [("linear", {}), ("fm", {"k": [1, 4]}), ("gbmlr", {"k": 4}),
                                      ("gbhsdt", {"k": 4}), ("gbmlr", {"k": 80}), ("gbhsdt", {"k": 70})])
def test_continuous_models_gpu_match_cpu(cuda, bin_data, tmp_path, model, kw):
    kw = dict(kw, **{"optimization.line_search.lbfgs.convergence.max_iter": 8})
    rc = train(model, _cfg(model, str(tmp_path / "c"), str(bin_data / "train.txt"), str(bin_data / "test.txt"),
                           **kw), comm=_local("cpu"))
    rg = train(model, _cfg(model, str(tmp_path / "g"), str(bin_data / "train.txt"), str(bin_data / "test.txt"),
                           **kw), comm=_local(cuda))
    np.testing.assert_allclose(rg.loss, rc.loss, rtol=2e-3)
    np.testing.assert_allclose(rg.test_loss, rc.test_loss, rtol=5e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("loss", ["softmax", "multiclass_hinge", "hsoftmax"])
def test_multiclass_linear_gpu_matches_cpu(cuda, tmp_path, loss):
    """The fused multiclass epilogue (mc_row_loss_kernel) inside L-BFGS training reaches the CPU
    (fp64 torch) run's losses."""
    write_multiclass(str(tmp_path / "tr.txt"), 2000, seed=1)
    write_multiclass(str(tmp_path / "te.txt"), 500, seed=2)
    kw = {"k": 4, "loss.loss_function": loss, "optimization.line_search.lbfgs.convergence.max_iter": 8}
    rc = train("multiclass_linear", _cfg("multiclass_linear", str(tmp_path / "c"), str(tmp_path / "tr.txt"),
                                         str(tmp_path / "te.txt"), **kw), comm=_local("cpu"))
    rg = train("multiclass_linear", _cfg("multiclass_linear", str(tmp_path / "g"), str(tmp_path / "tr.txt"),
                                         str(tmp_path / "te.txt"), **kw), comm=_local(cuda))
    np.testing.assert_allclose(rg.loss, rc.loss, rtol=2e-3)
    np.testing.assert_allclose(rg.test_loss, rc.test_loss, rtol=5e-3)


@pytest.mark.gpu
def test_ffm_gpu_matches_cpu_training(cuda, bin_data, tmp_path):
    kw = {"model.field_dict_path": str(bin_data / "fields.dict"), "k": [1, 4],
          "optimization.line_search.lbfgs.convergence.max_iter": 5}
    rc = train("ffm", _cfg("ffm", str(tmp_path / "c"), str(bin_data / "ftrain.txt"), str(bin_data / "ftest.txt"),
                           **kw), comm=_local("cpu"))
    rg = train("ffm", _cfg("ffm", str(tmp_path / "g"), str(bin_data / "ftrain.txt"), str(bin_data / "ftest.txt"),
                           **kw), comm=_local(cuda))
    np.testing.assert_allclose(rg.loss, rc.loss, rtol=5e-3)


def _sgd_kw(**kw):
    base = {"optimization.optimizer": "sgd", "optimization.sgd.learning_rate": 0.05,
            "optimization.sgd.batch_size": 64, "optimization.sgd.epochs": 6, "optimization.sgd.seed": 3}
    base.update(kw)
    return base


@pytest.mark.parametrize("model", ["linear", "fm", "ffm"])
def test_sgd_optimizer_learns(bin_data, tmp_path, model):
    """optimization.optimizer = sgd (extension): mini-batch Hogwild!-style SGD reaches a
    test loss well below the constant predictor's log(2) and writes the usual model files."""
    tr, te = ("ftrain.txt", "ftest.txt") if model == "ffm" else ("train.txt", "test.txt")
    kw = _sgd_kw()
    if model == "ffm":
        kw.update({"model.field_dict_path": str(bin_data / "fields.dict"), "k": [1, 2]})
    if model == "fm":
        kw["k"] = [1, 4]
    cfg = _cfg(model, str(tmp_path), str(bin_data / tr), str(bin_data / te), **kw)
    train_loss, test_loss = train(model, cfg, comm=_local())
    assert test_loss < 0.55 and train_loss < 0.55, (train_loss, test_loss)
    assert os.path.exists(os.path.join(str(tmp_path), f"{model}.model", "model-00000"))


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["linear", "fm", "ffm"])
def test_sgd_optimizer_gpu(cuda, bin_data, tmp_path, model):
    """The HIP Hogwild!-style update learns like the CPU mini-batch step (races differ)."""
    tr, te = ("ftrain.txt", "ftest.txt") if model == "ffm" else ("train.txt", "test.txt")
    kw = _sgd_kw()
    if model == "ffm":
        kw.update({"model.field_dict_path": str(bin_data / "fields.dict"), "k": [1, 2]})
    if model == "fm":
        kw["k"] = [1, 4]
    rc = train(model, _cfg(model, str(tmp_path / "c"), str(bin_data / tr), str(bin_data / te), **kw),
               comm=_local("cpu"))
    rg = train(model, _cfg(model, str(tmp_path / "g"), str(bin_data / tr), str(bin_data / te), **kw),
               comm=_local(cuda))
    assert rg[1] < 0.55
    assert abs(rg[1] - rc[1]) < 0.05, (rg, rc)


@pytest.mark.parametrize("model", ["linear", "fm", "ffm"])
@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_sgd_large_batch_per_feature_average(bin_data, tmp_path, model, dev):
    """Batches of 1024 rows (every row holds the bias and a few hot features): with
    optimization.sgd.average = feature each weight takes the mean step of the rows holding
    its feature and training converges; the summed per-sample steps (average = none) of
    the same run are ~1024x larger on the bias and diverge -- the NaN / 5e11 training losses
    of the round-1 Criteo-shape SGD benches."""
    import math

    import torch
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    tr, te = ("ftrain.txt", "ftest.txt") if model == "ffm" else ("train.txt", "test.txt")
    res = {}
    for avg in ("feature", "none"):
        kw = _sgd_kw(**{"optimization.sgd.batch_size": 1024, "optimization.sgd.learning_rate": 0.5,
                        "optimization.sgd.epochs": 8, "optimization.sgd.average": avg})
        if model == "ffm":
            kw.update({"model.field_dict_path": str(bin_data / "fields.dict"), "k": [1, 2]})
        if model == "fm":
            kw["k"] = [1, 4]
        res[avg] = train(model, _cfg(model, str(tmp_path / avg), str(bin_data / tr), str(bin_data / te), **kw),
                         comm=_local(dev))
    assert res["feature"][1] < 0.6 and res["feature"][0] < 0.6, res
    assert not (math.isfinite(res["none"][1]) and res["none"][1] < 0.6), res


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_fm_sgd_bf16_matches_fp32(bin_data, tmp_path, dev):
    """optimization.sgd.dtype = bf16 (bf16 working copy of the FM latents, fp32 master):
    the training run reaches the fp32 run's test loss within tolerance."""
    import torch
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    kw = _sgd_kw()
    kw["k"] = [1, 8]
    res = {}
    for dt in ("fp32", "bf16"):
        kw["optimization.sgd.dtype"] = dt
        res[dt] = train("fm", _cfg("fm", str(tmp_path / dt), str(bin_data / "train.txt"), str(bin_data / "test.txt"),
                                   **kw), comm=_local(dev))
    assert res["bf16"][1] < 0.55
    assert abs(res["bf16"][1] - res["fp32"][1]) < 0.02, res


def _agaricus_ytk(tmp_path):
    """The reference demo's agaricus libsvm files (bundled gzip copies, public dataset)
    converted to the ytk format with the LibSVM tool."""
    import gzip

    from ytk_learn_amd.tools.libsvm_convert import convert
    data = os.path.join(ROOT, "tests", "data")
    out = {}
    for part in ("train", "test"):
        raw = tmp_path / f"agaricus.{part}.libsvm"
        raw.write_bytes(gzip.decompress(open(os.path.join(data, f"agaricus.{part}.libsvm.gz"), "rb").read()))
        out[part] = tmp_path / f"{part}.ytk"
        convert("binary_classification@0,1", "###", ",", ",", ":", "local", str(raw), str(out[part]),
                log=lambda *_: None)
    return out


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_gbdt_demo_readme_losses_on_device(tmp_path, dev):
    """demo/gbdt/binary_classification (loss-wise, 3 rounds, sigmoid) through this repo's
    demo config: the reference README's per-round losses to 1e-12 -- on the CPU path and on
    the HIP path (exact int64 histograms make the GPU trees identical)."""
    import torch
    if dev == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = _agaricus_ytk(tmp_path)
    cfg = parse_file(os.path.join(ROOT, "demo", "gbdt", "binary_classification", "gbdt.conf")).with_overrides({
        "data.train.data_path": str(d["train"]), "data.test.data_path": str(d["test"]),
        "model.data_path": str(tmp_path / "gbdt.model"), "model.feature_importance_path": str(tmp_path / "fi")})
    losses = []

    class Log:
        verbose = False

        def info(self, msg, all_ranks=False):
            for line in msg.splitlines():
                if line.startswith("train loss = ") or line.startswith("test loss = "):
                    losses.append(float(line.split("=")[1]))

        def enabled_for_round(self, i):
            return True

        def error(self, msg):
            pass

    tr = train("gbdt", cfg, comm=_local(dev), log=Log())
    assert tr.bins.device.type == dev
    # README (demo/gbdt/binary_classification/README.md:42-58): iter 2 and iter 3
    np.testing.assert_allclose(losses[2:6], [0.17249267375913763, 0.17219528385526198, 0.09960066518065772,
                                             0.09943817574378232], rtol=1e-12)
