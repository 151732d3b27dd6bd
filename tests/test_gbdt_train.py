import os

import numpy as np
import pytest
import torch

from ytk_learn_amd.data.synthetic import higgs_like
from ytk_learn_amd.models.gbdt.builder import TreeParams
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer
from ytk_learn_amd.models.gbdt.tree import GBDTModel
from ytk_learn_amd.ops import gbdt as gops


def _data(n, seed, dev="cpu"):
    X, y = higgs_like(n, seed=seed, device=dev)
    return GBDTData(X, y)


def _params(policy, rounds=4, **kw):
    tp = TreeParams(max_depth=5 if policy == "level" else -1, max_leaf_cnt=24 if policy == "loss" else 32,
                    min_child_hessian_sum=5.0, grow_policy=policy, learning_rate=0.2, **kw)
    return GBDTParams(round_num=rounds, tree=tp, watch_test=True)


@pytest.mark.parametrize("policy", ["level", "loss"])
def test_train_cpu_loss_decreases(policy):
    tr = GBDTTrainer(_params(policy), _data(20000, 1), _data(4000, 2))
    tr.prepare()
    losses = []
    tr.init_gradients()
    for i in range(4):
        tr.step(i)
        losses.append(tr.last_train_loss)
    assert all(b < a for a, b in zip(losses, losses[1:]))
    t = tr.model.trees[0]
    assert t.leaf_count() <= (32 if policy == "level" else 24)
    if policy == "level":
        assert t.max_depth() <= 5


def test_model_roundtrip_and_forest_matches_training_scores():
    tr = GBDTTrainer(_params("level", rounds=3), _data(8000, 3), None)
    m = tr.train()
    text = m.dumps()
    m2 = GBDTModel.loads(text)
    assert m2.dumps() == text
    name2idx = {n: i for i, n in enumerate(tr.feature_names)}
    for t in m2.trees:
        t.update_feature_index(name2idx)
    fl = {k: torch.from_numpy(v) for k, v in m2.flatten().items()}
    out = torch.zeros((8000, 1))
    X = torch.where(torch.isnan(tr.train_data.X), 0.0, tr.train_data.X)
    gops.forest_predict(X, fl, out, 1.0)
    # raw-threshold inference reproduces the bin-threshold training scores
    torch.testing.assert_close(out, tr.score, rtol=1e-5, atol=1e-5)


def test_subsample_and_feature_sample_cpu():
    p = _params("level", rounds=2, instance_sample_rate=0.5, feature_sample_rate=0.5)
    tr = GBDTTrainer(p, _data(10000, 4), None)
    tr.train()
    used = {tr.model.trees[0].feat[i] for i in range(tr.model.trees[0].num_nodes) if not tr.model.trees[0].is_leaf[i]}
    assert len(used) <= 14
    assert tr.model.trees[0].sample_cnt[0] < 6000


@pytest.mark.parametrize("loss,K", [("l2", 1), ("l1", 1), ("softmax", 3), ("poisson", 1)])
def test_other_losses_cpu(loss, K):
    X, y = higgs_like(6000, seed=5)
    if loss == "softmax":
        c = torch.clamp((X[:, 25] * 1.5).long(), 0, K - 1)
        y = torch.nn.functional.one_hot(c, K).float()
    elif loss == "poisson":
        y = torch.poisson(torch.exp(0.3 * X[:, 25:26]))
    else:
        y = X[:, 25:26] * 2.0 + 0.1 * torch.randn(6000, 1)
    p = _params("level", rounds=3)
    p.loss_function = loss
    p.class_num = K
    p.uniform_base_prediction = 1.0 if loss == "poisson" else (0.0 if loss != "softmax" else 0.0)
    p.eval_metric = ["confusion_matrix"] if loss == "softmax" else ["rmse", "mae"]
    tr = GBDTTrainer(p, GBDTData(X, y), GBDTData(X[:1000], y[:1000]))
    tr.prepare()
    tr.init_gradients()
    l0 = None
    for i in range(3):
        tr.step(i)
        l0 = tr.last_train_loss if l0 is None else l0
    assert tr.last_train_loss < l0 or loss == "l1"
    assert len(tr.model.trees) == 3 * K
    tr.final_eval()


def test_random_forest_cpu():
    p = _params("level", rounds=3)
    p.type = "random_forest"
    tr = GBDTTrainer(p, _data(6000, 6), None)
    tr.train()
    assert np.isfinite(tr.last_train_loss)


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["level", "loss"])
def test_train_gpu_matches_cpu(cuda, policy):
    d_cpu = _data(30000, 7)
    d_gpu = GBDTData(d_cpu.X.to(cuda), d_cpu.y.to(cuda))
    t_cpu = GBDTTrainer(_params(policy, rounds=3), d_cpu, None)
    t_gpu = GBDTTrainer(_params(policy, rounds=3), d_gpu, None)
    t_cpu.train()
    t_gpu.train()
    assert t_gpu.bins.is_cuda
    np.testing.assert_allclose(t_gpu.last_train_loss, t_cpu.last_train_loss, rtol=2e-4)
    # first tree: identical structure (ties aside)
    a, b = t_cpu.model.trees[0], t_gpu.model.trees[0]
    assert a.feat[0] == b.feat[0] and a.slot_a[0] == b.slot_a[0]
    assert a.num_nodes == b.num_nodes


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, {"max_leaf_cnt": 11}, {"min_split_samples": 3000}, {"l2": 1.0, "l1": 0.5},
                                {"split_type": "median"}, {"feature_sample_rate": 0.6},
                                {"instance_sample_rate": 0.7, "feature_sample_rate": 0.5, "split_type": "median"},
                                {"max_cnt": 300, "feature_sample_rate": 0.6},
                                {"max_depth": 14, "max_leaf_cnt": 200}, {"max_depth": 16, "max_leaf_cnt": 1000},
                                {"max_depth": 14, "max_leaf_cnt": 300, "instance_sample_rate": 0.8}])
def test_device_builder_matches_host_builder(cuda, kw):
    """GPU-resident level builder == host-driven builder (integer histograms => identical trees),
    including median split values, feature / instance sampling, > 256 (uint16) bins and
    max_depth 14 / 16 under a leaf budget (per-level slots and arrays sized by the level width
    min(2^depth, leaves); these configurations ran on the host builder before)."""
    d = _data(40000, 9, cuda)
    trees = []
    special = ("max_leaf_cnt", "split_type", "max_cnt", "max_depth")
    for dev_builder in (False, True):
        p = _params("level", rounds=3, **{k: v for k, v in kw.items() if k not in special})
        if "max_depth" in kw:
            p.tree.max_depth = kw["max_depth"]
            p.tree.min_child_hessian_sum = 1.0
        if "max_leaf_cnt" in kw:
            p.tree.max_leaf_cnt = kw["max_leaf_cnt"]
        if "split_type" in kw:
            p.split_type = kw["split_type"]
        if "max_cnt" in kw:
            p.approximate = [{"cols": "default", "type": "sample_by_quantile", "max_cnt": kw["max_cnt"]}]
        p.device_builder = dev_builder
        tr = GBDTTrainer(p, d, _data(5000, 10, cuda))
        tr.train()
        assert tr.use_device_builder == dev_builder
        trees.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert trees[0][0] == trees[1][0]
    assert trees[0][1] == trees[1][1] and trees[0][2] == trees[1][2]



@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"YTK_PART_CHUNK": "4096"}, {"YTK_PART_CHUNK": "1024"}, {"YTK_FUSE_SPLIT_PLAN": "1"}, {"YTK_PART_PREFETCH": "0"}, {"YTK_PART_PREFETCH": "1"}, {"YTK_PART_PREFETCH": "2"},
                                 {"YTK_SPLIT_GROUPS": "1"}, {"YTK_SPLIT_GROUPS": "3"}, {"YTK_REDUCE_SPLIT": "8"},
                                 {"YTK_FUSED_TEST_TAIL": "0"}, {"YTK_TG_LDS_WALK": "0"}, {"YTK_FUSE_ROOT_HIST": "0"},
                                 {"YTK_FUSE_ROOT_HIST": "0", "YTK_DEFER_LEAF_COUNTS": "0"},
                                 {"YTK_PART_CHUNK": "4096", "YTK_FUSE_SPLIT_PLAN": "1"},
                                 {"YTK_FUSE_REDUCE_SPLIT": "1"}, {"YTK_FUSE_REDUCE_SPLIT": "1", "YTK_REDUCE_SPLIT": "1"},
                                 {"YTK_FUSE_REDUCE_SPLIT": "1", "YTK_REDUCE_SPLIT": "3"},
                                 {"YTK_FUSE_REDUCE_SPLIT": "1", "YTK_RS_GROUP": "8"},
                                 {"YTK_FUSE_REDUCE_SPLIT": "1", "YTK_RS_GROUP": "2"}, {"YTK_PLAN_FAST": "0"},
                                 {"YTK_PART_SCAN_MIN_ROWS": "0"}, {"YTK_PART_SCAN_LEVELS": "3", "YTK_PART_SCAN_MIN_ROWS": "0"},
                                 {"YTK_PART_SCAN_LEVELS": "8", "YTK_PART_SCAN_MIN_ROWS": "0"},
                                 {"YTK_PART_SCAN_LEVELS": "2", "YTK_PART_PREFETCH": "2", "YTK_PART_SCAN_MIN_ROWS": "0"},
                                 {"YTK_PART_SCAN_MIN_ROWS": "0", "YTK_PART_SCAN_KERNEL": "1"}])
def test_device_builder_kernel_variants_identical(cuda, monkeypatch, env):
    """Level-engine kernel variants (16-row-per-thread partition chunks; split search fused
    with the next level's planning) build the default engine's trees byte for byte."""
    d = _data(40000, 9, cuda)
    out = []
    for use_env in (False, True):
        for k, v in env.items():
            if use_env:
                monkeypatch.setenv(k, v)
            else:
                monkeypatch.delenv(k, raising=False)
        p = _params("level", rounds=3, feature_sample_rate=0.7)
        p.device_builder = True
        tr = GBDTTrainer(p, d, _data(5000, 10, cuda))
        tr.train()
        assert tr.use_device_builder
        out.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert out[0] == out[1]


@pytest.mark.parametrize("kw", [{}, {"max_leaf_cnt": 7}, {"max_depth": 4, "max_leaf_cnt": 20},
                                {"min_split_samples": 900}, {"min_split_loss": 2.0},
                                {"instance_sample_rate": 0.7, "feature_sample_rate": 0.6}])
def test_loss_guided_speculation_is_exact(monkeypatch, kw):
    """Speculative batched leaf-wise growth == one-leaf-at-a-time growth (node ids, splits,
    values and node statistics), on CPU."""
    dumps = []
    for spec in ("0", "1"):
        monkeypatch.setenv("YTK_LOSSGUIDE_SPEC", spec)
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 40
        for k, v in kw.items():
            setattr(p.tree, k, v)
        tr = GBDTTrainer(p, _data(12000, 11), _data(3000, 12))
        tr.train()
        dumps.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert dumps[0] == dumps[1]
    assert dumps[0][0].count("leaf=") > 3


@pytest.mark.parametrize("kw", [{}, {"max_depth": 4, "max_leaf_cnt": 20}, {"min_split_samples": 900},
                                {"min_split_loss": 2.0}, {"l1": 0.5, "max_abs_leaf_val": 0.3},
                                {"instance_sample_rate": 0.7, "feature_sample_rate": 0.6}, {"pool": 5},
                                {"spec": "0"}])
def test_native_leafwise_planner_matches_python(monkeypatch, kw):
    """The native leaf-wise planner (csrc/native/leafwise.cpp) == the Python reference
    planner (TreeBuilder._grow_loss_guided): model dump, losses, batches, pool misses."""
    kw = dict(kw)
    pool = kw.pop("pool", None)
    monkeypatch.setenv("YTK_LOSSGUIDE_SPEC", kw.pop("spec", "1"))
    res = []
    for native in ("0", "1"):
        monkeypatch.setenv("YTK_LEAF_NATIVE", native)
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 40
        for k, v in kw.items():
            setattr(p.tree, k, v)
        if pool is not None:
            p.histogram_pool_capacity = pool * 256 * 28 * 16 / float(1 << 20)  # ~pool live slots
        tr = GBDTTrainer(p, _data(12000, 11), _data(3000, 12))
        tr.train()
        assert tr.builder.native_leafwise == (native == "1")
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss, tr.builder.last_batches,
                    tr.builder.last_expanded, tr.builder.hist_miss))
    assert res[0] == res[1]
    if pool is not None:
        assert res[0][5] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plain", "pool", "depth"])
def test_native_leafwise_gpu_paths_match_python(monkeypatch, mode):
    """GPU: native planner with the lean launch path == native planner through the generic
    helpers == Python planner (exact int64 histograms => identical models)."""
    res = []
    for native, fast in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("YTK_LEAF_NATIVE", native)
        monkeypatch.setenv("YTK_LEAF_FAST", fast)
        p = _params("loss", rounds=3)
        p.device_builder = False  # the host-planned paths (the device engine is tested below)
        p.tree.max_leaf_cnt = 63
        if mode == "pool":
            p.histogram_pool_capacity = 6 * 256 * 28 * 16 / float(1 << 20)
        if mode == "depth":
            p.tree.max_depth = 5
        tr = GBDTTrainer(p, _data(60000, 21, "cuda"), _data(6000, 22, "cuda"))
        tr.train()
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss, tr.builder.hist_miss))
    assert res[0] == res[1] == res[2]
    if mode == "pool":
        assert res[0][3] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, {"max_leaf_cnt": 7}, {"max_depth": 5, "max_leaf_cnt": 40},
                                {"min_split_samples": 900}, {"min_split_loss": 2.0},
                                {"l1": 0.5, "max_abs_leaf_val": 0.3},
                                {"instance_sample_rate": 0.7, "feature_sample_rate": 0.6},
                                {"max_leaf_cnt": 255}, {"spec": "0"}, {"max_leaf_cnt": 1024},
                                {"max_leaf_cnt": 700, "min_split_samples": 60},
                                {"max_leaf_cnt": 255, "plan_global": "1"}])
def test_device_leafwise_matches_host(monkeypatch, kw):
    """GPU-resident leaf-wise engine (device queue replay + planner kernels,
    csrc/hip/gbdt_leafwise.hip) == the host-planned leaf-wise builder: model dump (node
    ids, splits, values, statistics) and losses, bit for bit. max_leaf_cnt > 512 runs the
    planner with its queue in global memory (plan_global: also below 512 leaves)."""
    from ytk_learn_amd.models.gbdt.device_leafwise import DeviceLeafBuilder
    kw = dict(kw)
    monkeypatch.setenv("YTK_LOSSGUIDE_SPEC", kw.pop("spec", "1"))
    monkeypatch.setenv("YTK_LW_PLAN_GLOBAL", kw.pop("plan_global", "0"))
    res = []
    for dev_builder in (False, True):
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 63
        for k, v in kw.items():
            setattr(p.tree, k, v)
        p.device_builder = dev_builder
        tr = GBDTTrainer(p, _data(60000, 21, "cuda"), _data(6000, 22, "cuda"))
        tr.train()
        assert isinstance(tr.builder, DeviceLeafBuilder) == dev_builder
        if dev_builder:
            batches, expanded, overflow = tr.builder.stats()
            assert overflow == 0 and batches >= 1 and expanded >= batches
            big = p.tree.max_leaf_cnt > 512 or os.environ["YTK_LW_PLAN_GLOBAL"] == "1"
            assert (tr.builder.plan_ws is not None) == big
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0][0] == res[1][0]
    assert res[0][1:] == res[1][1:]
    assert res[0][0].count("leaf=") > 3
    if p.tree.max_leaf_cnt > 512:  # the budget is reached: the trees really are that large
        assert max(t.count("leaf=") for t in res[0][0].split("booster[")) > 512


@pytest.mark.gpu
def test_device_leafwise_partition_prefetch_identical(monkeypatch):
    """Leaf-wise engine with the software-pipelined partition body (YTK_LW_PART_PREFETCH=1;
    3: + the next chunk's split-feature bytes) builds the default engine's trees byte for byte."""
    res = []
    for pf in ("0", "1", "2", "3"):
        monkeypatch.setenv("YTK_LW_PART_PREFETCH", pf)
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 63
        p.device_builder = True
        tr = GBDTTrainer(p, _data(60000, 21, "cuda"), _data(6000, 22, "cuda"))
        tr.train()
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1] == res[2] == res[3]


@pytest.mark.gpu
@pytest.mark.parametrize("depth,sample", [(6, 1.0), (9, 0.8)])
def test_device_level_histogram_pool_pingpong_identical(depth, sample):
    """histogram_pool_capacity below the level engine's full slab but above its two live levels:
    the GPU engine stays (odd / even levels alternate between two slot regions, each level's
    built slots zeroed before it accumulates) and builds the uncapped engine's trees byte for
    byte; below the two regions the run falls back to the host builder (same trees)."""
    from ytk_learn_amd.models.gbdt.device_builder import DeviceLevelBuilder, level_slots_needed, level_slots_pingpong
    res = []
    for cap in (None, "pingpong", "host"):
        p = _params("level", rounds=3, instance_sample_rate=sample)
        p.tree.max_depth = depth
        p.tree.max_leaf_cnt = 1 << depth
        p.tree.min_child_hessian_sum = 1.0
        p.device_builder = True
        tr = GBDTTrainer(p, _data(60000, 23, "cuda"), _data(6000, 24, "cuda"))
        tr.prepare()
        slot_mb = tr.B * tr.F * 16 / float(1 << 20)
        if cap is not None:
            full, pp = level_slots_needed(p.tree), level_slots_pingpong(p.tree)
            assert pp < full
            p.histogram_pool_capacity = (pp if cap == "pingpong" else pp - 1) * slot_mb
            tr = GBDTTrainer(p, _data(60000, 23, "cuda"), _data(6000, 24, "cuda"))
        tr.train()
        on_dev = isinstance(tr.builder, DeviceLevelBuilder)
        assert on_dev == (cap != "host")
        if cap == "pingpong":
            assert tr.builder.pingpong and tr.builder.n_slots == level_slots_pingpong(p.tree)
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1] == res[2]


@pytest.mark.gpu
@pytest.mark.parametrize("sample", [1.0, 0.7])
def test_device_leafwise_part_scan_identical(monkeypatch, sample):
    """The first leaf-wise batches reserve their partition chunks by a count pass + scan
    (YTK_LW_PART_SCAN batches; 0: the cursor atomics everywhere) -- the same trees."""
    res = []
    monkeypatch.setenv("YTK_PART_SCAN_MIN_ROWS", "0")  # the scan path at this small shard too
    for n, kern in (("0", "0"), ("2", "0"), ("8", "0"), ("2", "1")):  # kern 1: the scan launch
        monkeypatch.setenv("YTK_LW_PART_SCAN", n)
        monkeypatch.setenv("YTK_PART_SCAN_KERNEL", kern)
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 63
        p.tree.instance_sample_rate = sample
        p.device_builder = True
        tr = GBDTTrainer(p, _data(60000, 21, "cuda"), _data(6000, 22, "cuda"))
        tr.train()
        assert tr.builder.PART_SCAN == int(n)
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1] == res[2] == res[3]


@pytest.mark.gpu
@pytest.mark.parametrize("policy,sample", [("level", 1.0), ("level", 0.7), ("loss", 1.0)])
def test_part_scan_group_sums_identical(monkeypatch, policy, sample):
    """Partition reservations from the count pass's 32-chunk group sums (splits spanning
    several groups, first chunks mid-group: 300K rows = 147 root chunks) equal the cursor
    atomics' -- the same trees, level-wise (every level scanned) and leaf-wise."""
    monkeypatch.setenv("YTK_PART_SCAN_MIN_ROWS", "0")
    res = []
    for n in ("0", "8"):
        monkeypatch.setenv("YTK_PART_SCAN_LEVELS", n)
        monkeypatch.setenv("YTK_LW_PART_SCAN", n)
        p = _params(policy, rounds=3)
        p.tree.instance_sample_rate = sample
        if policy == "loss":
            p.tree.max_leaf_cnt = 63
        p.device_builder = True
        tr = GBDTTrainer(p, _data(300000, 31, "cuda"), _data(6000, 32, "cuda"))
        tr.train()
        assert tr.use_device_builder
        b = tr.builder
        assert (b.part_scan_levels if policy == "level" else b.PART_SCAN) == int(n)
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1]


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{"max_leaf_cnt": 63}, {"max_leaf_cnt": 255, "min_split_samples": 200},
                                {"max_leaf_cnt": 300, "instance_sample_rate": 0.7}])
def test_device_leafwise_children_fast_path_identical(monkeypatch, kw):
    """The partition kernel's one-thread-per-split children planning (default) and the
    general path (YTK_PLAN_FAST=0) build the same trees byte for byte (batches above 256
    splits take the general path either way)."""
    res = []
    for fast in ("0", "1"):
        monkeypatch.setenv("YTK_PLAN_FAST", fast)
        p = _params("loss", rounds=3)
        for k, v in kw.items():
            setattr(p.tree, k, v)
        p.device_builder = True
        tr = GBDTTrainer(p, _data(120000, 31, "cuda"), _data(6000, 32, "cuda"))
        tr.train()
        assert tr.use_device_builder
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1]
    assert res[0][0].count("leaf=") > 100


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, {"max_leaf_cnt": 255, "rows": "1000000000"}, {"sub_max": "2", "alpha": "0"},
                                {"max_depth": 7, "max_leaf_cnt": 40}, {"min_split_samples": 700},
                                {"instance_sample_rate": 0.7, "feature_sample_rate": 0.6, "gh_rows": "1"},
                                {"max_leaf_cnt": 255, "min_split_loss": 1.0, "rows": "4000", "sub_max": "128"},
                                {"l1": 0.5, "max_abs_leaf_val": 0.3, "alpha": "3"}])
def test_device_leafwise_subtrees_identical(monkeypatch, kw):
    """Small-node subtrees (lw_subtree_kernel: one workgroup grows a small batch entry's
    subtree speculatively) build the batch pipeline's trees byte for byte, whatever the row
    threshold (1e9: the root batch itself is one subtree), split budget and gain floor."""
    kw = dict(kw)
    monkeypatch.setenv("YTK_LW_PROF", "1")
    monkeypatch.setenv("YTK_LW_SUB_MAX", kw.pop("sub_max", "32"))
    monkeypatch.setenv("YTK_LW_SUB_ALPHA", kw.pop("alpha", "1.0"))
    monkeypatch.setenv("YTK_LW_GH_ROWS", kw.pop("gh_rows", "0"))
    rows = kw.pop("rows", "16384")
    res = []
    for sub in ("0", rows):
        monkeypatch.setenv("YTK_LW_SUB_ROWS", sub)
        p = _params("loss", rounds=4)
        p.tree.max_leaf_cnt = 63
        for k, v in kw.items():
            setattr(p.tree, k, v)
        p.device_builder = True
        tr = GBDTTrainer(p, _data(120000, 41, "cuda"), _data(6000, 42, "cuda"))
        tr.train()
        assert tr.use_device_builder and tr.builder.sub_on == (sub != "0")
        prof = tr.builder.prof_report()
        if sub != "0":
            assert prof["sub_roots"] > 0 and prof["sub_splits"] >= prof["sub_roots"]
        else:
            assert prof["sub_roots"] == 0
        assert tr.builder.stats()[2] == 0  # no overflow
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1]
    assert res[0][0].count("leaf=") > 40


@pytest.mark.gpu
@pytest.mark.parametrize("sample", [1.0, 0.7])
def test_device_leafwise_row_indexed_gh_identical(monkeypatch, sample):
    """YTK_LW_GH_ROWS=1: (g, h) stays row-indexed (the partition moves row ids only, the
    histograms gather (g, h) by row) -- the same trees byte for byte, with and without row
    sampling."""
    from ytk_learn_amd.models.gbdt.device_leafwise import DeviceLeafBuilder
    res = []
    for on in ("0", "1"):
        monkeypatch.setenv("YTK_LW_GH_ROWS", on)
        p = _params("loss", rounds=3)
        p.tree.max_leaf_cnt = 63
        p.tree.instance_sample_rate = sample
        p.device_builder = True
        tr = GBDTTrainer(p, _data(60000, 21, "cuda"), _data(6000, 22, "cuda"))
        tr.train()
        assert isinstance(tr.builder, DeviceLeafBuilder) and tr.builder.gh_rows == (on == "1")
        res.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert res[0] == res[1]


def test_histogram_pool_capacity_misses_do_not_change_the_tree():
    """histogram_pool_capacity (MB) bounds the live histograms of leaf-wise growth; evicted
    parents are rebuilt (pool miss) instead of derived -- exact int64 sums => same model."""
    dumps, misses, slot_mb = [], [], None
    for pool in (-1.0, "tiny"):
        p = _params("loss", rounds=2)
        p.tree.max_leaf_cnt = 30
        if pool == "tiny":
            p.histogram_pool_capacity = 5 * slot_mb  # 5 live histograms
        tr = GBDTTrainer(p, _data(8000, 13), None)
        tr.prepare()
        slot_mb = tr.B * tr.F * 16 / float(1 << 20)
        tr.init_gradients()
        for i in range(2):
            tr.step(i)
        tr.materialize()
        dumps.append(tr.model.dumps())
        misses.append(tr.builder.hist_miss)
    assert dumps[0] == dumps[1]
    assert misses[0] == 0 and misses[1] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("max_cnt", [300, 5000])
@pytest.mark.parametrize("policy", ["level", "loss"])
def test_wide_bins_device_builder_matches_cpu(cuda, max_cnt, policy):
    """> 256 bins (uint16): the GPU level / leaf-wise engines (row-major feature-group LDS
    histograms) == the host builder on the GPU == the CPU path, tree for tree (ADVICE r1:
    silent corruption above 256)."""
    d_cpu = _data(40000, 21)
    approx = [{"cols": "default", "type": "sample_by_quantile", "max_cnt": max_cnt, "alpha": 0.5}]
    dumps = []
    for dev, dev_builder in (("cpu", False), (cuda, False), (cuda, True)):
        p = _params(policy, rounds=3)
        p.approximate = approx
        p.device_builder = dev_builder
        d = GBDTData(d_cpu.X.to(dev), d_cpu.y.to(dev))
        tr = GBDTTrainer(p, d, GBDTData(d.X[:5000], d.y[:5000]))
        tr.train()
        assert tr.bins.dtype == torch.int16 and tr.B > 256
        assert tr.use_device_builder == (dev_builder and dev != "cpu")
        dumps.append((tr.model.dumps(), tr.last_train_loss))
    # integer histograms: the two GPU builders agree bitwise; the CPU gradient path agrees
    # to float rounding (same check as test_train_gpu_matches_cpu)
    assert dumps[1][0] == dumps[2][0]
    assert dumps[1][1] == dumps[2][1]
    assert dumps[0][0].split("\n")[5] == dumps[1][0].split("\n")[5]  # root split line
    np.testing.assert_allclose(dumps[0][1], dumps[1][1], rtol=2e-4)


def test_more_than_65536_candidates_is_an_error():
    from ytk_learn_amd.utils.errors import YtkLearnError

    X = torch.arange(70000, dtype=torch.float32)[:, None].repeat(1, 2)
    y = (torch.rand(70000, 1) < 0.5).float()
    p = _params("level", rounds=1)
    p.approximate = [{"cols": "default", "type": "no_sample"}]
    tr = GBDTTrainer(p, GBDTData(X, y), None)
    with pytest.raises(YtkLearnError, match="65536"):
        tr.prepare()


def test_split_groups_every_group_nonempty(monkeypatch):
    """Feature groups of the node-resident split search: every group holds >= 1 feature;
    no grouping where the node-resident kernel does not apply (B > 256)."""
    from ytk_learn_amd.ops import gbdt as gops
    monkeypatch.delenv("YTK_SPLIT_GROUPS", raising=False)
    for F in range(1, 70):
        g = gops.split_groups(256, F)
        fg = -(-F // g)
        assert 1 <= g <= min(4, F) and (g - 1) * fg < F
    assert gops.split_groups(300, 28) == 1
    monkeypatch.setenv("YTK_SPLIT_GROUPS", "1")
    assert gops.split_groups(256, 28) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, {"feature_sample_rate": 0.6}, {"max_leaf_cnt": 40}])
def test_fused_reduce_split_identical_depth6(cuda, monkeypatch, kw):
    """The one-launch staged reduce + split search (lv_reduce_split_kernel, YTK_FUSE_REDUCE_SPLIT=1)
    builds the trees of the separate hist_reduce + split_node launches byte for byte on a
    depth-6 tree (split-K slots at the top levels, direct slots below)."""
    d = _data(300000, 21, cuda)
    out = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("YTK_FUSE_REDUCE_SPLIT", fuse)
        p = _params("level", rounds=4, **{k: v for k, v in kw.items() if k != "max_leaf_cnt"})
        p.tree.max_depth = 6
        p.tree.max_leaf_cnt = kw.get("max_leaf_cnt", 64)
        p.device_builder = True
        tr = GBDTTrainer(p, d, _data(5000, 22, cuda))
        tr.train()
        assert tr.use_device_builder
        out.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert out[0] == out[1]
    assert out[0][0].count("leaf=") > 40
