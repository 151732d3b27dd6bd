"""GPU tree engines on every objective: the level engine and the leaf-wise engine must
build the host-driven builder's model byte for byte (exact int64 histograms) for softmax
(K = 3), random forest, poisson and l1 (device leaf refine, both refine modes); plus the
engines' capacity limits (depth-12 trees, trees too large for LDS, histogram pool cap)."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.data.synthetic import higgs_like
from ytk_learn_amd.models.gbdt.builder import TreeBuilder, TreeParams
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer
from ytk_learn_amd.ops import gbdt as gops

pytestmark = pytest.mark.gpu


def _objective_data(obj, n, seed, dev):
    X, y = higgs_like(n, seed=seed)
    K = 1
    if obj == "softmax":
        K = 3
        c = torch.clamp((X[:, 25] * 1.5).long(), 0, K - 1)
        y = torch.nn.functional.one_hot(c, K).float()
    elif obj == "poisson":
        y = torch.poisson(torch.exp(0.3 * X[:, 25:26]))
    elif obj.startswith("l1"):
        y = torch.round(X[:, 25:26] * 2.0 + 0.1 * torch.randn(n, 1), decimals=1)  # ties in the residuals
    return GBDTData(X.to(dev), y.to(dev)), K


def _params(obj, policy, K):
    tp = TreeParams(max_depth=5 if policy == "level" else -1, max_leaf_cnt=32 if policy == "level" else 24,
                    min_child_hessian_sum=5.0, grow_policy=policy, learning_rate=0.2)
    p = GBDTParams(round_num=3, tree=tp, class_num=K)
    if obj == "rf":
        p.type = "random_forest"
        tp.instance_sample_rate = 0.7
    else:
        p.loss_function = {"l1_appr": "l1", "l1_exact": "l1"}.get(obj, obj)
    p.lad_refine_appr = obj != "l1_exact"
    p.uniform_base_prediction = 1.0 if obj == "poisson" else (0.5 if obj == "rf" else 0.0)
    p.eval_metric = ["confusion_matrix"] if obj == "softmax" else ["rmse"]
    return p


@pytest.mark.parametrize("policy", ["level", "loss"])
@pytest.mark.parametrize("obj", ["softmax", "rf", "poisson", "l1_appr", "l1_exact"])
def test_device_engines_match_host_builder(cuda, policy, obj):
    tr_d, K = _objective_data(obj, 30000, 31, cuda)
    te_d, _ = _objective_data(obj, 4000, 32, cuda)
    out = []
    for dev_builder in (False, True):
        p = _params(obj, policy, K)
        p.device_builder = dev_builder
        tr = GBDTTrainer(p, tr_d, te_d)
        tr.train()
        assert tr.use_device_builder == dev_builder, (obj, policy)
        out.append((tr.model.dumps(), tr.last_train_loss, tr.last_test_loss))
    assert out[0][0] == out[1][0]
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]


def test_level_engine_depth12_matches_host(cuda):
    """max_depth 12 (8191 nodes): the score/gradient pass keeps its LDS budget (no deferred
    leaf counts for trees this size) and the model equals the host builder's."""
    X, y = higgs_like(40000, seed=41)
    d = GBDTData(X.to(cuda), y.to(cuda))
    out = []
    for dev_builder in (False, True):
        tp = TreeParams(max_depth=12, max_leaf_cnt=4096, min_child_hessian_sum=0.5, grow_policy="level",
                        learning_rate=0.2)
        p = GBDTParams(round_num=2, tree=tp, device_builder=dev_builder)
        tr = GBDTTrainer(p, d, None)
        tr.train()
        assert tr.use_device_builder == dev_builder
        if dev_builder:
            assert not tr.builder.defer_leaf_counts and tr.builder.max_nodes == 8191
        out.append((tr.model.dumps(), tr.last_train_loss))
    assert out[0] == out[1]


def test_tree_grad_nodes_beyond_lds_walk_global(cuda):
    """A 20001-node bin-threshold tree (node arrays > 160 KiB of LDS): tree_grad walks the
    nodes in global memory and matches the CPU walk + loss."""
    g = np.random.default_rng(5)
    N, F, nn = 50000, 28, 20001
    bins = torch.from_numpy(g.integers(0, 255, (N, 32), dtype=np.uint8))
    # a random full binary tree: node i has children 2i+1, 2i+2 while < nn
    feat = np.full(nn, -1, np.int32)
    thr = np.zeros(nn, np.int32)
    left = np.full(nn, -1, np.int32)
    right = np.full(nn, -1, np.int32)
    internal = np.arange(nn) * 2 + 2 < nn
    feat[internal] = g.integers(0, F, internal.sum())
    thr[internal] = g.integers(0, 255, internal.sum())
    left[internal] = (np.arange(nn) * 2 + 1)[internal]
    right[internal] = (np.arange(nn) * 2 + 2)[internal]
    val = g.normal(size=nn).astype(np.float32)
    arrs = [torch.from_numpy(a) for a in (feat, thr, left, right, val)]
    y = torch.from_numpy((g.random((N, 1)) < 0.5).astype(np.float32))
    score0 = torch.from_numpy(g.normal(size=(N, 1)).astype(np.float32))
    init = torch.zeros((N, 1))
    res = []
    for dev in ("cpu", cuda):
        score = score0.clone().to(dev)
        pred = torch.zeros((N, 1), device=dev)
        gh = torch.zeros((N, 2), device=dev)
        acc = gops.tree_grad(bins.to(dev), [a.to(dev) for a in arrs], score, init.to(dev), y.to(dev), None,
                             "sigmoid", 0.0, 1.0, pred, gh, True, None)
        res.append((score.cpu(), gh.cpu(), acc.cpu()))
    torch.testing.assert_close(res[1][0], res[0][0], rtol=0, atol=0)
    torch.testing.assert_close(res[1][1], res[0][1], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(res[1][2], res[0][2], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("policy", ["level", "loss"])
def test_histogram_pool_capacity_routes_engines(cuda, policy):
    """histogram_pool_capacity below the GPU engine's resident slot slab -> the host builder
    (its LRU pool honours the cap, HistogramPool.java:36-273); above it -> the GPU engine."""
    X, y = higgs_like(20000, seed=43)
    d = GBDTData(X.to(cuda), y.to(cuda))
    for cap_mb, want_device in ((0.5, False), (4096.0, True)):
        tp = TreeParams(max_depth=5 if policy == "level" else -1, max_leaf_cnt=32 if policy == "level" else 24,
                        min_child_hessian_sum=5.0, grow_policy=policy)
        p = GBDTParams(round_num=1, tree=tp, histogram_pool_capacity=cap_mb)
        tr = GBDTTrainer(p, d, None)
        tr.prepare()
        assert tr.use_device_builder == want_device
        assert isinstance(tr.builder, TreeBuilder) == (not want_device)
