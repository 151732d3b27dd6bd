"""Vectorised model conversion (convertModel, GBDTOptimizer.java:663-690) and the
pipelined per-round tree/loss readback of the trainer."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from ytk_learn_amd.models.gbdt.device_builder import DNODE_DTYPE, node_table_to_tree
from ytk_learn_amd.models.gbdt.tree import CandTable, Tree

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _random_table(rng, depth=6):
    """A complete-ish random tree as a device node table (BFS ids like the level builder)."""
    nodes = np.zeros(2 ** (depth + 1) - 1, DNODE_DTYPE)
    nn, frontier = 1, [0]
    for d in range(depth):
        nxt = []
        for nid in frontier:
            if d == depth - 1 or rng.random() < 0.2:
                continue
            nodes[nid]["left"], nodes[nid]["right"] = nn, nn + 1
            nxt += [nn, nn + 1]
            nn += 2
        frontier = nxt
    for i in range(nn):
        leaf = nodes[i]["left"] == 0 and i != 0 or (i == 0 and nn == 1)
        if leaf:
            nodes[i]["left"] = nodes[i]["right"] = -1
            nodes[i]["is_leaf"] = 1
            nodes[i]["value"] = rng.normal()
        else:
            nodes[i]["feat"] = rng.integers(0, 5)
            a = rng.integers(0, 8)
            nodes[i]["bin_a"], nodes[i]["bin_b"] = a, a + 1
        nodes[i]["loss_chg"] = rng.random()
        nodes[i]["H"] = rng.random() * 100
        nodes[i]["cnt_global"] = rng.integers(1, 1000)
    st = np.zeros(16, np.int32)
    st[0] = nn
    return nodes, st


def _to_tree_loop(nodes, st):
    """The per-node reference conversion (round-1 implementation)."""
    nn = int(st[0])
    t = Tree()
    for _ in range(nn - 1):
        t._alloc(-1)
    for i in range(nn):
        n = nodes[i]
        if bool(n["is_leaf"]) or n["left"] < 0:
            t.set_leaf(i, float(n["value"]))
        else:
            t.is_leaf[i] = False
            t.left[i], t.right[i] = int(n["left"]), int(n["right"])
            t.parent[t.left[i]] = i
            t.parent[t.right[i]] = i
            t.set_split(i, int(n["feat"]), int(n["bin_a"]), int(n["bin_b"]))
        t.loss_chg[i] = float(n["loss_chg"])
        t.hess_sum[i] = float(np.float32(n["H"]))
        t.sample_cnt[i] = int(n["cnt_global"])
    return t


def _convert_loop(t, cands, split_type, names, fill):
    for i in range(t.num_nodes):
        if t.is_leaf[i]:
            continue
        c = np.asarray(cands[t.feat[i]], np.float32)
        a, b = t.slot_a[i], t.slot_b[i]
        if split_type == "mean":
            v = np.float32(0.5) * (c[a] + c[b])
        else:
            s = a + b
            v = c[s // 2] if s % 2 == 0 else np.float32(0.5) * (c[(s - 1) // 2] + c[(s + 1) // 2])
        t.cond[i] = float(np.float32(v))
        t.feat_name[i] = names[t.feat[i]]
        t.default_left[i] = bool(np.float32(fill[t.feat[i]]) < np.float32(t.cond[i]))


@pytest.mark.parametrize("split_type", ["mean", "median"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_vectorised_conversion_matches_per_node_loop(split_type, seed):
    rng = np.random.default_rng(seed)
    nodes, st = _random_table(rng)
    cands = [np.sort(rng.normal(size=10)).astype(np.float32) for _ in range(5)]
    names = [f"f{i}" for i in range(5)]
    fill = rng.normal(size=5).astype(np.float32)
    ref = _to_tree_loop(nodes, st)
    _convert_loop(ref, cands, split_type, names, fill)
    t = node_table_to_tree(nodes.view(np.uint8), st)
    t.convert_split_values(CandTable(cands), split_type)
    t.add_feature_names(np.asarray(names, dtype=object))
    t.add_default_direction(fill)
    assert t.dump(0) == ref.dump(0)
    for attr in ("left", "right", "parent", "feat", "slot_a", "slot_b", "cond", "leaf", "is_leaf", "default_left",
                 "loss_chg", "hess_sum", "sample_cnt", "feat_name"):
        assert getattr(t, attr) == getattr(ref, attr), attr
    # list-of-arrays input takes the same path
    t2 = node_table_to_tree(nodes.view(np.uint8), st)
    t2.convert_split_values(cands, split_type)
    assert t2.cond == t.cond


def test_pipelined_rounds_land_every_tree_and_loss():
    from ytk_learn_amd.data.synthetic import higgs_like
    from ytk_learn_amd.models.gbdt.builder import TreeParams
    from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer

    X, y = higgs_like(6000, seed=3)
    Xt, yt = higgs_like(1000, seed=4)
    p = GBDTParams(round_num=5, tree=TreeParams(max_depth=4, max_leaf_cnt=16, min_child_hessian_sum=2.0))
    tr = GBDTTrainer(p, GBDTData(X, y), GBDTData(Xt, yt))
    tr.prepare()
    tr.init_gradients()
    for i in range(5):
        tr.run_round(i)
    tr.materialize()
    assert len(tr.model.trees) == 5 and sorted(tr.round_losses) == list(range(5))
    trl, tel = tr._losses()
    assert tr.round_losses[4] == pytest.approx((trl, tel), rel=1e-12)
    assert all(t.converted for t in tr.model.trees)


def test_bench_cpu_contract_times_whole_rounds():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--train-rows",
                          "6000", "--test-rows", "1000", "--steps", "2", "--warmup", "1", "--depth", "3",
                          "--leafwise-steps", "1", "--quiet"],
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["trees_converted"] == 3 and res["vs_baseline"] is None
    assert res["higher_is_better"] is False and res["steps"] == 2 and res["warmup"] == 1
    assert res["leafwise_s_per_tree"] > 0
