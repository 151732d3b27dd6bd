#!/usr/bin/env python3
"""Why does the per-tree time drift with the round index? Trains the bench's Higgs-shape
model for K rounds (leaf-wise 255 leaves by default, ``--policy level`` for depth 6) and
prints, per window of rounds: ms per tree (synchronised at the window edges), and for the
leaf-wise engine the mean batches and speculative expansions per tree, plus the mean
depth of the trees' leaves (from the converted host trees).

usage: python tools/dbg_leaf_drift.py [--rounds 500] [--window 50] [--policy loss]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402
from ytk_learn_amd.utils.logging import YtkLogger  # noqa: E402


def leaf_depths(tree):
    """Depths of the leaves of a host Tree (walk from the root by child ids)."""
    out = []
    stack = [(0, 0)]
    while stack:
        n, d = stack.pop()
        if tree.is_leaf[n]:
            out.append(d)
        else:
            stack.append((tree.left[n], d + 1))
            stack.append((tree.right[n], d + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=500)
    ap.add_argument("--window", type=int, default=50)
    ap.add_argument("--policy", default="loss", choices=["loss", "level"])
    ap.add_argument("--train-rows", type=int, default=10_500_000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    X, y = higgs_like(a.train_rows, seed=17000, device=dev)
    Xt, yt = higgs_like(500_000, seed=17500, device=dev)
    if a.policy == "loss":
        tp = TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0, min_split_loss=0.0,
                        min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="loss")
    else:
        tp = TreeParams(max_depth=6, max_leaf_cnt=64, min_child_hessian_sum=100.0, min_split_loss=0.0,
                        min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="level")
    params = GBDTParams(round_num=a.rounds, loss_function="sigmoid", eval_metric=["auc"], missing_value="value@0",
                        approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255,
                                      "use_sample_weight": False, "alpha": 0.5}], tree=tp)
    log = YtkLogger(0, stream=sys.stderr, every=100)
    tr = GBDTTrainer(params, GBDTData(X, y), GBDTData(Xt, yt), log=log)
    tr.prepare()
    tr.init_gradients()
    b = tr.builder
    rows = []
    for w0 in range(0, a.rounds, a.window):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batches = []
        for i in range(w0, min(a.rounds, w0 + a.window)):
            tr.run_round(i)
            batches.append(getattr(b, "last_batches", 0))
        tr.materialize()
        torch.cuda.synchronize()
        n = min(a.rounds, w0 + a.window) - w0
        ms = 1e3 * (time.perf_counter() - t0) / n
        trees = tr.model.trees[w0:w0 + n]
        depths = [np.mean(leaf_depths(t)) for t in trees]
        maxd = [max(leaf_depths(t)) for t in trees]
        rows.append({"rounds": f"{w0}-{w0 + n - 1}", "ms_per_tree": round(ms, 4),
                     "batches": round(float(np.mean(batches)), 2),
                     "mean_leaf_depth": round(float(np.mean(depths)), 2),
                     "max_leaf_depth": round(float(np.mean(maxd)), 2)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
