#!/usr/bin/env python3
"""Exact-greedy GBDT (tree_maker = "feature", presorted columns, every distinct value a
candidate) on the Higgs shape: seconds per whole boosting round on one GPU.

Reference: FeatureParallelTreeMakerByLevel.java (single machine, level-wise); ytk-learn
publishes no number for it. Synthetic Higgs-shape data (continuous columns: ~every row a
distinct value).

usage: python tools/bench_exact.py [--train-rows 10500000] [--rounds 5] [--warmup 1] [--depth 6]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402
from ytk_learn_amd.utils.logging import YtkLogger  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-rows", type=int, default=10_500_000)
    ap.add_argument("--test-rows", type=int, default=500_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--depth", type=int, default=6)
    a = ap.parse_args()
    dev = torch.device("cuda")
    X, y = higgs_like(a.train_rows, seed=17000, device=dev)
    Xt, yt = higgs_like(a.test_rows, seed=17500, device=dev)
    distinct = int(torch.unique(X[:, 0]).numel())
    tp = TreeParams(max_depth=a.depth, max_leaf_cnt=1 << a.depth, min_child_hessian_sum=100.0, min_split_loss=0.0,
                    min_split_samples=-1, learning_rate=0.1, grow_policy="level")
    p = GBDTParams(round_num=a.warmup + a.rounds, loss_function="sigmoid", missing_value="value@0",
                   tree_maker="feature", tree=tp)
    tr = GBDTTrainer(p, GBDTData(X, y), GBDTData(Xt, yt), log=YtkLogger(0, stream=sys.stderr, every=1000))
    t0 = time.perf_counter()
    tr.prepare()
    tr.init_gradients()
    torch.cuda.synchronize()
    prep = time.perf_counter() - t0
    for i in range(a.warmup):
        tr.run_round(i)
    tr.materialize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.warmup, a.warmup + a.rounds):
        tr.run_round(i)
    tr.materialize()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.rounds
    print(json.dumps({"metric": "exact greedy GBDT (presorted columns) sec/round", "value": round(el, 5),
                      "unit": "s/round", "train_rows": a.train_rows, "features": int(X.shape[1]),
                      "distinct_values_col0": distinct, "depth": a.depth, "rounds_timed": a.rounds,
                      "prep_s": round(prep, 3), "train_loss": tr.round_losses[a.warmup + a.rounds - 1][0],
                      "trees": len(tr.model.trees)}), flush=True)


if __name__ == "__main__":
    main()
