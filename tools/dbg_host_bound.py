#!/usr/bin/env python3
"""Is a bench configuration host-bound? Times the host side of K rounds (the run_round calls,
which only enqueue device work) against the synchronised wall time of the same rounds.

usage: python tools/dbg_host_bound.py [--train-rows N] [--policy level|loss] [--rounds K]
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
    ap.add_argument("--train-rows", type=int, default=1_312_500)
    ap.add_argument("--test-rows", type=int, default=62_500)
    ap.add_argument("--policy", default="level", choices=["level", "loss"])
    ap.add_argument("--rounds", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    X, y = higgs_like(a.train_rows, seed=17000, device=dev)
    Xt, yt = higgs_like(a.test_rows, seed=17500, device=dev)
    if a.policy == "level":
        tp = TreeParams(max_depth=6, max_leaf_cnt=64, min_child_hessian_sum=100.0, min_split_loss=0.0,
                        min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="level")
    else:
        tp = TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0, min_split_loss=0.0,
                        min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="loss")
    W = 5
    params = GBDTParams(round_num=W + a.rounds, loss_function="sigmoid", eval_metric=["auc"], missing_value="value@0",
                        approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255,
                                      "use_sample_weight": False, "alpha": 0.5}], tree=tp)
    tr = GBDTTrainer(params, GBDTData(X, y), GBDTData(Xt, yt), log=YtkLogger(0, stream=sys.stderr, every=1000))
    tr.prepare()
    tr.init_gradients()
    for i in range(W):
        tr.run_round(i)
    tr.materialize()
    torch.cuda.synchronize()
    # time spent blocked on the device (event waits of the readback pipeline) is not host work
    waited = [0.0]
    orig_sync = torch.cuda.Event.synchronize

    def timed_sync(self):
        t = time.perf_counter()
        orig_sync(self)
        waited[0] += time.perf_counter() - t

    torch.cuda.Event.synchronize = timed_sync
    host = 0.0
    t0 = time.perf_counter()
    for i in range(W, W + a.rounds):
        t1 = time.perf_counter()
        tr.run_round(i)
        host += time.perf_counter() - t1
    tr.materialize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(json.dumps({"policy": a.policy, "train_rows": a.train_rows, "rounds": a.rounds,
                      "host_ms_per_round": round(1e3 * host / a.rounds, 4),
                      "host_busy_ms_per_round": round(1e3 * (host - waited[0]) / a.rounds, 4),
                      "wall_ms_per_round": round(1e3 * wall / a.rounds, 4)}))


if __name__ == "__main__":
    main()
