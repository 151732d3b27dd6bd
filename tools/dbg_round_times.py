#!/usr/bin/env python3
"""Per-round host timestamps of the bench's timed loop (where does the fixed overhead of a
short timed region go?). Prints cumulative ms after each run_round and after materialize."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402
from ytk_learn_amd.utils.logging import YtkLogger  # noqa: E402

dev = torch.device("cuda")
X, y = higgs_like(10_500_000, seed=0, device=dev)
Xt, yt = higgs_like(500_000, seed=500, device=dev)
tp = TreeParams(max_depth=6, max_leaf_cnt=64, min_child_hessian_sum=100.0, min_split_loss=0.0,
                min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="level")
W, K = 5, int(sys.argv[1]) if len(sys.argv) > 1 else 20
params = GBDTParams(round_num=W + K, loss_function="sigmoid", eval_metric=["auc"], missing_value="value@0",
                    approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255,
                                  "use_sample_weight": False, "alpha": 0.5}], tree=tp)
log = YtkLogger(0, stream=sys.stderr, every=10)
tr = GBDTTrainer(params, GBDTData(X, y), GBDTData(Xt, yt), log=log)
tr.prepare()
tr.init_gradients()
for i in range(W):
    tr.run_round(i)
tr.materialize()
torch.cuda.synchronize()
t0 = time.perf_counter()
marks = []
for i in range(W, W + K):
    tr.run_round(i)
    marks.append(1e3 * (time.perf_counter() - t0))
tr.materialize()
m1 = 1e3 * (time.perf_counter() - t0)
torch.cuda.synchronize()
m2 = 1e3 * (time.perf_counter() - t0)
print("per-round host marks (ms):", " ".join(f"{m:.2f}" for m in marks))
print(f"after materialize {m1:.2f} ms, after sync {m2:.2f} ms, per round {m2 / K:.4f} ms")
