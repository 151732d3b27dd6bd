"""Leaf-wise speculation efficiency: batches and expanded nodes per 255-leaf tree,
host-planned (virtual replay) vs device engine (top-k candidates), Higgs shape."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_500_000
X, y = higgs_like(n, seed=1, device="cuda")
for dev_builder in (False, True):
    p = GBDTParams(round_num=6, tree=TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0,
                                                grow_policy="loss"))
    p.device_builder = dev_builder
    tr = GBDTTrainer(p, GBDTData(X, y), None)
    tr.prepare()
    tr.init_gradients()
    stats = []
    for i in range(6):
        tr.step(i)
        torch.cuda.synchronize()
        if dev_builder:
            b, e, _ = tr.builder.stats()
        else:
            b, e = tr.builder.last_batches, tr.builder.last_expanded
        stats.append((b, e))
    print(("device" if dev_builder else "host  ") + f" batches/expanded per tree: {stats}", flush=True)
