"""CPU vs GPU GBDT model dump comparison (host builder), for kernel/numerics debugging."""
import os, sys
sys.path.insert(0, "/root/repo")
import torch
from ytk_learn_amd.data.synthetic import higgs_like
from ytk_learn_amd.models.gbdt.builder import TreeParams
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer
n, policy, rounds = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
X, y = higgs_like(n, seed=1)
out = {}
for dev in ("cpu", "cuda"):
    tp = TreeParams(max_depth=-1 if policy == "loss" else 6, max_leaf_cnt=255 if policy == "loss" else 64,
                    min_child_hessian_sum=100.0, grow_policy=policy, learning_rate=0.1)
    p = GBDTParams(round_num=rounds, tree=tp, approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255, "alpha": 0.5}])
    p.device_builder = False
    tr = GBDTTrainer(p, GBDTData(X.to(dev), y.to(dev)), None)
    tr.train()
    out[dev] = tr.model.dumps()
a, b = out["cpu"].splitlines(), out["cuda"].splitlines()
print(policy, "spec", os.environ.get("YTK_LOSSGUIDE_SPEC", "1"), "identical", a == b, len(a), len(b), flush=True)
for i, (x, z) in enumerate(zip(a, b)):
    if x != z:
        print(i, x[:200]); print(i, z[:200]); break
