"""GPU: speculative vs sequential leaf-wise growth must give identical models."""
import os, sys
sys.path.insert(0, "/root/repo")
import torch
from ytk_learn_amd.data.synthetic import higgs_like
from ytk_learn_amd.models.gbdt.builder import TreeParams
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer
n, rounds = int(sys.argv[1]), int(sys.argv[2])
X, y = higgs_like(n, seed=1, device="cuda")
out = {}
for spec in sys.argv[3].split(","):
    os.environ["YTK_LOSSGUIDE_SPEC"] = spec
    tp = TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0, grow_policy="loss", learning_rate=0.1)
    p = GBDTParams(round_num=rounds, tree=tp, approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255, "alpha": 0.5}])
    tr = GBDTTrainer(p, GBDTData(X, y), None)
    tr.prepare(); tr.init_gradients()
    for i in range(rounds):
        tr.step(i)
        print("spec", spec, "tree", i, "batches", tr.builder.last_batches, tr.builder.last_expanded, flush=True)
    tr.materialize()
    out[spec] = tr.model.dumps()
    print([l for l in out[spec].splitlines() if l.startswith("booster")], flush=True)
a, b = list(out.values())[0].splitlines(), list(out.values())[-1].splitlines()
print("identical", a == b)
for i, (x, z) in enumerate(zip(a, b)):
    if x != z:
        print(i, x[:200]); print(i, z[:200]); break
