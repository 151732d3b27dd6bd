"""cProfile of leaf-wise tree building in steady state (after warmup trees) on the GPU:
python tools/prof_leaf_steady.py"""
import cProfile
import pstats
import sys

import torch

sys.path.insert(0, ".")
from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402

dev = torch.device("cuda", 0)
X, y = higgs_like(10_500_000, seed=1, device=dev)
p = GBDTParams(round_num=4, tree=TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0,
                                            grow_policy="loss"))
tr = GBDTTrainer(p, GBDTData(X, y), None)
tr.train()  # warmup (compiles, caches)
p.round_num = 10
pr = cProfile.Profile()
tr2 = GBDTTrainer(p, GBDTData(X, y), None)
pr.enable()
tr2.train()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
