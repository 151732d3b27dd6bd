#!/usr/bin/env python3
"""Block timestamps of the fused reduce + split kernel (lv_reduce_split_kernel, YTK_RS_PROF=1):
per level, the kernel's block-entry spread, when the reduce blocks counted themselves in and
how long the last-arriver tails (built + derived split search) took. Usage:
dbg_rs_prof.py [rows]"""
import os
import sys

os.environ["YTK_RS_PROF"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ytk_learn_amd.data.synthetic import higgs_like  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402

dev = torch.device("cuda")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_312_500
X, y = higgs_like(n, seed=0, device=dev)
Xt, yt = higgs_like(50_000, seed=500, device=dev)
tp = TreeParams(max_depth=6, max_leaf_cnt=64, min_child_hessian_sum=100.0, learning_rate=0.1, grow_policy="level")
params = GBDTParams(round_num=6, loss_function="sigmoid", tree=tp,
                    approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255,
                                  "use_sample_weight": False, "alpha": 0.5}])
tr = GBDTTrainer(params, GBDTData(X, y), GBDTData(Xt, yt))
tr.prepare()
tr.init_gradients()
for i in range(5):
    tr.run_round(i)
tr.materialize()
torch.cuda.synchronize()
b = tr.builder
assert b.fuse_rs and b.rs_prof is not None
for t in b.rs_prof:
    t.zero_()
tr.run_round(5)
tr.materialize()
torch.cuda.synchronize()
for c, t in enumerate(b.rs_prof):
    a = t.cpu().numpy().astype(np.int64)
    a = a[a[:, 0] > 0]
    if len(a) == 0:
        continue
    t0 = a[:, 0].min()
    ent = (a[:, 0] - t0) / 100.0  # 100 MHz -> us
    cin = (a[a[:, 1] > 0, 1] - t0) / 100.0
    tails = a[a[:, 7] > 0]
    msg = (f"level {c}: blocks {len(a)}, entry spread {ent.max():.2f} us, counted-in "
           f"p50 {np.median(cin):.2f} max {cin.max():.2f} us")
    if len(tails):
        tb = (tails[:, 1] - t0) / 100.0
        t1 = (tails[:, 2] - tails[:, 1]) / 100.0
        t2 = (tails[:, 7] - tails[:, 2]) / 100.0  # the pair search
        end = (tails[:, 7] - t0) / 100.0
        ph = [np.median((tails[:, i + 1] - tails[:, i]) / 100.0) for i in range(2, 7)]
        msg += (f" | tails {len(tails)}: start p50 {np.median(tb):.2f} max {tb.max():.2f}, search {np.median(t2):.2f}"
                f" (max {t2.max():.2f}) = load {ph[0]:.2f} + totals {ph[1]:.2f} + scan {ph[2]:.2f} + barrier {ph[3]:.2f}"
                f" + record {ph[4]:.2f}, last end {end.max():.2f} us")
        sc = [np.median((tails[:, 9 + i] - tails[:, 8 + i]) / 100.0) for i in range(2)]
        msg += ("\n   wave-0 scan: loads + prefix scans %.2f, gains %.2f" % tuple(sc))
    print(msg)
