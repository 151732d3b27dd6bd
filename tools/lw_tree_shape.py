#!/usr/bin/env python3
"""Shape of late leaf-wise trees (Higgs, 255 leaves): what a small-node subtree kernel would see.

Trains ``--trees`` leaf-wise trees on the bench's synthetic Higgs rows, then for the last
``--last`` trees reports, per row threshold T: the depth of the part of the tree made of nodes
with more than T rows (the batches the global pipeline still needs), the subtrees rooted at the
first small node on each path (splits, depth, rows, histogram rows = sum of the smaller child
over the subtree's splits) and the largest of them (the subtree kernel's critical path).

  python tools/lw_tree_shape.py --trees 350 --last 20 > gpurun_out/shape.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from ytk_learn_amd.data.synthetic import higgs_like_rows  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402


def shape(t, T):
    n = t.num_nodes
    depth = [0] * n
    order = [0]
    for u in order:
        if not t.is_leaf[u]:
            for c in (t.left[u], t.right[u]):
                depth[c] = depth[u] + 1
                order.append(c)
    big_depth = 0
    subs = []
    for u in order:
        if t.is_leaf[u]:
            continue
        cnt = t.sample_cnt[u]
        if cnt > T:
            big_depth = max(big_depth, depth[u] + 1)
            continue
        p = t.parent[u]
        if p >= 0 and t.sample_cnt[p] <= T:
            continue  # inside a subtree already counted
        # subtree rooted at u
        splits = hrows = 0
        sd = 0
        stack = [(u, 0)]
        while stack:
            v, d = stack.pop()
            if t.is_leaf[v]:
                continue
            splits += 1
            sd = max(sd, d + 1)
            hrows += min(t.sample_cnt[t.left[v]], t.sample_cnt[t.right[v]])
            stack += [(t.left[v], d + 1), (t.right[v], d + 1)]
        subs.append((splits, sd, cnt, hrows))
    return big_depth, subs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=350)
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--rows", type=int, default=10_500_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    X, y = higgs_like_rows(a.rows, 0, a.rows, seed=17000, device=dev)
    tp = TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0, min_split_loss=0.0,
                    min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="loss")
    p = GBDTParams(round_num=a.trees, loss_function="sigmoid", eval_metric=[], missing_value="value@0",
                   approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255,
                                 "use_sample_weight": False, "alpha": 0.5}], tree=tp)
    tr = GBDTTrainer(p, GBDTData(X, y), None)
    tr.train()
    trees = tr.model.trees[-a.last:]
    out = {"trees": a.trees, "last": a.last}
    for T in (4096, 8192, 16384, 32768, 65536, 131072):
        bd, mx_sub, nsub, sp, hr, mx_h, mx_sp = [], [], [], [], [], [], []
        for t in trees:
            b, subs = shape(t, T)
            bd.append(b)
            nsub.append(len(subs))
            sp.append(sum(s[0] for s in subs))
            hr.append(sum(s[3] for s in subs))
            mx_h.append(max([s[3] for s in subs] or [0]))
            mx_sp.append(max([s[0] for s in subs] or [0]))
            mx_sub.append(max([s[1] for s in subs] or [0]))
        out[str(T)] = {"big_depth": float(np.mean(bd)), "subtrees": float(np.mean(nsub)),
                       "sub_splits": float(np.mean(sp)), "sub_hist_rows": float(np.mean(hr)),
                       "max_sub_hist_rows": float(np.mean(mx_h)), "max_sub_splits": float(np.mean(mx_sp)),
                       "max_sub_depth": float(np.mean(mx_sub))}
    depths = []
    for t in trees:
        b, _ = shape(t, 0)
        depths.append(b)
    out["tree_depth"] = float(np.mean(depths))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
