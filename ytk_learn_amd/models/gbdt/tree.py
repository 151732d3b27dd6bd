"""Regression tree + GBDT model container and their text format.

Format and semantics follow the reference (byte-compatible text):
  * ``J/data/gbdt/Tree.java:47-48,258-291`` node lines / booster header
  * ``J/data/gbdt/GBDTModel.java:63-77`` model header
  * ``J/data/gbdt/Tree.java:293-309`` slot interval -> raw threshold
  * ``J/data/gbdt/Tree.java:357-375`` default direction = left iff fill < cond
  * ``J/feature/FeatureSplitType.java`` mean / median split value

Storage is struct-of-arrays (numpy) so a whole forest flattens to device arrays
for the forest inference kernel without per-node Python objects.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Sequence

import numpy as np

from ...utils.javafmt import java_float_str, parse_java_float

INNER_RE = re.compile(
    r"(\S+):\[f_(\S+)<=(\S+)] yes=(\S+),no=(\S+),missing=(\S+),gain=(\S+),hess_sum=(\S+),sample_cnt=(\S+)")
INNER_NOSTAT_RE = re.compile(r"(\S+):\[f_(\S+)<=(\S+)] yes=(\S+),no=(\S+),missing=(\S+)")
LEAF_RE = re.compile(r"(\S+):leaf=([^,\s]+),hess_sum=(\S+),sample_cnt=(\S+)")
LEAF_NOSTAT_RE = re.compile(r"(\S+):leaf=([^,\s]+)")


class Tree:
    def __init__(self):
        self.left: List[int] = [-1]
        self.right: List[int] = [-1]
        self.parent: List[int] = [-1]
        self.feat: List[int] = [-1]
        self.feat_name: List[Optional[str]] = [None]
        self.cond: List[float] = [0.0]           # raw threshold (float32) once converted
        self.slot_a: List[int] = [0]
        self.slot_b: List[int] = [0]
        self.leaf: List[float] = [0.0]
        self.is_leaf: List[bool] = [True]
        self.default_left: List[bool] = [True]
        self.loss_chg: List[float] = [0.0]
        self.hess_sum: List[float] = [0.0]
        self.sample_cnt: List[int] = [0]
        self.converted = False

    # -- construction -------------------------------------------------------
    @property
    def num_nodes(self) -> int:
        return len(self.left)

    def _alloc(self, parent: int) -> int:
        nid = len(self.left)
        self.left.append(-1); self.right.append(-1); self.parent.append(parent)
        self.feat.append(-1); self.feat_name.append(None); self.cond.append(0.0)
        self.slot_a.append(0); self.slot_b.append(0); self.leaf.append(0.0)
        self.is_leaf.append(True); self.default_left.append(True)
        self.loss_chg.append(0.0); self.hess_sum.append(0.0); self.sample_cnt.append(0)
        return nid

    def add_children(self, nid: int):
        l = self._alloc(nid)
        r = self._alloc(nid)
        self.left[nid] = l
        self.right[nid] = r
        self.is_leaf[nid] = False
        return l, r

    def set_split(self, nid: int, feat: int, a: int, b: int):
        self.feat[nid] = int(feat)
        self.slot_a[nid] = int(a)
        self.slot_b[nid] = int(b)
        # == float32 0.5 * (a + b): bin ids are < 2^24, so the double result is exact
        self.cond[nid] = 0.5 * (int(a) + int(b))
        self.is_leaf[nid] = False

    def set_leaf(self, nid: int, value: float):
        self.is_leaf[nid] = True
        self.left[nid] = -1
        self.right[nid] = -1
        self.leaf[nid] = float(np.float32(value))

    # -- queries ------------------------------------------------------------
    def depth_of(self, nid: int) -> int:
        d = 0
        while self.parent[nid] >= 0:
            nid = self.parent[nid]
            d += 1
        return d

    def max_depth(self) -> int:
        def rec(n):
            if self.is_leaf[n]:
                return 0
            return max(rec(self.left[n]), rec(self.right[n])) + 1
        return rec(0)

    def leaf_count(self) -> int:
        return sum(1 for i in range(self.num_nodes) if self.is_leaf[i])

    def leaf_nodes(self) -> List[int]:
        return [i for i in range(self.num_nodes) if self.is_leaf[i]]

    def bin_arrays(self):
        """Arrays for the training scorer: go left iff bin <= floor((a+b)/2)."""
        n = self.num_nodes
        feat = np.array([(-1 if self.is_leaf[i] else self.feat[i]) for i in range(n)], np.int32)
        thr = np.array([(self.slot_a[i] + self.slot_b[i]) // 2 for i in range(n)], np.int32)
        return (feat, thr, np.array(self.left, np.int32), np.array(self.right, np.int32),
                np.array(self.leaf, np.float32))

    def raw_arrays(self):
        n = self.num_nodes
        feat = np.array([(-1 if self.is_leaf[i] else self.feat[i]) for i in range(n)], np.int32)
        return (feat, np.array(self.cond, np.float32), np.array(self.left, np.int32),
                np.array(self.right, np.int32), np.array(self.default_left, np.uint8),
                np.array(self.leaf, np.float32))

    def predict_one(self, x: Dict[str, float]) -> int:
        """Leaf index for a name->value map (missing -> default child)."""
        n = 0
        while not self.is_leaf[n]:
            v = x.get(self.feat_name[n])
            if v is None or v != v:
                n = self.left[n] if self.default_left[n] else self.right[n]
            else:
                n = self.left[n] if np.float32(v) <= np.float32(self.cond[n]) else self.right[n]
        return n

    # -- conversions ----------------------------------------------------------
    def convert_split_values(self, cand_sorted: Sequence[np.ndarray], split_type: str = "mean"):
        for i in range(self.num_nodes):
            if self.is_leaf[i]:
                continue
            c = cand_sorted[self.feat[i]]
            if c.dtype != np.float32:
                c = c.astype(np.float32)
            a, b = self.slot_a[i], self.slot_b[i]
            if split_type == "mean":
                v = np.float32(0.5) * (c[a] + c[b])
            else:
                s = a + b
                v = c[s // 2] if s % 2 == 0 else np.float32(0.5) * (c[(s - 1) // 2] + c[(s + 1) // 2])
            self.cond[i] = float(np.float32(v))
        self.converted = True

    def add_feature_names(self, index2name: Sequence[str]):
        for i in range(self.num_nodes):
            if not self.is_leaf[i]:
                self.feat_name[i] = index2name[self.feat[i]]

    def update_feature_index(self, name2index: Dict[str, int]):
        for i in range(self.num_nodes):
            if not self.is_leaf[i]:
                idx = name2index.get(self.feat_name[i])
                if idx is None:
                    raise KeyError(f"[GBDT] can't find feature index for feature name({self.feat_name[i]})")
                self.feat[i] = idx

    def add_default_direction(self, fill: Optional[np.ndarray]):
        if fill is None or len(fill) == 0:
            return
        for i in range(self.num_nodes):
            if not self.is_leaf[i]:
                self.default_left[i] = bool(np.float32(fill[self.feat[i]]) < np.float32(self.cond[i]))

    # -- text format ----------------------------------------------------------
    def dump(self, it: int, with_stats: bool = True) -> str:
        out = [f"booster[{it + 1}] depth={self.max_depth()},node_num={self.num_nodes},leaf_cnt={self.leaf_count()}\n"]

        def rec(n, d):
            ind = "\t" * d
            if self.is_leaf[n]:
                s = f"{ind}{n}:leaf={java_float_str(self.leaf[n])}"
                if with_stats:
                    s += f",hess_sum={java_float_str(self.hess_sum[n])},sample_cnt={int(self.sample_cnt[n])}"
                out.append(s + "\n")
            else:
                dc = self.left[n] if self.default_left[n] else self.right[n]
                s = (f"{ind}{n}:[f_{self.feat_name[n]}<={java_float_str(self.cond[n])}] "
                     f"yes={self.left[n]},no={self.right[n]},missing={dc}")
                if with_stats:
                    s += (f",gain={java_float_str(self.loss_chg[n])},hess_sum={java_float_str(self.hess_sum[n])}"
                          f",sample_cnt={int(self.sample_cnt[n])}")
                out.append(s + "\n")
                rec(self.left[n], d + 1)
                rec(self.right[n], d + 1)

        rec(0, 0)
        return "".join(out)

    @classmethod
    def parse(cls, header: str, lines: List[str]) -> "Tree":
        node_num = int(header.strip().split(",")[1].split("=")[1])
        t = cls()
        for _ in range(node_num - 1):
            t._alloc(-1)
        for line in lines:
            s = line.strip()
            if "leaf" in s:
                m = LEAF_RE.search(s) or LEAF_NOSTAT_RE.search(s)
                nid = int(m.group(1))
                t.set_leaf(nid, parse_java_float(m.group(2)))
                if m.re is LEAF_RE:
                    t.hess_sum[nid] = parse_java_float(m.group(3))
                    t.sample_cnt[nid] = int(m.group(4))
            else:
                m = INNER_RE.search(s) or INNER_NOSTAT_RE.search(s)
                nid = int(m.group(1))
                l, r, miss = int(m.group(4)), int(m.group(5)), int(m.group(6))
                t.is_leaf[nid] = False
                t.left[nid], t.right[nid] = l, r
                t.parent[l] = nid
                t.parent[r] = nid
                t.feat_name[nid] = m.group(2)
                t.cond[nid] = float(np.float32(parse_java_float(m.group(3))))
                t.default_left[nid] = miss == l
                if m.re is INNER_RE:
                    t.loss_chg[nid] = parse_java_float(m.group(7))
                    t.hess_sum[nid] = parse_java_float(m.group(8))
                    t.sample_cnt[nid] = int(m.group(9))
        t.converted = True
        return t


class GBDTModel:
    """Header + trees (tree index = round * class_num + class)."""

    def __init__(self, base_prediction: float = 0.0, class_num: int = 1, loss_name: str = ""):
        self.base_prediction = float(np.float32(base_prediction))
        self.class_num = int(class_num)
        self.loss_name = loss_name
        self.trees: List[Tree] = []

    def dump_lines(self, with_stats: bool = True) -> List[str]:
        head = (f"uniform_base_prediction={java_float_str(self.base_prediction)}\n"
                f"class_num={self.class_num}\nloss_function={self.loss_name}\ntree_num={len(self.trees)}\n")
        return [head] + [t.dump(i, with_stats) for i, t in enumerate(self.trees)]

    def dumps(self, with_stats: bool = True) -> str:
        return "".join(self.dump_lines(with_stats))

    @classmethod
    def loads(cls, text: str) -> "GBDTModel":
        lines = text.splitlines()
        i = 0

        def nxt():
            nonlocal i
            while i < len(lines) and lines[i].strip() == "":
                i += 1
            s = lines[i]
            i += 1
            return s

        m = cls(parse_java_float(nxt().split("=")[1]), int(nxt().split("=")[1]), nxt().split("=")[1].strip())
        ntree = int(nxt().split("=")[1])
        if ntree == 0:
            raise ValueError("GBDT: load model error, tree number is 0!")
        for _ in range(ntree):
            header = nxt()
            nn = int(header.strip().split(",")[1].split("=")[1])
            body = [nxt() for _ in range(nn)]
            m.trees.append(Tree.parse(header, body))
        return m

    def feature_dict(self) -> Dict[str, int]:
        d: Dict[str, int] = {}
        for t in self.trees:
            for i in range(t.num_nodes):
                if not t.is_leaf[i] and t.feat_name[i] not in d:
                    d[t.feat_name[i]] = len(d)
        return d

    def feature_importance(self) -> Dict[str, List[float]]:
        imp: Dict[str, List[float]] = {}
        for t in self.trees:
            for i in range(t.num_nodes):
                if t.is_leaf[i]:
                    continue
                e = imp.setdefault(t.feat_name[i], [0, 0.0])
                e[0] += 1
                e[1] += float(np.float32(t.loss_chg[i]))
        return imp

    def flatten(self, n_round: Optional[int] = None):
        """Flatten trees to SoA arrays for the forest kernel."""
        trees = self.trees if n_round is None else self.trees[: n_round * self.class_num]
        feats, conds, lefts, rights, defl, vals, roots, outs = [], [], [], [], [], [], [], []
        off = 0
        for ti, t in enumerate(trees):
            f, c, l, r, d, v = t.raw_arrays()
            feats.append(f); conds.append(c)
            lefts.append(np.where(l >= 0, l + off, -1).astype(np.int32))
            rights.append(np.where(r >= 0, r + off, -1).astype(np.int32))
            defl.append(d); vals.append(v)
            roots.append(off); outs.append(ti % self.class_num)
            off += t.num_nodes
        cat = (lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt))
        return {
            "nfeat": cat(feats, np.int32), "nthr": cat(conds, np.float32),
            "nleft": cat(lefts, np.int32), "nright": cat(rights, np.int32),
            "ndefl": cat(defl, np.uint8), "nval": cat(vals, np.float32),
            "troot": np.array(roots, np.int32), "tout": np.array(outs, np.int32),
        }
