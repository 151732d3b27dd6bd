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


class CandTable:
    """Sorted split candidates of every feature, concatenated (float32) + offsets, for
    vectorised slot -> threshold conversion (FeatureSplitType.java:32-78)."""

    def __init__(self, cands: Sequence[np.ndarray]):
        cands = [np.asarray(c, np.float32) for c in cands]
        self.cat = np.concatenate(cands).astype(np.float32) if cands else np.zeros(0, np.float32)
        self.off = np.concatenate([[0], np.cumsum([len(c) for c in cands])]).astype(np.int64)

    def split_values(self, f: np.ndarray, a: np.ndarray, b: np.ndarray, split_type: str) -> np.ndarray:
        base = self.off[f]
        c = self.cat
        if split_type == "mean":
            return np.float32(0.5) * (c[base + a] + c[base + b])
        s = a + b
        even = (s & 1) == 0
        lo = np.where(even, s >> 1, (s - 1) >> 1)
        hi = np.where(even, s >> 1, (s + 1) >> 1)
        return np.where(even, c[base + lo], np.float32(0.5) * (c[base + lo] + c[base + hi])).astype(np.float32)


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
        isl = np.asarray(self.is_leaf, bool)
        feat = np.where(isl, -1, np.asarray(self.feat, np.int32)).astype(np.int32)
        thr = ((np.asarray(self.slot_a, np.int64) + np.asarray(self.slot_b, np.int64)) // 2).astype(np.int32)
        return (feat, thr, np.asarray(self.left, np.int32), np.asarray(self.right, np.int32),
                np.asarray(self.leaf, np.float32))

    def raw_arrays(self):
        isl = np.asarray(self.is_leaf, bool)
        feat = np.where(isl, -1, np.asarray(self.feat, np.int32)).astype(np.int32)
        return (feat, np.asarray(self.cond, np.float32), np.asarray(self.left, np.int32),
                np.asarray(self.right, np.int32), np.asarray(self.default_left, np.uint8),
                np.asarray(self.leaf, np.float32))

    def _inner(self) -> np.ndarray:
        return np.flatnonzero(~np.asarray(self.is_leaf, bool))

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
    def convert_split_values(self, cand_sorted, split_type: str = "mean"):
        """Bin-slot interval -> raw float32 threshold for every inner node (vectorised).
        ``cand_sorted``: a :class:`CandTable` or a per-feature list of sorted candidates."""
        tab = cand_sorted if isinstance(cand_sorted, CandTable) else CandTable(cand_sorted)
        inner = self._inner()
        if inner.size:
            f = np.asarray(self.feat, np.int64)[inner]
            a = np.asarray(self.slot_a, np.int64)[inner]
            b = np.asarray(self.slot_b, np.int64)[inner]
            cond = np.asarray(self.cond, np.float64)
            cond[inner] = tab.split_values(f, a, b, split_type)
            self.cond = cond.tolist()
        self.converted = True

    def add_feature_names(self, index2name: Sequence[str]):
        inner = self._inner()
        if inner.size:
            names = index2name if isinstance(index2name, np.ndarray) else np.asarray(index2name, dtype=object)
            fn = np.asarray(self.feat_name, dtype=object)
            fn[inner] = names[np.asarray(self.feat, np.int64)[inner]]
            self.feat_name = fn.tolist()

    def update_feature_index(self, name2index: Dict[str, int]):
        for i in range(self.num_nodes):
            if not self.is_leaf[i]:
                idx = name2index.get(self.feat_name[i])
                if idx is None:
                    raise KeyError(f"[GBDT] can't find feature index for feature name({self.feat_name[i]})")
                self.feat[i] = idx

    def add_default_direction(self, fill: Optional[np.ndarray]):
        """Missing values go left iff fill < cond (Tree.java:357-375), float32 compare."""
        if fill is None or len(fill) == 0:
            return
        inner = self._inner()
        if inner.size:
            f32 = np.asarray(fill, np.float32)
            dl = np.asarray(self.default_left, bool)
            dl[inner] = f32[np.asarray(self.feat, np.int64)[inner]] < np.asarray(self.cond, np.float32)[inner]
            self.default_left = dl.tolist()

    @classmethod
    def from_arrays(cls, left, right, feat, slot_a, slot_b, leaf, is_leaf, loss_chg, hess_sum,
                    sample_cnt) -> "Tree":
        """Build a tree from per-node numpy arrays (node ids = array positions) without a
        per-node Python loop. ``leaf`` values are float32; inner nodes get cond = (a+b)/2."""
        n = len(left)
        isl = np.asarray(is_leaf, bool)
        left = np.where(isl, -1, np.asarray(left, np.int64))
        right = np.where(isl, -1, np.asarray(right, np.int64))
        parent = np.full(n, -1, np.int64)
        inner = np.flatnonzero(~isl)
        parent[left[inner]] = inner
        parent[right[inner]] = inner
        a = np.where(isl, 0, np.asarray(slot_a, np.int64))
        b = np.where(isl, 0, np.asarray(slot_b, np.int64))
        t = cls.__new__(cls)
        t.left, t.right, t.parent = left.tolist(), right.tolist(), parent.tolist()
        t.feat = np.where(isl, -1, np.asarray(feat, np.int64)).tolist()
        t.feat_name = [None] * n
        t.cond = (0.5 * (a + b)).tolist()
        t.slot_a, t.slot_b = a.tolist(), b.tolist()
        t.leaf = np.where(isl, np.asarray(leaf, np.float32), np.float32(0)).astype(np.float64).tolist()
        t.is_leaf = isl.tolist()
        t.default_left = [True] * n
        t.loss_chg = np.asarray(loss_chg, np.float32).astype(np.float64).tolist()
        t.hess_sum = np.asarray(hess_sum, np.float32).astype(np.float64).tolist()
        t.sample_cnt = np.asarray(sample_cnt, np.int64).tolist()
        t.converted = False
        return t

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
