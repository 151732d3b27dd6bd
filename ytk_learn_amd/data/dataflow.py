"""Data ingest: sharded read -> native parse -> global dictionary -> CSR on device.

Reference: ``J/dataflow/DataFlow.java`` (loadFlow :468-764, loadDict :244-285,
reduceFeature :294-378, getAssignedDatas :391-410, handleLocalIdx :413-446,
replaceFeatureTransform :448-466) and ``J/dataflow/CoreData.java`` (globalSync :613-645).

Pipeline per rank (one process per GPU):
  1. pick this rank's input: ``assigned`` (the path is already this rank's shard),
     ``files_avg`` (contiguous slice of the sorted file list) or ``lines_avg``
     (line i goes to rank i mod world; done inside the native parser);
  2. optional user line transform ``transform(bytes) -> [str]`` (reference: Jython hook,
     ``bin/transform.py``) -- here plain CPython, applied before the native parser;
  3. native multithreaded parse (``csrc/native/parser.cpp``) -> local dictionary + CSR;
  4. global sync: row/weight/error counts (one batched allreduce), feature counts
     (object allgather + merge), optional transform stats;
  5. dictionary: user dict file, or count-filtered names sorted lexicographically with
     the bias at index 0 (TreeSet order, DataFlow.java:296-327);
  6. remap local ids -> global ids (dropping filtered / unknown names), append the bias
     column (CoreData.java:424-428), apply feature transforms.
"""
from __future__ import annotations

import importlib.util
import math
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..config.params import DataParams, FeatureParams
from ..io.fs import FileSystem
from ..utils.errors import YtkLearnError
from ..utils.javafmt import java_double_str

TRANSFORM_STAT_SUFFIX = "_feature_transform_stat"


def _native():
    from ..ops._ext import native  # built in-tree by csrc/build.py
    return native()


# ---------------------------------------------------------------------------
# raw parse
# ---------------------------------------------------------------------------
@dataclass
class RawShard:
    """Output of the native parser for one rank (local dictionary ids)."""
    n_rows: int
    weight: np.ndarray
    label_ptr: np.ndarray
    labels: np.ndarray
    init_ptr: np.ndarray
    init: np.ndarray
    indptr: np.ndarray
    feat: np.ndarray
    val: np.ndarray
    field: np.ndarray
    names: List[str]
    counts: np.ndarray
    stats: Optional[Dict[str, np.ndarray]]
    fields: List[str]
    n_lines: int = 0
    n_errors: int = 0

    @classmethod
    def from_native(cls, r: dict, want_stats: bool) -> "RawShard":
        st = None
        if want_stats:
            st = {k: r["st_" + k] for k in ("sum", "sum2", "max", "min")}
        return cls(int(r["n_rows"]), r["weight"], r["label_ptr"], r["labels"], r["init_ptr"], r["init"],
                   r["indptr"], r["feat"], r["val"], r["field"], list(r["names"]), r["counts"], st,
                   list(r["fields"]), int(r["n_lines"]), int(r["n_errors"]))


def load_transform_fn(path: Optional[str]) -> Optional[Callable[[bytes], List[str]]]:
    """User line transform (reference ``bin/transform.py``: ``transform(bytes) -> list``)."""
    if not path:
        return None
    spec = importlib.util.spec_from_file_location("ytk_user_transform", path)
    if spec is None or spec.loader is None:
        raise YtkLearnError(f"cannot load python transform script {path}")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if not hasattr(mod, "transform"):
        raise YtkLearnError(f"python transform script {path} has no transform(line) function")
    return mod.transform


def assigned_paths(fs: FileSystem, data_path: str, dp: DataParams, rank: int, world: int) -> Tuple[List[str], int, int]:
    """Files this rank reads and the (line_mod, line_rem) line filter (DataFlow.java:391-410)."""
    paths = fs.recur_get_paths([p.strip() for p in data_path.split(",") if p.strip()])
    if dp.assigned or world <= 1:
        return paths, 1, 0
    if dp.unassigned_mode == "files_avg":
        paths = sorted(paths)
        base, rem = divmod(len(paths), world)
        start = rank * base + min(rank, rem)
        end = start + base + (1 if rank < rem else 0)
        return paths[start:end], 1, 0
    return paths, world, rank  # lines_avg


def parse_paths(fs: FileSystem, paths: Sequence[str], opts: dict, transform=None,
                line_mod: int = 1, line_rem: int = 0) -> dict:
    nat = _native()
    opts = dict(opts)
    opts["line_mod"], opts["line_rem"] = line_mod, line_rem
    local = [fs.local_path(p) for p in paths]
    if transform is None and all(lp is not None for lp in local):
        return nat.parse_files(list(local), opts)
    # transform hook / remote FS: build the buffer in Python, sharding applied first
    chunks: List[bytes] = []
    li = 0
    for p in paths:
        with fs.open_read(p, binary=True) as f:
            for raw in f:
                keep = (li % line_mod) == line_rem
                li += 1
                if not keep:
                    continue
                raw = raw.rstrip(b"\r\n")
                if transform is not None:
                    for out in transform(raw) or []:
                        s = out if isinstance(out, str) else bytes(out).decode("utf-8")
                        chunks.append(s.encode("utf-8"))
                else:
                    chunks.append(raw)
    opts["line_mod"], opts["line_rem"] = 1, 0
    return nat.parse_buffer(b"\n".join(chunks) + b"\n", opts)


def parse_options(dp: DataParams, fp: Optional[FeatureParams], *, max_error_tol: int,
                  y_sampling: Optional[Dict[int, float]] = None, split_field: bool = False,
                  want_stats: bool = False, seed: int = 0, threads: int = 0) -> dict:
    d = dp.delim
    o = {"x_delim": d.x_delim, "y_delim": d.y_delim, "features_delim": d.features_delim,
         "feature_name_val_delim": d.feature_name_val_delim, "field_delim": d.field_delim,
         "max_error_tol": int(max_error_tol), "split_field": bool(split_field),
         "want_stats": bool(want_stats), "sample_seed": int(seed) & ((1 << 63) - 1), "threads": int(threads)}
    if fp is not None and fp.feature_hash.need_feature_hash:
        o.update(feature_hash=True, hash_bucket=int(fp.feature_hash.bucket_size),
                 hash_seed=int(fp.feature_hash.seed) & 0xffffffff, hash_prefix=fp.feature_hash.feature_prefix)
    if y_sampling:
        n = max(y_sampling) + 1
        rates = [1.0] * n
        for k, v in y_sampling.items():
            rates[k] = float(v)
        o["y_sampling"] = rates
    return o


# ---------------------------------------------------------------------------
# global dictionary
# ---------------------------------------------------------------------------
def read_dict_files(fs: FileSystem, dict_path: str) -> List[str]:
    names: List[str] = []
    for p in sorted(fs.recur_get_paths([dict_path])):
        for line in fs.read_lines(p):
            s = line.strip()
            if s:
                names.append(s)
    return names


def build_dictionary(shard: RawShard, comm, filter_threshold: int, need_bias: bool, bias_name: str,
                     user_names: Optional[List[str]] = None) -> Tuple[Dict[str, int], List[str]]:
    """name -> global index and the index -> name list (bias at 0 when need_bias)."""
    if user_names is not None:
        names = [bias_name] if need_bias else []
        seen = set(names)
        for n in user_names:
            if n not in seen:
                seen.add(n)
                names.append(n)
        return {n: i for i, n in enumerate(names)}, names
    if comm is not None and comm.is_dist:
        # hash-partitioned keyed reduction (CoreData.java:628 allreduceMap of feature counts)
        nm, cnt = comm.merge_named(list(shard.names), np.asarray(shard.counts, np.float64), ["sum"])
        keep = [n for n, c in zip(nm, cnt[:, 0].tolist()) if c >= filter_threshold]
    else:
        local = dict(zip(shard.names, shard.counts.tolist()))
        keep = sorted(n for n, c in local.items() if c >= filter_threshold)
    if need_bias:
        keep = [n for n in keep if n != bias_name]
        names = [bias_name] + keep
    else:
        names = keep
    return {n: i for i, n in enumerate(names)}, names


# ---------------------------------------------------------------------------
# feature transforms (CoreData.FeatureStat / TransformNode, CoreData.java:106-220)
# ---------------------------------------------------------------------------
@dataclass
class TransformNode:
    mode: str
    mean: float
    stdvar: float
    max: float
    min: float
    range_max: float
    range_min: float

    def apply(self, v: np.ndarray) -> np.ndarray:
        v = v.astype(np.float64)
        if self.mode == "standardization":
            if self.stdvar < 0.000001:
                return v.astype(np.float32)
            return ((v - self.mean) / self.stdvar).astype(np.float32)
        if abs(self.max - self.min) < 0.000001:
            return np.ones_like(v, dtype=np.float32)
        return (self.range_min + (self.range_max - self.range_min) * ((v - self.min) / (self.max - self.min))
                ).astype(np.float32)

    def to_line(self) -> str:
        j = java_double_str
        return (f"mode={self.mode}, mean={j(self.mean)}, stdvar={j(self.stdvar)}, max={j(self.max)}, "
                f"min={j(self.min)}, rangeMax={j(self.range_max)}, rangeMin={j(self.range_min)}")

    @classmethod
    def from_line(cls, s: str) -> "TransformNode":
        kv = {}
        for part in s.split(","):
            k, v = part.split("=")
            kv[k.strip()] = v.strip()
        return cls(kv["mode"].lower(), float(kv["mean"]), float(kv["stdvar"]), float(kv["max"]),
                   float(kv["min"]), float(kv["rangeMax"]), float(kv["rangeMin"]))


def merge_stats(shard: RawShard, comm) -> Dict[str, Tuple[int, float, float, float, float]]:
    st = shard.stats
    local = {n: (int(c), float(st["sum"][i]), float(st["sum2"][i]), float(st["max"][i]), float(st["min"][i]))
             for i, (n, c) in enumerate(zip(shard.names, shard.counts.tolist()))}

    if comm is None or not comm.is_dist:
        return local
    # hash-partitioned keyed reduction (CoreData.java:632 allreduceMap of FeatureStat)
    names = list(local)
    rows = np.array([local[n] for n in names], np.float64).reshape(len(names), 5)
    nm, red = comm.merge_named(names, rows, ["sum", "sum", "sum", "max", "min"])
    return {n: (int(r[0]), float(r[1]), float(r[2]), float(r[3]), float(r[4])) for n, r in zip(nm, red.tolist())}


def make_transform_nodes(stats, names: List[str], fp: FeatureParams, need_bias: bool, bias_name: str
                         ) -> Dict[str, TransformNode]:
    tp = fp.transform
    cand = [n for n in names if not (need_bias and n == bias_name)]
    if tp.include:
        target = list(tp.include)
    elif tp.exclude:
        target = [n for n in cand if n not in tp.exclude]
    else:
        target = cand
    out = {}
    for n in target:
        if n not in stats:
            continue
        c, s, s2, mx, mn = stats[n]
        mean = s / c
        out[n] = TransformNode(tp.mode, mean, math.sqrt(max(s2 / c - mean * mean, 0.0)), mx, mn, tp.scale_max,
                               tp.scale_min)
    return out


def write_transform_stats(fs: FileSystem, path: str, nodes: Dict[str, TransformNode]):
    with fs.open_write(path) as f:
        for n, node in nodes.items():
            f.write(f"{n}###{node.to_line()}\n")


def read_transform_stats(fs: FileSystem, path: str) -> Dict[str, TransformNode]:
    out = {}
    if not fs.exists(path):
        return out
    for line in fs.read_lines(path):
        if "###" not in line:
            continue
        n, rest = line.split("###", 1)
        out[n] = TransformNode.from_line(rest)
    return out


# ---------------------------------------------------------------------------
# final CSR dataset
# ---------------------------------------------------------------------------
@dataclass
class SparseData:
    """One rank's rows, global feature ids, on a device. Bias (if any) is column 0."""
    indptr: torch.Tensor          # int64 [n+1]
    indices: torch.Tensor         # int32 [nnz]
    values: torch.Tensor          # float32 [nnz]
    y: torch.Tensor               # float32 [n, ylen]
    weight: torch.Tensor          # float32 [n]
    fields: Optional[torch.Tensor] = None  # int32 [nnz] (ffm)
    init: Optional[torch.Tensor] = None    # float32 [n, k] (sample-dependent base prediction)
    real_num: float = 0.0         # global row count
    weight_sum: float = 0.0       # global weight sum
    local_weight_sum: float = 0.0
    n_errors: int = 0
    label_counts: Optional[np.ndarray] = None

    @property
    def n(self) -> int:
        return int(self.weight.shape[0])

    @property
    def nnz(self) -> int:
        return int(self.indices.shape[0])

    def to(self, device) -> "SparseData":
        mv = lambda t: t.to(device) if t is not None else None
        return SparseData(mv(self.indptr), mv(self.indices), mv(self.values), mv(self.y), mv(self.weight),
                          mv(self.fields), mv(self.init), self.real_num, self.weight_sum, self.local_weight_sum,
                          self.n_errors, self.label_counts)


def labels_matrix(shard: RawShard, width: int, class_ids: bool = False, allow_empty: bool = False) -> np.ndarray:
    """[n, width] label matrix. With ``class_ids`` a single label per row is a class index that
    is one-hot encoded (multiclass: a class id or a K-vector, MulticlassLinearModelDataFlow.java:104-151)."""
    n = shard.n_rows
    cnt = np.diff(shard.label_ptr)
    out = np.zeros((n, width), np.float32)
    if n == 0:
        return out
    if width == 1:
        bad = cnt < 1
        if bad.any() and not allow_empty:
            raise YtkLearnError("rows without label in training data")
        has = ~bad
        out[has, 0] = shard.labels[shard.label_ptr[:-1][has]]
        return out
    single = cnt == 1
    if single.any():
        if not class_ids:
            raise YtkLearnError(f"expected {width} labels per row")
        ids = shard.labels[shard.label_ptr[:-1][single]].astype(np.int64)
        if (ids < 0).any() or (ids >= width).any():
            raise YtkLearnError(f"class id out of range [0, {width})")
        rows = np.nonzero(single)[0]
        out[rows, ids] = 1.0
    multi = cnt == width
    if multi.any():
        rows = np.nonzero(multi)[0]
        starts = shard.label_ptr[:-1][multi]
        out[rows] = shard.labels[starts[:, None] + np.arange(width)[None, :]]
    bad = ~(single | multi)
    if bad.any() and not (allow_empty and (cnt[bad] == 0).all()):
        raise YtkLearnError(f"label count must be 1 (class id) or {width}")
    return out


def init_matrix(shard: RawShard, width: int) -> Optional[np.ndarray]:
    cnt = np.diff(shard.init_ptr)
    if shard.init.size == 0:
        return None
    if not (cnt == width).all():
        raise YtkLearnError(f"init prediction must have {width} value(s) per row")
    return shard.init.reshape(-1, width).astype(np.float32)


def remap_csr(shard: RawShard, name2idx: Dict[str, int], need_bias: bool,
              transforms: Optional[Dict[int, TransformNode]] = None,
              field_map: Optional[Dict[str, int]] = None, bias_field: int = 0):
    """Local ids -> global ids (unknown names dropped), bias appended, transforms applied."""
    lut = np.array([name2idx.get(n, -1) for n in shard.names], dtype=np.int64) if shard.names else \
        np.zeros(0, np.int64)
    gid = lut[shard.feat.astype(np.int64)] if shard.feat.size else np.zeros(0, np.int64)
    keep = gid >= 0
    if need_bias:
        keep &= gid != 0  # a feature literally named like the bias is the bias
    rows = np.repeat(np.arange(shard.n_rows, dtype=np.int64), np.diff(shard.indptr))
    rows, gid, val = rows[keep], gid[keep], shard.val[keep].astype(np.float32)
    fld = None
    if field_map is not None:
        flut = np.array([field_map.get(f, -1) for f in shard.fields], dtype=np.int64) if shard.fields else \
            np.zeros(0, np.int64)
        fld = flut[shard.field.astype(np.int64)][keep] if shard.field.size else np.zeros(0, np.int64)
        ok = fld >= 0
        rows, gid, val, fld = rows[ok], gid[ok], val[ok], fld[ok]
    if transforms:
        tidx = np.array(sorted(transforms), dtype=np.int64)
        hit = np.isin(gid, tidx)
        if hit.any():
            order = np.argsort(gid[hit], kind="stable")
            hv = val[hit][order]
            hg = gid[hit][order]
            out = np.empty_like(hv)
            bounds = np.searchsorted(hg, tidx, side="left"), np.searchsorted(hg, tidx, side="right")
            for t, a, b in zip(tidx, *bounds):
                if b > a:
                    out[a:b] = transforms[int(t)].apply(hv[a:b])
            tmp = np.empty_like(hv)
            tmp[order] = out
            val[hit] = tmp
    if need_bias:
        n = shard.n_rows
        rows = np.concatenate([rows, np.arange(n, dtype=np.int64)])
        gid = np.concatenate([gid, np.zeros(n, np.int64)])
        val = np.concatenate([val, np.ones(n, np.float32)])
        if fld is not None:
            fld = np.concatenate([fld, np.full(n, bias_field, np.int64)])
    order = np.argsort(rows, kind="stable")
    rows, gid, val = rows[order], gid[order], val[order]
    if fld is not None:
        fld = fld[order]
    indptr = np.zeros(shard.n_rows + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=shard.n_rows), out=indptr[1:])
    return indptr, gid.astype(np.int32), val, (fld.astype(np.int32) if fld is not None else None)


def to_sparse_data(shard: RawShard, name2idx, need_bias, ylen, device, comm, *, class_ids=False,
                   allow_empty_label=False, init_width=0, transforms=None, field_map=None, bias_field=0
                   ) -> SparseData:
    indptr, idx, val, fld = remap_csr(shard, name2idx, need_bias, transforms, field_map, bias_field)
    y = labels_matrix(shard, ylen, class_ids, allow_empty_label)
    w = shard.weight.astype(np.float32)
    init = init_matrix(shard, init_width) if init_width > 0 else None
    local_w = float(w.astype(np.float64).sum())
    sums = [float(shard.n_rows), local_w, float(shard.n_errors)]
    if comm is not None and comm.is_dist:
        sums = comm.allreduce_scalars(sums)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dtype=dt, device=device)
    return SparseData(t(indptr, torch.int64), t(idx, torch.int32), t(val, torch.float32), t(y, torch.float32),
                      t(w, torch.float32), t(fld, torch.int32) if fld is not None else None,
                      t(init, torch.float32) if init is not None else None, sums[0], sums[1], local_w,
                      int(sums[2]))
