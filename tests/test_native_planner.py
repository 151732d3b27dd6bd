"""Native leaf-wise planner (csrc/native/leafwise.cpp): launch packs against the Python
chunking they replace, and the slot pool / LRU bookkeeping in isolation (CPU)."""
import numpy as np
import pytest

from ytk_learn_amd.models.gbdt.builder import TreeBuilder, _chunk_segments
from ytk_learn_amd.ops import gbdt as gops
from ytk_learn_amd.ops._ext import native


def _rec(loss, feat=0, a=3, b=4, g=1.0, h=100.0, gl=0.4, hl=50.0):
    r = np.zeros(1, gops.SPLIT_DTYPE)
    r["loss_chg"], r["feat"], r["bin_a"], r["bin_b"] = loss, feat, a, b
    r["g"], r["h"], r["gl"], r["hl"] = g, h, gl, hl
    return r


def _grower(n_slots=16, max_leaf=8, speculate=True):
    nat = native()
    p = nat.LwParams()
    p.max_leaf, p.max_depth, p.min_split_samples = max_leaf, -1, -1
    p.min_split_loss, p.mcw, p.l1, p.l2, p.max_abs_leaf, p.mcw2 = 0.0, 1.0, 0.0, 0.0, -1.0, 2.0
    p.lr, p.speculate = 0.1, speculate
    return nat.LeafGrower(p, n_slots)


def test_root_batch_and_partition_pack_match_python_chunking():
    g = _grower()
    assert g.root(10000, 10000) == 0  # first free slot
    g.apply_recs(np.zeros(1, np.int32), _rec(5.0, feat=2, a=7, b=9))
    batch = g.replay()
    assert batch == [0]
    splits, counts_only = g.expand(batch)
    assert splits == [0] and counts_only == []
    arr, off, nitems, nblocks = g.pack_partition(splits, gops.PART_CHUNK, TreeBuilder.TARGET_BLOCKS,
                                                 TreeBuilder.MIN_ROWS_PER_BLOCK)
    begins, counts = np.array([0]), np.array([10000])
    ch = max(TreeBuilder.MIN_ROWS_PER_BLOCK, -(-10000 // TreeBuilder.TARGET_BLOCKS))
    seg, s, e, k, _, _ = _chunk_segments(begins, counts, ch)
    items = np.stack([seg, s, e, k], axis=1).astype(np.int32).reshape(-1)
    assert nitems * 4 == len(items) and np.array_equal(arr[off[0]:off[1]], items)
    assert arr[off[1]] == 2 and arr[off[2]] == 8  # feat, thr = (7 + 9) // 2
    assert arr[off[3]] == 0 and arr[off[4]] == 10000 and arr[off[5]] == 0
    assert nblocks == -(-10000 // gops.PART_CHUNK) and list(arr[off[6]:off[6] + 2]) == [1, nblocks]


def test_hist_plan_builds_small_child_and_derives_large():
    g = _grower()
    g.root(10000, 10000)
    g.apply_recs(np.zeros(1, np.int32), _rec(5.0))
    splits, _ = g.expand(g.replay())
    g.set_children(splits, np.array([3000]), np.array([3000]), True)
    order, nb, arr, off, nwork = g.plan_hist_packed(splits, TreeBuilder.TARGET_BLOCKS,
                                                    TreeBuilder.MIN_ROWS_PER_BLOCK)
    assert nb == 1 and order == [1, 2]  # left child (3000 rows) is the smaller one
    items = arr[off[1]:off[2]].reshape(-1, 4)
    built, derived = items[0], items[1]
    assert built[3] == 0 and derived[3] == 1
    assert derived[1] == 0 and derived[2] == built[0]  # parent slot 0, sibling = built slot
    work = arr[off[0]:off[1]].reshape(-1, 4)
    assert work[:, 0].tolist() == [built[0]] * nwork and work[0, 1] == 0 and work[-1, 2] == 3000


def test_pool_exhaustion_raises():
    """Parents of derived children are pinned; with no evictable slot left the planner
    raises (the reference's pool-too-small condition) instead of corrupting a histogram."""
    g = _grower(n_slots=3)
    g.root(10000, 10000)
    g.apply_recs(np.zeros(1, np.int32), _rec(5.0))
    b = g.replay()
    splits, _ = g.expand(b)
    g.set_children(splits, np.array([4000]), np.array([4000]), True)
    order, nb, arr, off, nwork = g.plan_hist_packed(splits, 256, 2048)
    g.apply_recs(np.asarray(order, np.int32), np.concatenate([_rec(3.0), _rec(2.0)]))
    g.release_batch(b)
    b2 = g.replay()
    assert b2 == [1] and g.hist_miss == 0  # no slack for speculation with 1 free slot
    splits2, _ = g.expand([1, 2])  # force both: 4 slots needed, 1 free, both parents pinned
    g.set_children(splits2, np.full(2, 1000), np.full(2, 1000), True)
    with pytest.raises(RuntimeError):
        g.plan_hist_packed(splits2, 256, 2048)
