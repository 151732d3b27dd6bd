"""L1 leaf refinement (TreeRefiner.java:72-254) on the device vs the host summaries.

The per-leaf entry arrays + seg_median rule must give, for every leaf, exactly
  * exact mode: the sorted weighted median (_weighted_median_sorted), and
  * approximate mode: WQSummary::query(W / 2) of the native summary built from the leaf's
    rows and pruned to ``size`` entries (csrc/native/wquantile.cpp),
on the CPU fallback and (GPU) in the HIP kernels.
"""
import numpy as np
import pytest
import torch

from ytk_learn_amd.models.gbdt import refine as rf
from ytk_learn_amd.utils import quantile as wq


def _case(seed, n=6000, leaves=9, ties=True):
    g = np.random.default_rng(seed)
    leaf = g.integers(0, leaves, n)
    leaf[leaf == 4] = 5  # leaf 4 empty
    v = np.round(g.normal(size=n) * 4, 1 if ties else 6)
    v[leaf == 2] = 1.5  # one distinct value
    w = g.integers(1, 4, n).astype(np.float64)  # integer weights: every rank sum exact
    return leaf, v, w


def _check(leaf, v, w, n_nodes, exact, size, dev="cpu"):
    lt = torch.from_numpy(leaf).to(dev)
    ent = rf.leaf_entries(lt, torch.from_numpy(v).to(dev), torch.from_numpy(w).to(dev), n_nodes)
    got = rf.seg_median(*ent, exact=exact, size=size).cpu().numpy()
    for s in range(n_nodes):
        m = leaf == s
        if not m.any():
            assert np.isnan(got[s])
            continue
        if exact:
            o = np.argsort(v[m], kind="stable")
            want = rf._weighted_median_sorted(v[m][o], w[m][o])
        else:
            want = wq.query(wq.build(v[m], w[m], size), [0.5])[0]
        assert got[s] == want, (s, exact, size)
    return ent


@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("size", [100_000, 40, 7])
def test_seg_median_matches_host_rules(exact, size):
    leaf, v, w = _case(1)
    _check(leaf, v, w, 10, exact, size)


def test_leaf_summaries_match_native_pruned_build():
    leaf, v, w = _case(2, ties=False)
    ent = rf.leaf_entries(torch.from_numpy(leaf), torch.from_numpy(v), torch.from_numpy(w), 10)
    summ = rf.leaf_summaries(*ent, list(range(10)), size=30)
    for s in range(10):
        m = leaf == s
        want = wq.build(v[m], w[m], 30) if m.any() else np.zeros((0, 4))
        np.testing.assert_array_equal(summ[s].numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("size", [100_000, 40])
def test_seg_median_kernel_matches_host_rules(cuda, exact, size):
    leaf, v, w = _case(3, n=50_000, leaves=33)
    _check(leaf, v, w, 40, exact, size, dev=cuda)


@pytest.mark.gpu
def test_seg_prune_kernel_matches_native(cuda):
    leaf, v, w = _case(4, n=40_000, leaves=5, ties=False)
    ent = rf.leaf_entries(torch.from_numpy(leaf).to(cuda), torch.from_numpy(v).to(cuda), torch.from_numpy(w).to(cuda), 6)
    summ = rf.leaf_summaries(*ent, list(range(6)), size=50)
    for s in range(6):
        m = leaf == s
        want = wq.build(v[m], w[m], 50) if m.any() else np.zeros((0, 4))
        np.testing.assert_array_equal(summ[s].cpu().numpy(), want)
