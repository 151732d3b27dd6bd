"""Weighted mergeable quantile summary (native WQSummary) vs exact weighted quantiles."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.utils import quantile as wq


def _rank_err(x, w, v, q):
    o = np.argsort(x, kind="stable")
    cw = np.cumsum(w[o]) / w.sum()
    lo = cw[np.searchsorted(x[o], v, side="left") - 1] if np.searchsorted(x[o], v, side="left") > 0 else 0.0
    hi = cw[np.searchsorted(x[o], v, side="right") - 1]
    return 0.0 if lo <= q <= hi else min(abs(lo - q), abs(hi - q))


@pytest.mark.parametrize("parts", [1, 3, 8])
def test_merged_summary_rank_error(parts):
    g = np.random.default_rng(parts)
    x = np.concatenate([g.normal(size=20000), g.exponential(size=10000) * 3])
    w = g.random(x.size) + 0.1
    size = 1000
    chunks = np.array_split(np.arange(x.size), parts)
    s = wq.merge([wq.build(x[c], w[c], size) for c in chunks], size)
    assert len(s) <= size + 2
    for q in (0.0, 0.01, 0.25, 0.5, 0.75, 0.99, 1.0):
        v = wq.query(s, [q])[0]
        assert _rank_err(x, w, v, q) <= 3.0 / size * parts + 1e-9


def test_exact_when_small():
    x = np.array([3.0, 1.0, 2.0, 2.0, 5.0])
    w = np.array([1.0, 1.0, 1.0, 1.0, 1.0])
    s = wq.build(x, w)
    np.testing.assert_array_equal(s[:, 0], [1.0, 2.0, 3.0, 5.0])   # equal values merged
    np.testing.assert_array_equal(s[:, 3], [1.0, 2.0, 1.0, 1.0])
    assert wq.query(s, [0.5])[0] == 2.0
    assert wq.total(s) == 5.0


@pytest.mark.parametrize("seed,gather_max,buckets", [(0, 8192, 1024), (1, 40, 8), (2, 5, 4)])
def test_distributed_weighted_median_matches_sort(seed, gather_max, buckets):
    """Bucketed exact median (PreciseQuantile-style rounds) == single-process sorted median,
    with ties, integer and fractional weights, degenerate and empty groups."""
    import torch

    from ytk_learn_amd.models.gbdt.refine import _weighted_median_sorted
    from ytk_learn_amd.parallel.comm import Comm
    from ytk_learn_amd.utils.quantile import distributed_weighted_median

    rng = np.random.default_rng(seed)
    n, G = 20000, 9
    g = rng.integers(0, G - 1, n)  # group G-1 stays empty
    v = np.round(rng.normal(size=n) * 3, 1)  # many ties
    v[g == 3] = 2.5  # one distinct value
    w = rng.integers(1, 4, n).astype(np.float64) if seed != 1 else rng.random(n) + 0.5
    got = distributed_weighted_median(torch.from_numpy(v), torch.from_numpy(w), torch.from_numpy(g), G,
                                      Comm.local(), buckets=buckets, gather_max=gather_max)
    for k in range(G):
        m = g == k
        if not m.any():
            assert np.isnan(got[k])
            continue
        o = np.argsort(v[m], kind="stable")
        assert got[k] == _weighted_median_sorted(v[m][o], w[m][o]), k


def test_distributed_weighted_median_heavy_ties_resolve_without_gather():
    """A leaf of 200k identical integer residuals plus a few outliers: the tied bucket is
    resolved in place (survivors' range collapses) instead of all-gathering every tied row."""
    import torch

    from ytk_learn_amd.models.gbdt.refine import _weighted_median_sorted
    from ytk_learn_amd.parallel.comm import Comm
    from ytk_learn_amd.utils import quantile as q

    rng = np.random.default_rng(3)
    n = 200_000
    v = np.full(n, 1.0)
    v[:50] = rng.normal(size=50) * 100
    v[50:90] = 7.0
    g = np.zeros(n, np.int64)
    g[n // 2:] = 1
    v[n // 2:] = rng.integers(-3, 4, n - n // 2).astype(np.float64)  # 7 heavy tie values
    w = np.ones(n)
    got = q.distributed_weighted_median(torch.from_numpy(v), torch.from_numpy(w), torch.from_numpy(g), 2,
                                        Comm.local(), buckets=64, gather_max=16)
    for k in range(2):
        m = g == k
        o = np.argsort(v[m], kind="stable")
        assert got[k] == _weighted_median_sorted(v[m][o], w[m][o])
    # the final survivor gather holds no tied bulk
    assert q.MEDIAN_STATS["gathered_local"] <= 16


@pytest.mark.gpu
def test_weighted_binning_gpu_matches_cpu():
    """Weighted sample_by_quantile candidates (segmented run sums on the GPU) and the
    quantile missing-value fill equal the CPU path, on tie-heavy columns."""
    from ytk_learn_amd.models.gbdt import binning as bn
    from ytk_learn_amd.parallel.comm import Comm
    g = np.random.default_rng(11)
    n = 300_000
    X = np.stack([g.integers(0, 3, n).astype(np.float32),  # 3 distinct values
                  np.round(g.normal(size=n), 2).astype(np.float32),
                  g.normal(size=n).astype(np.float32)], 1)
    X[g.random(n) < 0.05, 2] = np.nan
    w = g.uniform(0.5, 2.0, n).astype(np.float32)
    spec = bn.SamplerSpec(max_cnt=31, use_sample_weight=True)
    Xc, wc = torch.from_numpy(X), torch.from_numpy(w)
    for f in range(2):
        cpu = bn.feature_candidates(Xc[:, f], wc, spec, Comm.local())
        gpu = bn.feature_candidates(Xc[:, f].cuda(), wc.cuda(), spec, Comm.local())
        np.testing.assert_array_equal(gpu, cpu)
    bc = bn._quantile_candidates_batched(Xc[:, :2], wc, [spec, spec], [0, 1], Comm.local())
    bg = bn._quantile_candidates_batched(Xc[:, :2].cuda(), wc.cuda(), [spec, spec], [0, 1], Comm.local())
    for f in range(2):
        np.testing.assert_array_equal(bg[f], bc[f])
    np.testing.assert_array_equal(bn.compute_missing_fill(Xc.cuda(), wc.cuda(), "quantile@0.5", Comm.local()),
                                  bn.compute_missing_fill(Xc, wc, "quantile@0.5", Comm.local()))
