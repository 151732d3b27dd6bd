"""Weighted mergeable quantile summary (native WQSummary) vs exact weighted quantiles."""
import numpy as np
import pytest

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
