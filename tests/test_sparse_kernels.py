"""Sparse products (segmented SpMV/SpMM, CSC chunk reduce) and FFM pair kernels:
CPU torch path vs a dense fp64 reference, and the HIP kernels vs the CPU path."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.ops.ffm import ffm_backward, ffm_backward_csc, ffm_forward
from ytk_learn_amd.ops.sparse import CHUNK, SparseMatrix


def _rand_csr(n, F, avg, seed=0, bias=True):
    g = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for r in range(n):
        k = int(g.integers(1, 2 * avg))
        c = np.unique(g.integers(1 if bias else 0, F, size=k))
        rows += [r] * len(c)
        cols += c.tolist()
        vals += g.normal(size=len(c)).tolist()
        if bias:
            rows.append(r); cols.append(0); vals.append(1.0)
    rows, cols, vals = np.array(rows), np.array(cols), np.array(vals, np.float32)
    o = np.lexsort((cols, rows))
    rows, cols, vals = rows[o], cols[o], vals[o]
    indptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=indptr[1:])
    dense = np.zeros((n, F), np.float64)
    dense[rows, cols] = vals
    return torch.from_numpy(indptr), torch.from_numpy(cols.astype(np.int32)), torch.from_numpy(vals), dense


def test_spmm_cpu_matches_dense():
    n, F = 3000, 50
    ip, ix, vv, D = _rand_csr(n, F, 6)
    X = SparseMatrix(ip, ix, vv, F)
    g = torch.Generator().manual_seed(1)
    w = torch.randn(F, generator=g)
    W = torch.randn((F, 5), generator=g)
    d = torch.randn(n, generator=g)
    Dm = torch.randn((n, 5), generator=g)
    np.testing.assert_allclose(X.matmul(w).numpy(), D @ w.double().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(X.matmul(W).numpy(), D @ W.double().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(X.t_matmul(d).numpy(), D.T @ d.double().numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(X.t_matmul(Dm).numpy(), D.T @ Dm.double().numpy(), rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(X.t_matmul(d, square=True).numpy(), (D * D).T @ d.double().numpy(), rtol=1e-4,
                               atol=1e-3)
    # the bias column spans several CSC chunks
    assert n > CHUNK // 2 or X.n_chunks >= F


def test_tile_blocks_and_heavy_columns_tables():
    """Host-side tables of the tiled SpMV and the heavy-column reduce: every block holds at
    most TILE_SEGS whole segments that start inside one (TILE_CAP - 256)-entry window, the
    blocks cover the segments in order; non-contiguous segments give None; heavy columns are
    exactly those with more than REDUCE_LIGHT chunks."""
    import ytk_learn_amd.ops.sparse as sp
    g = np.random.default_rng(3)
    lens = torch.from_numpy(np.concatenate([g.integers(0, 40, 5000), [9000, 0, 3], g.integers(0, 3, 2000)]))
    beg = torch.zeros(lens.numel(), dtype=torch.int64)
    beg[1:] = torch.cumsum(lens, 0)[:-1]
    end = beg + lens
    bseg = sp.tile_blocks(beg, end)
    assert bseg is not None and int(bseg[0]) == 0 and int(bseg[-1]) == lens.numel()
    assert bool((bseg[1:] >= bseg[:-1]).all())
    win = sp.TILE_CAP - 256
    for b in range(bseg.numel() - 1):
        s0, s1 = int(bseg[b]), int(bseg[b + 1])
        if s1 == s0:
            continue
        assert s1 - s0 <= sp.TILE_SEGS
        starts = (beg[s0:s1] - beg[0]) // win
        assert int(starts.min()) == int(starts.max())  # one window
    gap = end.clone()
    gap[10] += 1  # segment 11 no longer starts where 10 ends
    assert sp.tile_blocks(beg, gap) is None
    cptr = torch.tensor([0, 1, 18, 20, 57, 57], dtype=torch.int64)  # chunks per column: 1, 17, 2, 37, 0
    assert sp.heavy_columns(cptr).tolist() == [1, 3]


def _pairs_dense(ip, ix, vv, fl, V, nf, k):
    """fp64 reference of the FFM pair sum per row."""
    V3 = V.double().view(-1, nf, k)
    out = torch.zeros(ip.shape[0] - 1, dtype=torch.float64)
    for r in range(ip.shape[0] - 1):
        a, b = int(ip[r]), int(ip[r + 1])
        for p in range(a, b):
            for q in range(p + 1, b):
                out[r] += (V3[ix[p], fl[q]] * V3[ix[q], fl[p]]).sum() * float(vv[p]) * float(vv[q])
    return out


def test_ffm_cpu_matches_loops():
    n, F, nf, k = 40, 20, 4, 4
    ip, ix, vv, _ = _rand_csr(n, F, 5, seed=3)
    g = torch.Generator().manual_seed(2)
    fl = torch.randint(0, nf, (ix.shape[0],), generator=g, dtype=torch.int32)
    V = torch.randn(F * nf * k, generator=g) * 0.3
    fx = ffm_forward(ip, ix, vv, fl, V, nf, k)
    np.testing.assert_allclose(fx.numpy(), _pairs_dense(ip, ix, vv, fl, V, nf, k).numpy(), rtol=1e-4, atol=1e-5)
    # gradient vs autograd of the dense formulation
    Vg = V.clone().double().requires_grad_(True)
    c = torch.randn(n, generator=g)
    tot = (_pairs_dense_t(ip, ix, vv, fl, Vg, nf, k) * c.double()).sum()
    tot.backward()
    gV = torch.zeros_like(V)
    ffm_backward(ip, ix, vv, fl, V, nf, k, c, gV)
    np.testing.assert_allclose(gV.numpy(), Vg.grad.numpy(), rtol=1e-4, atol=1e-5)


def _pairs_dense_t(ip, ix, vv, fl, V, nf, k):
    V3 = V.view(-1, nf, k)
    outs = []
    for r in range(ip.shape[0] - 1):
        a, b = int(ip[r]), int(ip[r + 1])
        s = torch.zeros((), dtype=V.dtype)
        for p in range(a, b):
            for q in range(p + 1, b):
                s = s + (V3[ix[p], fl[q]] * V3[ix[q], fl[p]]).sum() * float(vv[p]) * float(vv[q])
        outs.append(s)
    return torch.stack(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("J,one_hot,nnz", [(1, False, 12), (3, False, 12), (16, False, 12), (31, False, 12),
                                           (70, False, 12), (1, True, 40), (1, False, 130), (5, True, 40)])
def test_spmm_gpu_matches_cpu(cuda, J, one_hot, nnz):
    """Segmented SpMV / SpMM (CSR rows and CSC chunks) vs the CPU index-op reference,
    including one-hot matrices (value loads skipped) and long rows (4 loads per lane)."""
    n, F = 20000, 300
    ip, ix, vv, _ = _rand_csr(n, F, nnz, seed=J)
    if one_hot:
        vv = torch.ones_like(vv)
    Xc = SparseMatrix(ip, ix, vv, F)
    Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
    assert Xg.one_hot == one_hot
    g = torch.Generator().manual_seed(5)
    W = torch.randn((F, J), generator=g) if J > 1 else torch.randn(F, generator=g)
    Dm = torch.randn((n, J), generator=g) if J > 1 else torch.randn(n, generator=g)
    torch.testing.assert_close(Xg.matmul(W.to(cuda)).cpu(), Xc.matmul(W), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(Xg.matmul(W.to(cuda), square=True).cpu(), Xc.matmul(W, square=True),
                               rtol=1e-5, atol=1e-4)
    tg = Xg.t_matmul(Dm.to(cuda))
    torch.testing.assert_close(tg.cpu(), Xc.t_matmul(Dm), rtol=1e-4, atol=2e-3)
    # deterministic: identical bits on a second run
    assert torch.equal(Xg.t_matmul(Dm.to(cuda)), tg)
    # accumulate / alpha
    out = torch.ones_like(tg)
    Xg.t_matmul(Dm.to(cuda), out=out, alpha=2.0, accumulate=True)
    torch.testing.assert_close(out, 1.0 + 2.0 * tg, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,J", [(64, 1), (4096, 1), (64, 18), (4096, 3)])
def test_tiled_spmv_and_heavy_chunk_reduce(cuda, monkeypatch, chunk, J):
    """Entry-tiled SpMV (seg_tile_spmv_kernel: blocks of whole rows / CSC chunks, LDS
    products, G threads per segment incl. the LDS tree for G > 64, multi-pass rows longer
    than TILE_CAP) and the heavy-column chunk reduce (one block per column with more than
    REDUCE_LIGHT chunks) vs the CPU reference and the per-segment kernels; bitwise
    deterministic."""
    import ytk_learn_amd.ops.sparse as sparse_mod
    monkeypatch.setattr(sparse_mod, "CHUNK", chunk)
    monkeypatch.setattr(sparse_mod, "TILE_ROWS", True)  # rows through the tiled kernel too
    n, F = 30000, 200
    ip, ix, vv, _ = _rand_csr(n, F, 8, seed=11)
    # + rows longer than one tile pass (TILE_CAP entries) and an empty row
    g = np.random.default_rng(4)
    extra = [np.sort(g.choice(np.arange(1, 12000), size=9000, replace=False)), np.array([], np.int64),
             np.sort(g.choice(np.arange(1, 12000), size=5000, replace=False))]
    F2 = 12000
    ix2 = torch.cat([ix] + [torch.from_numpy(e.astype(np.int32)) for e in extra])
    vv2 = torch.cat([vv] + [torch.from_numpy(g.normal(size=e.size).astype(np.float32)) for e in extra])
    lens = torch.tensor([e.size for e in extra], dtype=torch.int64)
    ip2 = torch.cat([ip, ip[-1] + torch.cumsum(lens, 0)])
    n2 = n + len(extra)
    Xc = SparseMatrix(ip2, ix2, vv2, F2)
    Xg = SparseMatrix(ip2.to(cuda), ix2.to(cuda), vv2.to(cuda), F2)
    assert Xg.row_tiles is not None and Xg.chunk_tiles is not None
    assert (Xg.heavy_cols.numel() > 0) == (chunk == 64)
    gen = torch.Generator().manual_seed(6)
    w = torch.randn(F2, generator=gen)
    D = torch.randn((n2, J), generator=gen) if J > 1 else torch.randn(n2, generator=gen)
    z = Xg.matmul(w.to(cuda))
    torch.testing.assert_close(z.cpu(), Xc.matmul(w), rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(Xg.matmul(w.to(cuda), square=True).cpu(), Xc.matmul(w, square=True),
                               rtol=1e-4, atol=2e-3)
    tg = Xg.t_matmul(D.to(cuda))
    torch.testing.assert_close(tg.cpu(), Xc.t_matmul(D), rtol=1e-4, atol=2e-3)
    assert torch.equal(Xg.matmul(w.to(cuda)), z) and torch.equal(Xg.t_matmul(D.to(cuda)), tg)
    out = torch.ones_like(z)
    Xg.matmul(w.to(cuda), out=out, alpha=0.5, accumulate=True)
    torch.testing.assert_close(out, 1.0 + 0.5 * z, rtol=1e-5, atol=1e-4)
    # the per-segment kernels (tiling off) agree
    monkeypatch.setattr(sparse_mod, "TILE_ON", False)
    Xo = SparseMatrix(ip2.to(cuda), ix2.to(cuda), vv2.to(cuda), F2)
    assert Xo.row_tiles is None and Xo.chunk_tiles is None
    torch.testing.assert_close(Xo.matmul(w.to(cuda)), z, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(Xo.t_matmul(D.to(cuda)), tg, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("one_hot", [True, False])
def test_fixed_layout_spmv(cuda, monkeypatch, one_hot):
    """Fixed-layout rows (m entries per row, each position's columns in its own range: the
    Criteo shape) take fixed_spmv_kernel (position slices of w staged in LDS, uint16
    position-major offsets): X w, X∘X w and accumulate/alpha vs the CPU reference; a layout
    that does not qualify (ragged rows) keeps the per-row kernel."""
    import ytk_learn_amd.ops.sparse as sparse_mod
    monkeypatch.setattr(sparse_mod, "FIX_MIN_ROWS", 1000)
    n, m, width = 40000, 12, 3000
    g = np.random.default_rng(8)
    base = np.concatenate([[0], 1 + width * np.arange(m - 1)])  # bias column + (m - 1) fields
    cols = np.zeros((n, m), np.int64)
    cols[:, 1:] = base[None, 1:] + g.integers(0, width, size=(n, m - 1))
    F = int(base[-1] + width)
    ip = torch.arange(n + 1, dtype=torch.int64) * m
    ix = torch.from_numpy(cols.reshape(-1).astype(np.int32))
    vv = torch.ones(n * m) if one_hot else torch.from_numpy(g.normal(size=n * m).astype(np.float32))
    Xc = SparseMatrix(ip, ix, vv, F, build_csc=False)
    Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F, build_csc=False)
    w = torch.from_numpy(g.normal(size=F).astype(np.float32))
    z = Xg.matmul(w.to(cuda))
    fx = Xg._fixed_layout()
    assert fx and fx["m"] == m and (fx["valT"] is None) == one_hot and fx["max_span"] <= width
    torch.testing.assert_close(z.cpu(), Xc.matmul(w), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(Xg.matmul(w.to(cuda), square=True).cpu(), Xc.matmul(w, square=True), rtol=1e-5,
                               atol=1e-4)
    out = torch.full_like(z, 2.0)
    Xg.matmul(w.to(cuda), out=out, alpha=-1.5, accumulate=True)
    torch.testing.assert_close(out, 2.0 - 1.5 * z, rtol=1e-5, atol=1e-4)
    assert torch.equal(Xg.matmul(w.to(cuda)), z)  # deterministic
    # ragged rows: no fixed layout
    ip2 = ip.clone()
    ip2[1:n] += 1
    ip2[n] = ip[n]
    Xr = SparseMatrix(ip2.to(cuda), ix.to(cuda), vv.to(cuda), F, build_csc=False)
    assert Xr._fixed_layout() is False


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(4, 12), (3, 8), (8, 70)])
def test_ffm_gpu_matches_cpu(cuda, k, m, monkeypatch):
    n, F, nf = 3000, 400, 7
    ip, ix, vv, _ = _rand_csr(n, F, m, seed=k)
    g = torch.Generator().manual_seed(9)
    fl = torch.randint(0, nf, (ix.shape[0],), generator=g, dtype=torch.int32)
    V = torch.randn(F * nf * k, generator=g) * 0.2
    c = torch.randn(n, generator=g)
    fx_c = ffm_forward(ip, ix, vv, fl, V, nf, k)
    fx_g = ffm_forward(ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), V.to(cuda), nf, k)
    torch.testing.assert_close(fx_g.cpu(), fx_c, rtol=1e-4, atol=1e-4)
    gc = torch.zeros_like(V)
    ffm_backward(ip, ix, vv, fl, V, nf, k, c, gc)
    gg = torch.zeros_like(V).to(cuda)
    ffm_backward(ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), gg)
    torch.testing.assert_close(gg.cpu(), gc, rtol=1e-3, atol=1e-3)
    # SGD batch counts (optimization.sgd.average = feature): steps into V[i] divided by cnt[i]
    cnt = torch.randint(1, 5, (F,), generator=g, dtype=torch.int32)
    gcn = torch.zeros_like(V)
    ffm_backward(ip, ix, vv, fl, V, nf, k, c, gcn, cnt=cnt)
    ggn = torch.zeros_like(V).to(cuda)
    ffm_backward(ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), ggn,
                 cnt=cnt.to(cuda))
    torch.testing.assert_close(ggn.cpu(), gcn, rtol=1e-3, atol=1e-3)
    # column-ordered backward (no atomics), with and without a skipped feature
    import ytk_learn_amd.ops.sparse as sparse_mod
    monkeypatch.setattr(sparse_mod, "CHUNK", 100)  # several chunks per column
    Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
    assert Xg.n_chunks > F
    gcsc = torch.ones_like(V).to(cuda)
    ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), gcsc)
    torch.testing.assert_close(gcsc.cpu(), gc + 1.0, rtol=1e-3, atol=1e-3)
    for skip in (0, int(ix[0])):
        gs = torch.zeros_like(V)
        ffm_backward(ip, ix, vv, fl, V, nf, k, c, gs, skip_feat=skip)
        gsg = torch.zeros_like(V).to(cuda)
        ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), gsg, skip_feat=skip)
        torch.testing.assert_close(gsg.cpu(), gs, rtol=1e-3, atol=1e-3)
        fs = ffm_forward(ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), V.to(cuda), nf, k, skip_feat=skip)
        torch.testing.assert_close(fs.cpu(), ffm_forward(ip, ix, vv, fl, V, nf, k, skip_feat=skip), rtol=1e-4,
                                   atol=1e-4)
    # misaligned V (linear weights in front, as inside the model vector)
    big = torch.zeros(V.numel() + 3).to(cuda)
    big[3:] = V.to(cuda)
    fx_m = ffm_forward(ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), big[3:], nf, k)
    torch.testing.assert_close(fx_m.cpu(), fx_c, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("avg,nf", [(12, 7), (20, 40), (31, 16)])
def test_ffm_lds_forward_matches_cpu(cuda, avg, nf):
    """LDS-staged pair forward (ffm_pairs_lds_kernel, max_m given): ragged rows of up to 64
    entries, fields repeating inside a row, with and without a skipped feature -- against the
    CPU sums and the gather kernel (fp32 sums in another order)."""
    from ytk_learn_amd.ops.ffm import lds_forward_ok
    n, F, k = 3000, 400, 4
    ip, ix, vv, _ = _rand_csr(n, F, avg, seed=avg)
    g = torch.Generator().manual_seed(avg)
    fl = torch.randint(0, nf, (ix.shape[0],), generator=g, dtype=torch.int32)
    V = torch.randn(F * nf * k, generator=g) * 0.2
    max_m = int((ip[1:] - ip[:-1]).max())
    Vg = V.to(cuda)
    assert max_m <= 64 and lds_forward_ok(max_m, nf, k, Vg)
    args = (ip.to(cuda), ix.to(cuda), vv.to(cuda), fl.to(cuda), Vg, nf, k)
    for skip in (-1, int(ix[0])):
        fx_c = ffm_forward(ip, ix, vv, fl, V, nf, k, skip_feat=skip)
        fx_l = ffm_forward(*args, skip_feat=skip, max_m=max_m)
        fx_g = ffm_forward(*args, skip_feat=skip)
        torch.testing.assert_close(fx_l.cpu(), fx_c, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(fx_l, fx_g, rtol=1e-5, atol=1e-5)
        assert torch.equal(fx_l, ffm_forward(*args, skip_feat=skip, max_m=max_m))  # deterministic


@pytest.mark.gpu
def test_ffm_csc_backward_one_hot(cuda):
    """Distinct fields per row and unit values: the atomic-free LDS path and the value-free
    codes; checked against the CPU pair scatter, and bitwise repeatable."""
    from ytk_learn_amd.data.synthetic import criteo_like
    nf, k = 9, 4
    ip, ix, vv, fl, _ = criteo_like(5000, nf, 900, seed=3)
    F = nf * (900 // nf)
    g = torch.Generator().manual_seed(2)
    V = torch.randn(F * nf * k, generator=g) * 0.2
    c = torch.randn(5000, generator=g)
    gc = torch.zeros_like(V)
    ffm_backward(ip, ix, vv, fl, V, nf, k, c, gc)
    Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
    gg = torch.zeros_like(V).to(cuda)
    ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), gg)
    assert Xg._ffm_layout[1][0] is True and Xg._ffm_layout[1][3] is None  # distinct fields, unit values
    torch.testing.assert_close(gg.cpu(), gc, rtol=1e-3, atol=1e-3)
    g2 = torch.zeros_like(V).to(cuda)
    ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), g2)
    assert torch.equal(g2, gg)
    # fixed field layout (every row: fields 0..8 in order) -> the streamed XCD-split kernel ran
    assert Xg._ffm_stream[1] is not None
    import os
    os.environ["YTK_FFM_STREAM"] = "0"
    try:
        Xo = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
        g3 = torch.zeros_like(V).to(cuda)
        ffm_backward_csc(Xo, fl.to(cuda), V.to(cuda), nf, k, c.to(cuda), g3)
    finally:
        del os.environ["YTK_FFM_STREAM"]
    assert Xo._ffm_stream[1] is None
    torch.testing.assert_close(g3, gg, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,tile", [(4, 40, 0), (8, 12, 700), (16, 9, 0)])
def test_ffm_fixed_layout_backward(cuda, monkeypatch, k, m, tile):
    """Fixed-layout rows (same permuted field order in every row, a bias column in front that
    is skipped, non-unit values): the streamed XCD-split kernel matches the CPU pair scatter, small
    per-wave entry targets (many chunks per wave) included, and is bitwise repeatable."""
    import ytk_learn_amd.ops.ffm as ffm_mod
    import ytk_learn_amd.ops.sparse as sparse_mod
    monkeypatch.setattr(sparse_mod, "CHUNK", 50)
    monkeypatch.setattr(sparse_mod, "ROW_TILE", tile)
    monkeypatch.setattr(ffm_mod, "WAVE_NNZ", 300)
    n, per = 3000, 40
    g = torch.Generator().manual_seed(k + m)
    perm = torch.randperm(m, generator=g).to(torch.int32)
    loc = (per * torch.rand((n, m), generator=g).pow(3)).long().clamp_(max=per - 1)
    ix = (1 + perm.long()[None, :] * per + loc).to(torch.int32)
    ix[:, 0] = 0  # bias feature in position 0
    F = 1 + m * per
    ip = torch.arange(n + 1, dtype=torch.int64) * m
    vv = torch.rand(n * m, generator=g) + 0.5
    fl = perm.repeat(n)
    V = torch.randn(F * m * k, generator=g) * 0.2
    V.view(F, m * k)[0] = 0.0
    c = torch.randn(n, generator=g)
    ixf = ix.reshape(-1).contiguous()
    gc = torch.zeros_like(V)
    ffm_backward(ip, ixf, vv, fl, V, m, k, c, gc, skip_feat=0)
    Xg = SparseMatrix(ip.to(cuda), ixf.to(cuda), vv.to(cuda), F)
    gg = torch.zeros_like(V).to(cuda)
    ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), m, k, c.to(cuda), gg, skip_feat=0)
    st = Xg._ffm_stream[1]
    assert st is not None and st["wc"].numel() - 1 < st["beg"].numel()  # waves walk several chunks
    assert st["beg"].numel() > F  # columns split into several chunks
    torch.testing.assert_close(gg.cpu(), gc, rtol=1e-4, atol=1e-4)
    g2 = torch.zeros_like(V).to(cuda)
    ffm_backward_csc(Xg, fl.to(cuda), V.to(cuda), m, k, c.to(cuda), g2, skip_feat=0)
    assert torch.equal(g2, gg)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(3, 10), (16, 40), (40, 70)])
def test_fm_fused_gpu_matches_cpu(cuda, k, m, monkeypatch):
    from ytk_learn_amd.ops.fm import fm_backward, fm_forward
    import ytk_learn_amd.ops.sparse as sparse_mod
    n, F = 3000, 500
    ip, ix, vv, _ = _rand_csr(n, F, m, seed=k)
    g = torch.Generator().manual_seed(k)
    w = torch.randn(F + F * k + 1, generator=g) * 0.1
    c = torch.randn(n, generator=g)
    Xc = SparseMatrix(ip, ix, vv, F)
    monkeypatch.setattr(sparse_mod, "CHUNK", 64)
    Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
    wg = w.to(cuda)
    # V deliberately misaligned (starts at float offset F + 1 inside the model vector)
    Vc, Vg = w[F + 1:].view(F, k), wg[F + 1:].view(F, k)
    fc, Sc = fm_forward(Xc, w[:F], Vc)
    fg, Sg = fm_forward(Xg, wg[:F], Vg)
    torch.testing.assert_close(fg.cpu(), fc, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(Sg.cpu(), Sc, rtol=1e-5, atol=1e-5)
    glc, gVc = torch.zeros(F), torch.zeros(F, k)
    fm_backward(Xc, c, Sc, Vc, glc, gVc)
    glg, gVg = torch.zeros(F, device=cuda), torch.zeros(F, k, device=cuda)
    fm_backward(Xg, c.to(cuda), Sg, Vg, glg, gVg)
    torch.testing.assert_close(glg.cpu(), glc, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gVg.cpu(), gVc, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_row_tiled_csc_products(cuda, monkeypatch):
    """Row-tiled CSC (chunks ordered by (row tile, column); the ordered chunk reduce walks a
    column's chunks through chunk_ids): transposed SpMV / SpMM, the FM backward and both FFM
    backward kernels match the CPU path and the untiled GPU path."""
    from ytk_learn_amd.data.synthetic import criteo_like
    from ytk_learn_amd.ops.fm import fm_backward, fm_forward
    import ytk_learn_amd.ops.sparse as sparse_mod
    monkeypatch.setattr(sparse_mod, "CHUNK", 64)
    n, F, k = 5000, 600, 4
    ip, ix, vv, _ = _rand_csr(n, F, 12, seed=5)
    g = torch.Generator().manual_seed(3)
    D = torch.randn(n, 5, generator=g)
    c = torch.randn(n, generator=g)
    Xc = SparseMatrix(ip, ix, vv, F)
    ref1 = Xc.t_matmul(c)
    ref5 = Xc.t_matmul(D, square=True)
    w = torch.randn(F + F * k, generator=g) * 0.1
    Vc = w[F:].view(F, k)
    fc, Sc = fm_forward(Xc, w[:F], Vc)
    glc, gVc = torch.zeros(F), torch.zeros(F, k)
    fm_backward(Xc, c, Sc, Vc, glc, gVc)
    for tile in (700, 0):
        monkeypatch.setattr(sparse_mod, "ROW_TILE", tile)
        Xg = SparseMatrix(ip.to(cuda), ix.to(cuda), vv.to(cuda), F)
        assert (Xg.chunk_ids is not None) == (tile > 0)
        torch.testing.assert_close(Xg.t_matmul(c.to(cuda)).cpu(), ref1, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(Xg.t_matmul(D.to(cuda), square=True).cpu(), ref5, rtol=1e-4, atol=1e-4)
        fg, Sg = fm_forward(Xg, w[:F].to(cuda), Vc.to(cuda))
        glg, gVg = torch.zeros(F, device=cuda), torch.zeros(F, k, device=cuda)
        fm_backward(Xg, c.to(cuda), Sg, Vc.to(cuda), glg, gVg)
        torch.testing.assert_close(glg.cpu(), glc, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(gVg.cpu(), gVc, rtol=1e-4, atol=1e-3)
    # FFM (criteo-like rows) through the tiled chunks
    nf = 6
    ip2, ix2, vv2, fl2, _ = criteo_like(4000, nf, 600, seed=8)
    F2 = nf * (600 // nf)
    V2 = torch.randn(F2 * nf * k, generator=g) * 0.2
    c2 = torch.randn(4000, generator=g)
    gref = torch.zeros_like(V2)
    ffm_backward(ip2, ix2, vv2, fl2, V2, nf, k, c2, gref)
    monkeypatch.setattr(sparse_mod, "ROW_TILE", 900)
    Xf = SparseMatrix(ip2.to(cuda), ix2.to(cuda), vv2.to(cuda), F2)
    gg = torch.zeros_like(V2).to(cuda)
    ffm_backward_csc(Xf, fl2.to(cuda), V2.to(cuda), nf, k, c2.to(cuda), gg)
    torch.testing.assert_close(gg.cpu(), gref, rtol=1e-3, atol=1e-3)
