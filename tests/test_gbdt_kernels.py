"""HIP GBDT kernels vs the CPU (PyTorch/NumPy fp32/fp64) reference of the same op."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.ops import gbdt as gops
from ytk_learn_amd.ops._ext import hist_cols

pytestmark = pytest.mark.gpu


def _rand_bins(N, F, nb, seed=0, dtype=torch.uint8):
    g = torch.Generator().manual_seed(seed)
    stride = ((F + 31) // 32) * 32
    bins = torch.zeros((N, stride), dtype=dtype)
    b = torch.randint(0, nb, (N, F), generator=g)
    bins[:, :F] = b.to(dtype)
    return bins


def _gh(N, seed=1):
    g = torch.Generator().manual_seed(seed)
    gh = torch.empty((N, 2))
    gh[:, 0] = torch.randn(N, generator=g)
    gh[:, 1] = torch.rand(N, generator=g) * 0.25
    return gh



SG, SH = gops.fixed_point_scales(3.0, 0.25, 200000)


@pytest.mark.parametrize("F,nb", [(28, 255), (7, 16), (40, 64)])
def test_hist_build_matches_cpu(cuda, F, nb):
    N = 50000
    bins = _rand_bins(N, F, nb)
    gh = _gh(N)
    B = ((nb + 3) // 4) * 4
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(3)).to(torch.int32)
    work = torch.tensor([[0, 0, 20000, 0], [0, 20000, 31000, 0], [2, 31000, 50000, 0]], dtype=torch.int32)
    hc = torch.zeros((3, B, F, 2), dtype=torch.int64)
    gops.hist_build(bins, F, gh, perm, work, hc, B, SG, SH)
    hg = torch.zeros((3, B, F, 2), dtype=torch.int64, device=cuda)
    gops.hist_build(bins.to(cuda), F, gh.to(cuda), perm.to(cuda), work.to(cuda), hg, B, SG, SH)
    assert torch.equal(hg.cpu(), hc)  # exact integer sums: bitwise identical
    # identity rows (root path)
    hc2 = torch.zeros((1, B, F, 2), dtype=torch.int64)
    w2 = torch.tensor([[0, 0, N, 0]], dtype=torch.int32)
    gops.hist_build(bins, F, gh, None, w2, hc2, B, SG, SH)
    hg2 = torch.zeros((1, B, F, 2), dtype=torch.int64, device=cuda)
    gops.hist_build(bins.to(cuda), F, gh.to(cuda), None, w2.to(cuda), hg2, B, SG, SH)
    assert torch.equal(hg2.cpu(), hc2)
    # fixed point is faithful to the fp64 sums
    ref = torch.zeros((B, F, 2), dtype=torch.float64)
    b64 = bins[:, :F].long()
    for f in range(F):
        ref[:, f, 0].index_add_(0, b64[:, f], gh[:, 0].double())
        ref[:, f, 1].index_add_(0, b64[:, f], gh[:, 1].double())
    got = hc2[0].double() * torch.tensor([1.0 / SG, 1.0 / SH], dtype=torch.float64)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-6)


def test_hist_build_uint16_global(cuda):
    N, F, nb = 20000, 5, 1000
    bins = _rand_bins(N, F, nb, dtype=torch.int16)
    gh = _gh(N)
    B = 1000
    work = torch.tensor([[0, 0, N, 0]], dtype=torch.int32)
    hc = torch.zeros((1, B, F, 2), dtype=torch.int64)
    gops.hist_build(bins, F, gh, None, work, hc, B, SG, SH)
    hg = torch.zeros((1, B, F, 2), dtype=torch.int64, device=cuda)
    gops.hist_build(bins.to(cuda), F, gh.to(cuda), None, work.to(cuda), hg, B, SG, SH)
    assert torch.equal(hg.cpu(), hc)


def _hist_from(N, F, nb, B, seed):
    bins = _rand_bins(N, F, nb, seed, dtype=torch.uint8 if nb <= 256 else torch.int16)
    gh = _gh(N, seed + 1)
    h = torch.zeros((1, B, F, 2), dtype=torch.int64)
    gops.hist_build(bins, F, gh, None, torch.tensor([[0, 0, N, 0]], dtype=torch.int32), h, B, SG, SH)
    return h[0]


@pytest.mark.parametrize("l1,l2,mal,nb", [(0.0, 0.0, -1.0, 200), (0.5, 1.0, -1.0, 200), (0.0, 1.0, 0.3, 200),
                                         (0.0, 0.0, -1.0, 600), (0.5, 1.0, -1.0, 5000), (0.0, 0.0, -1.0, 9000)])
def test_split_find_matches_cpu(cuda, l1, l2, mal, nb):
    F, B = 28, nb
    parent = _hist_from(40000, F, nb, B, 5)
    small = _hist_from(15000, F, nb, B, 6)
    # Structural invariant of real histograms, which the kernels may rely on for the node
    # totals: every row adds its (g, h) to exactly one bin of EVERY feature, so all features
    # of a node sum to the same totals, and a feature has no mass past its bin count. The
    # sparse and short features below move mass between bins instead of dropping it.
    small[49, 3] += small[50:120, 3].sum(dim=0)
    small[50:120, 3] = 0  # sparse bins (empty-bin skipping)
    parent[29, 7] += parent[30:, 7].sum(dim=0)
    parent[30:, 7] = 0
    small[29, 7] += small[30:, 7].sum(dim=0)
    small[30:, 7] = 0
    hist = torch.zeros((4, B, F, 2), dtype=torch.int64)
    hist[0] = parent + small  # parent contains the small child
    hist[1] = small
    nbins = torch.full((F,), nb, dtype=torch.int32)
    nbins[7] = 30
    fmask = torch.ones(F, dtype=torch.uint8)
    fmask[2] = 0
    items = torch.tensor([[0, 0, 0, 0], [1, 0, 0, 0], [2, 0, 1, 1]], dtype=torch.int32)
    params = {"mcw": 10.0, "l1": l1, "l2": l2, "max_abs_leaf": mal, "sg": SG, "sh": SH}
    hc = hist.clone()
    oc = gops.split_find(hc, B, F, nbins, fmask, 0, items, params).numpy().view(gops.SPLIT_DTYPE).reshape(-1)
    hg = hist.to(cuda)
    og = gops.split_find(hg, B, F, nbins.to(cuda), fmask.to(cuda), 0, items.to(cuda), params)
    og = og.cpu().numpy().view(gops.SPLIT_DTYPE).reshape(-1)
    for a, b in zip(oc, og):
        assert a["feat"] == b["feat"] and a["bin_a"] == b["bin_a"] and a["bin_b"] == b["bin_b"]
        # fp64 gain evaluation may contract to FMA on the GPU: 1 float ulp
        np.testing.assert_allclose(a["loss_chg"], b["loss_chg"], rtol=1e-6)
        np.testing.assert_allclose([a["gl"], a["hl"], a["g"], a["h"]], [b["gl"], b["hl"], b["g"], b["h"]],
                                   rtol=1e-12, atol=0)
    # derived histogram written back exactly (bins < nbins of each sampled feature)
    ref = hist[0] - hist[1]
    for f in range(F):
        if fmask[f]:
            n = int(nbins[f])
            assert torch.equal(hg[2, :n, f].cpu(), ref[:n, f])


def test_partition_matches_cpu(cuda):
    N, F = 100000, 28
    bins = _rand_bins(N, F, 255, 9)
    rows = torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(torch.int32)
    segs = [(0, 30000), (30000, 45000), (75000, 25000)]
    feat = torch.tensor([3, 17, 0], dtype=torch.int32)
    thr = torch.tensor([100, 7, 250], dtype=torch.int32)
    ch = 4096
    items, first, nblk = [], [], []
    for i, (b, c) in enumerate(segs):
        first.append(len(items))
        k = 0
        for s in range(b, b + c, ch):
            items.append((i, s, min(s + ch, b + c), k))
            k += 1
        nblk.append(k)
    args = [torch.tensor(items, dtype=torch.int32), feat, thr,
            torch.tensor([s[0] for s in segs], dtype=torch.int32),
            torch.tensor(first, dtype=torch.int32), torch.tensor(nblk, dtype=torch.int32)]
    binsT = bins[:, :F].t().contiguous()
    gh = _gh(N, 11)
    oc = torch.zeros(N, dtype=torch.int32)
    ghc = torch.zeros(N, 2)
    lc = gops.partition(binsT, rows, oc, gh, ghc, torch.zeros(N, dtype=torch.uint8), *args, 3)
    og = torch.zeros(N, dtype=torch.int32, device=cuda)
    ghg = torch.zeros(N, 2, device=cuda)
    lg = gops.partition(binsT.to(cuda), rows.to(cuda), og, gh.to(cuda), ghg,
                        torch.zeros(N, dtype=torch.uint8, device=cuda), *[a.to(cuda) for a in args], 3)
    assert lg.cpu().tolist() == lc.tolist()
    assert torch.equal(og.cpu(), oc)
    assert torch.equal(ghg.cpu(), ghc)
    # count-only variant agrees with the full partition's left counts
    cnt = gops.partition_count(binsT.to(cuda), rows.to(cuda), torch.zeros(N, dtype=torch.uint8, device=cuda),
                               args[0].to(cuda), feat.to(cuda), thr.to(cuda)).cpu()
    per = [int(cnt[first[i]:first[i] + nblk[i]].sum()) for i in range(3)]
    assert per == lc.tolist()
    cc = gops.partition_count(binsT, rows, torch.zeros(N, dtype=torch.uint8), args[0], feat, thr)
    assert torch.equal(cc, cnt)


def test_tree_add_bins_and_forest(cuda):
    from ytk_learn_amd.models.gbdt.tree import GBDTModel, Tree

    t = Tree()
    l, r = t.add_children(0)
    t.set_split(0, 2, 10, 12)
    ll, lr_ = t.add_children(l)
    t.set_split(l, 5, 3, 4)
    for n, v in [(ll, 0.5), (lr_, -0.25), (r, 1.5)]:
        t.set_leaf(n, v)
    N, F = 10000, 8
    bins = _rand_bins(N, F, 20, 4)
    binsT = bins[:, :F].t().contiguous()
    arrs = tuple(torch.from_numpy(a) for a in t.bin_arrays())
    sc = torch.zeros((N, 2))
    gops.tree_add_bins(binsT, arrs, sc, 1)
    sg = torch.zeros((N, 2), device=cuda)
    gops.tree_add_bins(binsT.to(cuda), tuple(a.to(cuda) for a in arrs), sg, 1)
    torch.testing.assert_close(sg.cpu(), sc)
    # brute-force reference of the bin walk
    ref = torch.zeros(N)
    for i in range(N):
        n = 0
        while not t.is_leaf[n]:
            n = t.left[n] if int(bins[i, t.feat[n]]) <= (t.slot_a[n] + t.slot_b[n]) // 2 else t.right[n]
        ref[i] = t.leaf[n]
    torch.testing.assert_close(sc[:, 1], ref)
    # raw forest predict with NaN defaults
    cands = [np.arange(20, dtype=np.float32) * 0.5 for _ in range(F)]
    t.convert_split_values(cands)
    t.default_left = [True, False, True, True, True]
    m = GBDTModel(0.5, 1, "sigmoid")
    m.trees = [t, t]
    fl = {k: torch.from_numpy(v) for k, v in m.flatten().items()}
    X = torch.randn(N, F) * 5
    X[::7, 2] = float("nan")
    oc = torch.zeros((N, 1))
    gops.forest_predict(X, fl, oc, 0.5)
    og = torch.zeros((N, 1), device=cuda)
    gops.forest_predict(X.to(cuda), {k: v.to(cuda) for k, v in fl.items()}, og, 0.5)
    torch.testing.assert_close(og.cpu(), oc)
    lo_c = torch.zeros((N, 2), dtype=torch.int32)
    gops.forest_predict(X, fl, None, 1.0, lo_c)
    lo_g = torch.zeros((N, 2), dtype=torch.int32, device=cuda)
    gops.forest_predict(X.to(cuda), {k: v.to(cuda) for k, v in fl.items()}, None, 1.0, lo_g)
    assert torch.equal(lo_g.cpu(), lo_c)
    # F = 8: the row-register kernel ran above; F = 6 (not a multiple of 4) takes the generic one
    X6 = X[:, :6].contiguous()
    oc6 = torch.zeros((N, 1))
    gops.forest_predict(X6, fl, oc6, 0.5)
    og6 = torch.zeros((N, 1), device=cuda)
    gops.forest_predict(X6.to(cuda), {k: v.to(cuda) for k, v in fl.items()}, og6, 0.5)
    torch.testing.assert_close(og6.cpu(), oc6)


@pytest.mark.parametrize("lds,N,F", [("1", 30000, 6), ("0", 30000, 6), ("1", 70001, 28)])
def test_bin_assign_matches_cpu(cuda, monkeypatch, lds, N, F):
    """GPU bin assignment (LDS-tiled kernel by default, the per-element kernel with
    YTK_BIN_ASSIGN_LDS=0) == the CPU rule, row-major and column-major outputs."""
    monkeypatch.setenv("YTK_BIN_ASSIGN_LDS", lds)
    X = torch.randn(N, F)
    X[:, 3] = torch.round(X[:, 3] * 2) / 2  # ties with candidates
    cands = [np.sort(np.unique(np.random.default_rng(f).normal(size=50).astype(np.float32))) for f in range(F)]
    cands[3] = np.array([-1.0, -0.5, 0.0, 0.5, 1.0], np.float32)
    cands[5] = np.array([0.0], np.float32)
    if F > 6:
        cands[7] = np.sort(np.unique(np.random.default_rng(99).normal(size=255).astype(np.float32)))
    cand = torch.from_numpy(np.concatenate(cands))
    coff = torch.from_numpy(np.concatenate([[0], np.cumsum([len(c) for c in cands])]).astype(np.int32))
    oc = torch.zeros((N, 32), dtype=torch.uint8)
    ocT = torch.zeros((F, N), dtype=torch.uint8)
    gops.bin_assign(X, cand, coff, oc, ocT)
    assert int(oc.max()) > 4
    og = torch.zeros((N, 32), dtype=torch.uint8, device=cuda)
    ogT = torch.zeros((F, N), dtype=torch.uint8, device=cuda)
    gops.bin_assign(X.to(cuda), cand.to(cuda), coff.to(cuda), og, ogT)
    assert torch.equal(og.cpu(), oc)
    assert torch.equal(ogT.cpu(), ocT)
    assert torch.equal(ocT, oc[:, :F].t())


def test_tree_grad_fused_matches_cpu(cuda):
    from ytk_learn_amd.models.gbdt.tree import Tree

    t = Tree()
    l, r = t.add_children(0)
    t.set_split(0, 1, 5, 6)
    ll, lr = t.add_children(l)
    t.set_split(l, 13, 3, 4)
    rl, rr = t.add_children(r)
    t.set_split(r, 27, 8, 9)
    for leaf, v in ((ll, 0.3), (lr, 0.1), (rl, -0.2), (rr, -0.05)):
        t.set_leaf(leaf, v)
    N, F = 40000, 28
    bins = _rand_bins(N, F, 12, 8)  # row-major, padded row stride 32 -> register walk
    arrs = tuple(torch.from_numpy(a) for a in t.bin_arrays())
    g = torch.Generator().manual_seed(2)
    score = torch.randn((N, 1), generator=g)
    init = torch.full((N, 1), 0.1)
    lab = (torch.rand((N, 1), generator=g) < 0.5).float()
    w = torch.rand(N, generator=g) + 0.5
    sc, pc, ghc = score.clone(), torch.zeros((N, 1)), torch.zeros((1, N, 2))
    mc = torch.zeros(2)
    ac = gops.tree_grad(bins, arrs, sc, init, lab, w, "sigmoid", 0.0, 1.0, pc, ghc[0], True, mc)
    # the bin-space walk equals a column walk on the same tree
    ref = score[:, 0] + gops._walk_bins(bins[:, :F].t().contiguous(), arrs)
    torch.testing.assert_close(sc[:, 0], ref)
    torch.testing.assert_close(mc, ghc[0].abs().amax(dim=0))
    sg, pg, ghg = score.to(cuda), torch.zeros((N, 1), device=cuda), torch.zeros((1, N, 2), device=cuda)
    mg = torch.zeros(2, device=cuda)
    ag = gops.tree_grad(bins.to(cuda), tuple(a.to(cuda) for a in arrs), sg, init.to(cuda), lab.to(cuda),
                        w.to(cuda), "sigmoid", 0.0, 1.0, pg, ghg[0], True, mg)
    torch.testing.assert_close(sg.cpu(), sc)
    torch.testing.assert_close(pg.cpu(), pc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ghg.cpu(), ghc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mg.cpu(), ghg[0].abs().amax(dim=0).cpu(), rtol=0, atol=0)
    np.testing.assert_allclose(ag.cpu().numpy(), ac.numpy(), rtol=1e-6)
    # pred is optional
    sg2, ghg2 = score.to(cuda), torch.zeros((N, 2), device=cuda)
    gops.tree_grad(bins.to(cuda), tuple(a.to(cuda) for a in arrs), sg2, init.to(cuda), lab.to(cuda),
                   w.to(cuda), "sigmoid", 0.0, 1.0, None, ghg2)
    torch.testing.assert_close(ghg2, ghg[0], rtol=0, atol=0)
    # generic byte-load walk (row stride 40 B) and uint16 rows (64 B register walk)
    wide = torch.zeros((N, 40), dtype=torch.uint8)
    wide[:, :32] = bins
    b16 = bins.to(torch.int16)
    for bb in (wide, b16):
        s3 = score.to(cuda)
        gops.tree_grad(bb.to(cuda), tuple(a.to(cuda) for a in arrs), s3, init.to(cuda), lab.to(cuda),
                       w.to(cuda), "sigmoid", 0.0, 1.0, None, torch.zeros((N, 2), device=cuda))
        torch.testing.assert_close(s3.cpu(), sc, rtol=0, atol=0)


@pytest.mark.parametrize("loss,K", [("sigmoid", 1), ("l2", 1), ("l1", 1), ("poisson", 1), ("huber", 1), ("softmax", 4)])
def test_grad_hess_matches_cpu(cuda, loss, K):
    N = 20000
    g = torch.Generator().manual_seed(0)
    score = torch.randn((N, K), generator=g)
    init = torch.randn((N, K), generator=g) * 0.1
    if loss == "softmax":
        lab = torch.nn.functional.one_hot(torch.randint(0, K, (N,), generator=g), K).float()
    elif loss == "sigmoid":
        lab = (torch.rand((N, K), generator=g) < 0.4).float()
    elif loss == "poisson":
        lab = torch.randint(0, 5, (N, K), generator=g).float()
    else:
        lab = torch.randn((N, K), generator=g)
    w = torch.rand(N, generator=g) + 0.5
    param = 0.5 if loss == "huber" else 0.0
    pc, ghc = torch.zeros((N, K)), torch.zeros((K, N, 2))
    ac = gops.grad_hess(score, init, lab, w, loss, param, 1.0, pc, ghc)
    pg, ghg = torch.zeros((N, K), device=cuda), torch.zeros((K, N, 2), device=cuda)
    mg = torch.zeros((K, 2), device=cuda)
    ag = gops.grad_hess(score.to(cuda), init.to(cuda), lab.to(cuda), w.to(cuda), loss, param, 1.0, pg, ghg,
                        True, mg)
    torch.testing.assert_close(pg.cpu(), pc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ghg.cpu(), ghc, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mg.cpu(), ghg.abs().amax(dim=1).cpu(), rtol=0, atol=0)
    np.testing.assert_allclose(ag.cpu().numpy(), ac.numpy(), rtol=2e-6)


@pytest.mark.parametrize("F,nb,N,items_per_slot", [(28, 255, 1_000_000, 64), (28, 255, 300_000, 7),
                                                   (40, 64, 200_000, 33)])
def test_hist_build_staged_matches_cpu(cuda, F, nb, N, items_per_slot):
    """Two-stage (staging + split-K reduce) flush, contiguous slots and scattered slot ids."""
    bins = _rand_bins(N, F, nb, seed=5)
    gh = _gh(N, seed=6)
    B = ((nb + 3) // 4) * 4
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(7)).to(torch.int32)
    nslot = 3
    edges = np.linspace(0, N, nslot * items_per_slot + 1).astype(np.int64)
    slots_scattered = [5, 1, 3]
    for slot_ids in (None, slots_scattered):
        ids = list(range(2, 2 + nslot)) if slot_ids is None else slot_ids
        work = np.zeros((nslot * items_per_slot, 4), np.int32)
        for k in range(nslot * items_per_slot):
            work[k] = (ids[k // items_per_slot], edges[k], edges[k + 1], 0)
        work_t = torch.from_numpy(work)
        hc = torch.zeros((6, B, F, 2), dtype=torch.int64)
        gops.hist_build(bins, F, gh, perm, work_t, hc, B, SG, SH)
        hg = torch.zeros((6, B, F, 2), dtype=torch.int64, device=cuda)
        staging = torch.empty(len(work) * hist_cols(F) * B * 2, dtype=torch.int64, device=cuda)
        gops.hist_build(bins.to(cuda), F, gh.to(cuda), perm.to(cuda), work_t.to(cuda), hg, B, SG, SH,
                        staging=staging, slot_base=2, nslots=nslot,
                        slot_ids=None if slot_ids is None else torch.tensor(slot_ids, dtype=torch.int32, device=cuda))
        assert torch.equal(hg.cpu(), hc), f"slot_ids={slot_ids}"


@pytest.mark.parametrize("identity", [False, True])
def test_partition_atomic_is_a_segmentwise_partition(cuda, identity):
    """Single-pass partition: same left counts as the stable CPU partition and, per segment,
    the same SET of (row, g, h) on each side (chunk order inside a side is free); rows
    outside the split segments are untouched."""
    N, F = 100000, 28
    bins = _rand_bins(N, F, 255, 9)
    rows = (torch.arange(N, dtype=torch.int32) if identity
            else torch.randperm(N, generator=torch.Generator().manual_seed(1)).to(torch.int32))
    segs = [(0, 30000), (30000, 4500), (40000, 1), (75000, 25000)]
    feat = torch.tensor([3, 17, 5, 0], dtype=torch.int32)
    thr = torch.tensor([100, 7, 30, 250], dtype=torch.int32)
    binsT = bins[:, :F].t().contiguous()
    gh = _gh(N, 11)
    # CPU reference: stable partition of every segment
    items, first, nblk = [], [], []
    for i, (b, c) in enumerate(segs):
        first.append(len(items))
        items.append((i, b, b + c, 0))
        nblk.append(1)
    args = [torch.tensor(items, dtype=torch.int32), feat, thr, torch.tensor([s[0] for s in segs], dtype=torch.int32),
            torch.tensor(first, dtype=torch.int32), torch.tensor(nblk, dtype=torch.int32)]
    oc = torch.full((N,), -1, dtype=torch.int32)
    ghc = torch.zeros(N, 2)
    lc = gops.partition(binsT, rows, oc, gh, ghc, torch.zeros(N, dtype=torch.uint8), *args, len(segs))
    # GPU single pass
    counts = np.array([c for _, c in segs], np.int64)
    nb = (counts + gops.PART_CHUNK - 1) // gops.PART_CHUNK
    first_a = np.concatenate([[0], np.cumsum(nb)[:-1]])
    hdr = torch.tensor([len(segs), int(nb.sum())], dtype=torch.int32, device=cuda)
    og = torch.full((N,), -1, dtype=torch.int32, device=cuda)
    ghg = torch.zeros(N, 2, device=cuda)
    lg = gops.partition_atomic(binsT.to(cuda), None if identity else rows.to(cuda), og,
                               gh.to(cuda), ghg, torch.from_numpy(first_a.astype(np.int32)).to(cuda), hdr,
                               int(nb.sum()), feat.to(cuda), thr.to(cuda),
                               torch.tensor([s[0] for s in segs], dtype=torch.int32, device=cuda),
                               torch.from_numpy(counts.astype(np.int32)).to(cuda))
    assert lg.cpu().tolist() == lc.tolist()
    og, ghg = og.cpu(), ghg.cpu()
    covered = torch.zeros(N, dtype=torch.bool)
    for (b, c), nl in zip(segs, lc.tolist()):
        for lo, hi in ((b, b + nl), (b + nl, b + c)):
            covered[lo:hi] = True
            kc = sorted(zip(oc[lo:hi].tolist(), ghc[lo:hi, 0].tolist(), ghc[lo:hi, 1].tolist()))
            kg = sorted(zip(og[lo:hi].tolist(), ghg[lo:hi, 0].tolist(), ghg[lo:hi, 1].tolist()))
            assert kc == kg
    assert bool((og[~covered] == -1).all())


@pytest.mark.parametrize("F,nb,B", [(7, 300, 300), (28, 5000, 5000), (3, 9000, 9000), (40, 700, 704)])
@pytest.mark.parametrize("gathered", [False, True])
@pytest.mark.parametrize("staged", [False, True])
def test_hist_build_wide_matches_cpu(cuda, F, nb, B, gathered, staged):
    """Wide-bin (uint16, B > 256) row-major LDS kernel == the exact CPU integer histogram,
    with several work items over several slots, (optionally) a row permutation, and the
    atomic or the staged (block partials + split-K reduce) flush."""
    N = 60000
    bins = _rand_bins(N, F, nb, seed=3, dtype=torch.int16)
    binsT = bins[:, :F].t().contiguous()
    gh = _gh(N, 4)
    rows = torch.randperm(N, generator=torch.Generator().manual_seed(5)).to(torch.int32) if gathered else None
    work = torch.tensor([[0, 0, 20000, 0], [0, 20000, 31000, 0], [1, 31000, 31001, 0], [2, 31001, N, 0]],
                        dtype=torch.int32)
    hc = torch.zeros((3, B, F, 2), dtype=torch.int64)
    gops.hist_build(bins, F, gh, rows, work, hc, B, SG, SH)
    hg = torch.zeros((3, B, F, 2), dtype=torch.int64, device=cuda)
    stg = (torch.empty(len(work) * ((F + 31) // 32) * 32 * B * 2, dtype=torch.int64, device=cuda)
           if staged else None)
    gops.hist_build(bins.to(cuda), F, gh.to(cuda), rows.to(cuda) if rows is not None else None, work.to(cuda),
                    hg, B, SG, SH, binsT=binsT.to(cuda), staging=stg, slot_base=0, nslots=3 if staged else 0)
    assert torch.equal(hg.cpu(), hc)

