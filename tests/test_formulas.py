"""Golden-formula property tests ("golden-value unit tests of every formula ...
kernel-vs-NumPy property tests (hypothesis is available)"):

* every single-output loss: grad == d loss / dz (torch fp64 autograd) away from its kinks, and
  hess == d grad / dz where the reference's hessian is the true second derivative
  (J/loss/*Function.java); softmax: grad == autograd, hess == the reference's 2 p (1 - p);
* AUC (slot-bucketed, J/eval/AucEvaluator.java) == the brute-force weighted Mann-Whitney
  statistic with ties counted 1/2, when predictions sit on the bucket grid;
* the L-BFGS two-loop recursion (HoagOptimizer.hv, HoagOptimizer.java:904-929) == the
  explicit recursive BFGS inverse-Hessian update applied to the vector.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ytk_learn_amd.losses.functions import create_loss
from ytk_learn_amd.metrics.evaluators import AucEvaluator
from ytk_learn_amd.parallel.comm import Comm

# name -> (label sampler, score sampler, kink test: z, y -> bool, hessian is d grad / dz)
_POS = lambda g, n: g.uniform(0.5, 5.0, n)  # noqa: E731
_BIN = lambda g, n: g.integers(0, 2, n).astype(np.float64)  # noqa: E731
_SCORE = lambda g, n: g.uniform(-3.0, 3.0, n)  # noqa: E731
_LOSSES = {
    "sigmoid": (_BIN, _SCORE, lambda z, y: np.zeros_like(z, bool), True),
    "l2": (_POS, _SCORE, lambda z, y: np.zeros_like(z, bool), True),
    "l1": (_POS, _SCORE, lambda z, y: np.abs(z - y) < 1e-3, False),
    "huber": (_POS, _SCORE, lambda z, y: np.abs(np.abs(z - y) - 0.5) < 1e-3, False),
    "poisson": (lambda g, n: g.integers(0, 6, n).astype(np.float64), _SCORE, lambda z, y: np.zeros_like(z, bool),
                True),
    "hinge": (_BIN, _SCORE, lambda z, y: np.abs(np.abs(z) - 1.0) < 1e-3, False),
    "smooth_hinge": (_BIN, _SCORE, lambda z, y: (np.abs(z) < 1e-3) | (np.abs(np.abs(z) - 1.0) < 1e-3), False),
    "l2_hinge": (_BIN, _SCORE, lambda z, y: np.abs(np.abs(z) - 1.0) < 1e-3, False),
    "exponential": (_BIN, _SCORE, lambda z, y: np.zeros_like(z, bool), False),
    "mape": (_POS, _SCORE, lambda z, y: np.abs(z - y) < 1e-3, False),
    "smape": (_POS, _SCORE, lambda z, y: (np.abs(z - y) < 1e-3) | (np.abs(z) < 1e-3), False),
    "inv_mape": (_POS, lambda g, n: g.uniform(0.5, 5.0, n), lambda z, y: np.abs(z - y) < 1e-3, False),
}


@pytest.mark.parametrize("name", sorted(_LOSSES))
@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 2 ** 31 - 1))
def test_loss_derivatives_match_autograd(name, seed):
    ys, zs, kink, true_hess = _LOSSES[name]
    g = np.random.default_rng(seed)
    n = 64
    y = torch.from_numpy(ys(g, n))
    z = torch.from_numpy(zs(g, n))
    keep = torch.from_numpy(~kink(z.numpy(), y.numpy()))
    L = create_loss(name)
    zz = z.clone().requires_grad_(True)
    L.loss(zz, y).sum().backward()
    auto = zz.grad
    got = L.grad(z, y)
    torch.testing.assert_close(got[keep], auto[keep], rtol=1e-9, atol=1e-12)
    if true_hess:
        zz = z.clone().requires_grad_(True)
        L.grad(zz, y).sum().backward()
        torch.testing.assert_close(L.hess(z, y)[keep], zz.grad[keep], rtol=1e-9, atol=1e-12)


@settings(max_examples=25, deadline=None)
@given(seed=st.integers(0, 2 ** 31 - 1), K=st.integers(2, 6))
def test_softmax_derivatives(seed, K):
    g = np.random.default_rng(seed)
    n = 32
    z = torch.from_numpy(g.normal(size=(n, K)) * 2)
    y = torch.zeros((n, K), dtype=torch.float64)
    y[torch.arange(n), torch.from_numpy(g.integers(0, K, n))] = 1.0
    L = create_loss("softmax")
    zz = z.clone().requires_grad_(True)
    L.loss(zz, y).sum().backward()
    torch.testing.assert_close(L.grad(z, y), zz.grad, rtol=1e-9, atol=1e-12)
    p = torch.softmax(z, 1)
    torch.testing.assert_close(L.hess(z, y), 2 * p * (1 - p), rtol=0, atol=0)  # the reference's 2 p (1 - p)


def _auc_pairs(y, p, w):
    pos, neg = y == 1.0, y != 1.0
    wp, wn = w[pos], w[neg]
    gt = (p[pos][:, None] > p[neg][None, :]).astype(np.float64)
    eq = (p[pos][:, None] == p[neg][None, :]).astype(np.float64)
    return float(((gt + 0.5 * eq) * wp[:, None] * wn[None, :]).sum() / (wp.sum() * wn.sum()))


@settings(max_examples=40, deadline=None)
@given(seed=st.integers(0, 2 ** 31 - 1), slots=st.sampled_from([16, 100, 1000]))
def test_auc_matches_pairwise_statistic(seed, slots):
    g = np.random.default_rng(seed)
    n = 300
    y = g.integers(0, 2, n).astype(np.float32)
    if y.min() == y.max():
        y[0] = 1.0 - y[0]
    k = g.integers(0, slots, n)
    p = ((k + 0.5) / slots).astype(np.float32)  # on the bucket grid: equal bucket <=> equal score
    w = g.uniform(0.2, 3.0, n)
    ev = AucEvaluator(f"auc@{slots}")
    a_w, a_r = ev.compute(torch.from_numpy(y), torch.from_numpy(p), torch.from_numpy(w), Comm.local())
    assert a_w == pytest.approx(_auc_pairs(y, p, w), rel=1e-9, abs=1e-12)
    assert a_r == pytest.approx(_auc_pairs(y, p, np.ones(n)), rel=1e-9, abs=1e-12)


@settings(max_examples=20, deadline=None)
@given(seed=st.integers(0, 2 ** 31 - 1), m=st.integers(1, 6), extra=st.integers(0, 4))
def test_lbfgs_two_loop_matches_explicit_bfgs(seed, m, extra):
    from types import SimpleNamespace

    from ytk_learn_amd.optim.lbfgs import HoagOptimizer
    g = np.random.default_rng(seed)
    d = 7
    npairs = m + extra  # the ring buffer wraps when there are more pairs than slots
    A = g.normal(size=(d, d))
    Hs = A @ A.T + d * np.eye(d)  # SPD: curvature pairs y = Hs s with s'y > 0
    opt = HoagOptimizer.__new__(HoagOptimizer)
    opt.ls = SimpleNamespace(m=m)
    opt.S = [torch.zeros(d, dtype=torch.float64) for _ in range(m)]
    opt.Y = [torch.zeros(d, dtype=torch.float64) for _ in range(m)]
    opt.YS = [0.0] * m
    pairs = []
    for i in range(npairs):
        s = g.normal(size=d)
        yv = Hs @ s
        c = i % m
        opt.S[c] = torch.from_numpy(s.copy())
        opt.Y[c] = torch.from_numpy(yv.copy())
        opt.YS[c] = float(s @ yv)
        pairs.append((s, yv))
    cursor = npairs % m
    loops = min(m, npairs)
    s_l, y_l = pairs[-1]
    ys, yy = float(s_l @ y_l), float(y_l @ y_l)
    # explicit: H0 = (ys / yy) I, then the BFGS inverse update for the last `loops` pairs, oldest first
    H = (ys / yy) * np.eye(d)
    for s, yv in pairs[-loops:]:
        rho = 1.0 / float(s @ yv)
        V = np.eye(d) - rho * np.outer(yv, s)
        H = V.T @ H @ V + rho * np.outer(s, s)
    v = g.normal(size=d)
    p = torch.from_numpy(v.copy())
    opt.hv(p, cursor, loops, ys, yy)
    np.testing.assert_allclose(p.numpy(), H @ v, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_slot_sums_gpu_matches_bincount_and_cpu_auc():
    """The evaluators' GPU slot sums (sort + segmented sums) == torch.bincount on the CPU;
    AUC and the confusion matrix on the GPU == the CPU evaluators."""
    from ytk_learn_amd.metrics.evaluators import ConfusionMatrixEvaluator, slot_sums
    g = np.random.default_rng(5)
    n, S = 200_000, 1000
    p = 1.0 / (1.0 + np.exp(-g.normal(size=n) * 0.7))
    y = (g.random(n) < p).astype(np.float32)
    w = g.uniform(0.5, 2.0, n)
    slot = torch.from_numpy((np.minimum((p * S).astype(np.int64), S - 1) * 2 + (y != 1.0)).astype(np.int64))
    ref = torch.stack([torch.bincount(slot, weights=torch.from_numpy(w), minlength=2 * S),
                       torch.bincount(slot, minlength=2 * S).double()])
    got = slot_sums(slot.cuda(), torch.from_numpy(w).cuda(), 2 * S).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-9)
    assert slot_sums(slot[:0].cuda(), torch.from_numpy(w[:0]).cuda(), 8).abs().sum() == 0
    pt, yt, wt = torch.from_numpy(p.astype(np.float32)), torch.from_numpy(y), torch.from_numpy(w)
    ev = AucEvaluator(f"auc@{S}")
    cpu = ev.compute(yt, pt, wt, Comm.local())
    gpu = ev.compute(yt.cuda(), pt.cuda(), wt.cuda(), Comm.local())
    assert gpu == pytest.approx(cpu, rel=1e-12)
    cm = ConfusionMatrixEvaluator("confusion_matrix")
    torch.testing.assert_close(cm.matrix(yt.cuda(), pt.cuda(), wt.cuda(), Comm.local(), 2, False),
                               cm.matrix(yt, pt, wt, Comm.local(), 2, False), rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("m,loops,cursor", [(5, 5, 0), (6, 3, 2), (4, 1, 1)])
def test_fused_two_loop_matches_unfused(monkeypatch, m, loops, cursor):
    """The GPU two-loop with every update fused with the next dot (blas.axpy_dot) == the
    unfused dot / axpy sequence (fp32 vectors, fp64 dots; tails off the 16-B path)."""
    from types import SimpleNamespace

    from ytk_learn_amd.optim.lbfgs import HoagOptimizer
    g = torch.Generator(device="cuda").manual_seed(m * 10 + loops)
    d = 100_003
    opt = HoagOptimizer.__new__(HoagOptimizer)
    opt.ls = SimpleNamespace(m=m)
    opt.S = [torch.randn(d, device="cuda", generator=g) for _ in range(m)]
    opt.Y = [s + 0.3 * torch.randn(d, device="cuda", generator=g) for s in opt.S]
    opt.YS = [float(torch.dot(s.double(), y.double())) for s, y in zip(opt.S, opt.Y)]
    p0 = torch.randn(d, device="cuda", generator=g)
    monkeypatch.setenv("YTK_FUSED_TWO_LOOP", "0")
    ref = p0.clone()
    opt.hv(ref, cursor, loops, 2.0, 3.0)
    monkeypatch.setenv("YTK_FUSED_TWO_LOOP", "1")
    got = p0.clone()
    assert opt._fused_two_loop(got)
    opt.hv(got, cursor, loops, 2.0, 3.0)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sigmoid", "l2"])
@pytest.mark.parametrize("z64,with_z1", [(False, False), (True, False), (False, True)])
def test_fused_row_loss_matches_torch_formulas(name, z64, with_z1):
    """ops.blas.row_loss (one fused HIP pass: loss sum, pred, weight * l') == the loss classes'
    fp64 torch formulas that the linear / FM / FFM models run otherwise."""
    from ytk_learn_amd.ops.blas import row_loss
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(5)
    n = 100_003
    z0 = (torch.randn(n, generator=g) * 6).to(torch.float64 if z64 else torch.float32)
    z1 = torch.randn(n, generator=g).float() if with_z1 else None
    yy = torch.stack([(torch.rand(n, generator=g) < 0.4).float(), torch.rand(n, generator=g)], 1)
    wt = torch.rand(n, generator=g) + 0.5
    loss = create_loss(name)
    out = row_loss(loss, z0.to(dev), yy.to(dev)[:, 0], wt.to(dev), z1=z1.to(dev) if z1 is not None else None)
    assert out is not None
    lsum, pred, c = out
    z = z0.double() + (z1.double() if z1 is not None else 0.0)
    y, w = yy[:, 0].double(), wt.double()
    ref_sum = float((w * loss.loss(z, y)).sum())
    assert abs(lsum - ref_sum) <= 1e-12 * abs(ref_sum) + 1e-9
    torch.testing.assert_close(pred.cpu(), loss.predict(z).float(), rtol=1e-6, atol=0)
    torch.testing.assert_close(c.cpu(), (w * loss.grad(z, y)).float(), rtol=1e-6, atol=1e-7)
    assert row_loss(loss, z0.to(dev), yy.to(dev)[:, 0], wt.to(dev), want_grad=False)[2] is None
    assert row_loss(create_loss("hinge"), z0.to(dev), yy.to(dev)[:, 0], wt.to(dev)) is None


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["softmax", "multiclass_hinge", "multiclass_l2_hinge", "multiclass_smooth_hinge",
                                  "hsoftmax"])
@pytest.mark.parametrize("K", [2, 3, 10, 33, 64])
def test_fused_multiclass_row_loss_matches_torch(name, K):
    """ops.blas.multiclass_row_loss (one fused HIP pass over the n x (K-1) scores with the
    implicit zero K-th logit: loss sum, pred [n, K], D = weight * d1[:, :K-1]) == the loss
    classes' fp64 torch formulas that MulticlassLinearModel runs otherwise (reference
    MulticlassLinearHoagOptimizer.java:82-149). n is not a multiple of the 64-row tile."""
    from ytk_learn_amd.ops.blas import multiclass_row_loss
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(K)
    n = 20_011
    S = (torch.randn(n, K - 1, generator=g) * 3).float()
    cls = torch.randint(0, K, (n,), generator=g)
    if name in ("softmax", "hsoftmax"):  # soft labels summing to 1 on half the rows, one-hot on the rest
        soft = torch.softmax(torch.randn(n, K, generator=g), 1)
        y = torch.where((torch.arange(n) % 2 == 0)[:, None], soft, torch.nn.functional.one_hot(cls, K).double())
    else:
        y = torch.nn.functional.one_hot(cls, K).double()
    y = y.float()
    wt = torch.rand(n, generator=g) + 0.5
    loss = create_loss(name)
    out = multiclass_row_loss(loss, S.to(dev), y.to(dev), wt.to(dev))
    assert out is not None
    lsum, pred, D = out
    z = torch.zeros((n, K), dtype=torch.float64)
    z[:, :K - 1] = S.double()
    lv, p_ref, d1 = loss.all(z, y.double())
    w = wt.double()
    ref_sum = float((w * lv).sum())
    assert abs(lsum - ref_sum) <= 1e-11 * abs(ref_sum) + 1e-9, (lsum, ref_sum)
    torch.testing.assert_close(pred.cpu(), p_ref.float(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(D.cpu(), (d1[:, :K - 1] * w[:, None]).float(), rtol=2e-6, atol=1e-6)
    assert multiclass_row_loss(loss, S.to(dev), y.to(dev), wt.to(dev), want_grad=False)[2] is None
