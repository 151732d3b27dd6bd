"""Fused soft-tree epilogue (csrc/hip/gbst.hip) vs the fp64 PyTorch reference of the same
op (gbst_mixture + the loss classes of losses/functions.py + the gradient algebra of
GBSTModel._forward), for every scalar loss the kernel takes by id."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.losses.functions import create_loss
from ytk_learn_amd.models.gbst.model import GBST_LOSS_IDS, gbst_mixture

pytestmark = pytest.mark.gpu


def _reference(A, z, y, w, mask, rate, leaves, K, gate, expert, loss, rf, T):
    g, H, mu, sig = gbst_mixture(A.double(), K, gate, expert, leaves)
    mix = (g * H).sum(1) if mu is None else mu[:, 1]
    zz, yy = z.double(), y.double()
    fx = mix if rf else zz + mix
    wt = w.double()
    if mask is not None:
        wt = wt * mask.double() / rate
    L = create_loss(loss)
    lv = L.loss(fx, yy)
    grad = L.grad(fx, yy)
    pr = L.predict
    avg = (zz + mix) / T
    lvr = L.loss(avg, yy)
    c = wt * grad
    purefx = fx - zz
    Km1 = K - 1
    stride = 2 * K - 1 if expert == "linear" else K - 1
    D = torch.zeros((A.shape[0], stride), dtype=torch.float64)
    if gate == "softmax":
        D[:, :Km1] = c[:, None] * g[:, :Km1] * (H[:, :Km1] - purefx[:, None])
    else:
        for p in range(1, K):
            D[:, p - 1] = c * (mu[:, 2 * p] - sig[:, p - 1] * mu[:, p])
    if expert == "linear":
        D[:, Km1:] = c[:, None] * g
    samples = (g * mask.double()[:, None]).sum(0) if mask is not None else torch.zeros(K, dtype=torch.float64)
    lgrad = (c[:, None] * g).sum(0) if expert == "scalar" else torch.zeros(K, dtype=torch.float64)
    pred = pr(avg if rf else fx)
    return float((wt * lv).sum()), float((wt * lvr).sum()) if rf else 0.0, D, pred, samples, lgrad


def _labels(loss, n, g):
    if loss in ("sigmoid", "hinge", "smooth_hinge", "l2_hinge", "exponential"):
        return (torch.rand(n, generator=g) < 0.5).float()
    if loss == "poisson":
        return torch.poisson(torch.full((n,), 2.0), generator=g)
    if loss in ("mape", "smape", "inv_mape"):
        return torch.rand(n, generator=g) + 0.5
    return torch.randn(n, generator=g)


def _run(cuda, gate, expert, K, loss, rf, train, n=5000):
    from ytk_learn_amd.ops._ext import hip, ptr, stream
    g = torch.Generator().manual_seed(K)
    stride = 2 * K - 1 if expert == "linear" else K - 1
    A = torch.randn((n, stride), generator=g)
    z = torch.randn(n, generator=g) * 0.3
    if loss in ("inv_mape",):
        z = z + 3.0  # keep the score away from 0 (the loss divides by it)
    y = _labels(loss, n, g)
    w = torch.rand(n, generator=g) + 0.5
    mask = (torch.rand(n, generator=g) < 0.7) if train else None
    leaves = torch.randn(K, generator=g)
    rate, T = 0.7, 3
    ref = _reference(A, z, y, w, mask, rate, leaves if expert == "scalar" else None, K, gate, expert, loss, rf, T)
    Ad, zd, yd, wd = A.to(cuda), z.to(cuda), y.to(cuda), w.to(cuda)
    md = mask.to(cuda).view(torch.uint8) if mask is not None else None
    ld = leaves.to(cuda)
    acc = torch.zeros(2 + 2 * K, dtype=torch.float64, device=cuda)
    D = torch.empty((n, stride), device=cuda)
    pred = torch.empty(n, device=cuda)
    lgy = torch.lgamma(yd.double() + 1.0) if loss == "poisson" else None
    hip().gbst_epilogue(ptr(Ad), stride, ptr(zd), ptr(yd), ptr(wd), ptr(md), 1.0 / rate,
                        ptr(ld) if expert == "scalar" else 0, n, K, 1 if gate == "tree" else 0,
                        1 if expert == "linear" else 0, GBST_LOSS_IDS[loss], 0.5, 1 if rf else 0, T, 1, ptr(D),
                        stride, ptr(pred), ptr(acc), ptr(lgy) if lgy is not None else 0, stream(Ad))
    return acc.cpu().numpy(), D.cpu(), pred.cpu(), ref


def _check(a, D, pred, ref, K, rtol=1e-10):
    np.testing.assert_allclose(a[0], ref[0], rtol=rtol)
    np.testing.assert_allclose(a[1], ref[1], rtol=rtol)
    torch.testing.assert_close(D.double(), ref[2].float().double(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(pred.double(), ref[3].float().double(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(a[2:2 + K], ref[4].numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(a[2 + K:2 + 2 * K], ref[5].numpy(), rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("gate,expert", [("softmax", "linear"), ("softmax", "scalar"), ("tree", "linear"),
                                         ("tree", "scalar")])
@pytest.mark.parametrize("K", [2, 4, 7, 16, 3, 45, 64])
@pytest.mark.parametrize("loss,rf,train", [("sigmoid", False, True), ("l2", False, False), ("sigmoid", True, True)])
def test_gbst_epilogue_matches_torch(cuda, gate, expert, K, loss, rf, train):
    a, D, pred, ref = _run(cuda, gate, expert, K, loss, rf, train)
    _check(a, D, pred, ref, K)


@pytest.mark.parametrize("loss", [n for n in GBST_LOSS_IDS if n not in ("sigmoid", "l2")])
@pytest.mark.parametrize("gate,expert,K", [("softmax", "linear", 16), ("tree", "scalar", 11)])
def test_gbst_epilogue_every_loss(cuda, loss, gate, expert, K):
    """Every scalar loss (poisson, huber, the hinge family, exponential, the mape family) runs
    in the fused kernel and matches the loss classes' fp64 formulas."""
    a, D, pred, ref = _run(cuda, gate, expert, K, loss, False, True)
    _check(a, D, pred, ref, K, rtol=1e-9)


@pytest.mark.parametrize("gate,expert", [("softmax", "linear"), ("softmax", "scalar"), ("tree", "linear"),
                                         ("tree", "scalar")])
@pytest.mark.parametrize("K", [65, 96, 128, 200, 512])
@pytest.mark.parametrize("loss,rf,train", [("sigmoid", False, True), ("poisson", True, False)])
def test_gbst_epilogue_wide_k_matches_torch(cuda, gate, expert, K, loss, rf, train):
    """K > 64 (gbst_epilogue_wide_kernel: one wave per row, several experts per lane, the tree
    gate's sigmas and heap sums in a per-wave LDS row) against the same fp64 reference -- the
    reference optimizers are K-generic (GBMLRHoagOptimizer.java:159-222)."""
    a, D, pred, ref = _run(cuda, gate, expert, K, loss, rf, train, n=3000)
    _check(a, D, pred, ref, K, rtol=1e-9)
