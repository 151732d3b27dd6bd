"""Fused soft-tree epilogue (csrc/hip/gbst.hip) vs the fp64 PyTorch reference of the same
op (gbst_mixture + loss / gradient algebra of GBSTModel._forward)."""
import numpy as np
import pytest
import torch

from ytk_learn_amd.models.gbst.model import gbst_mixture

pytestmark = pytest.mark.gpu


def _reference(A, z, y, w, mask, rate, leaves, K, gate, expert, loss, rf, T):
    g, H, mu, sig = gbst_mixture(A.double(), K, gate, expert, leaves)
    mix = (g * H).sum(1) if mu is None else mu[:, 1]
    zz, yy = z.double(), y.double()
    fx = mix if rf else zz + mix
    wt = w.double()
    if mask is not None:
        wt = wt * mask.double() / rate
    if loss == "sigmoid":
        lv = torch.where(fx >= 0, torch.log1p(torch.exp(-fx)) + fx * (1 - yy), torch.log1p(torch.exp(fx)) - fx * yy)
        grad = torch.sigmoid(fx) - yy
        pr = torch.sigmoid
    else:
        lv = 0.5 * (yy - fx) ** 2
        grad = fx - yy
        pr = (lambda t: t)
    avg = (zz + mix) / T
    lvr = (torch.where(avg >= 0, torch.log1p(torch.exp(-avg)) + avg * (1 - yy), torch.log1p(torch.exp(avg)) - avg * yy)
           if loss == "sigmoid" else 0.5 * (yy - avg) ** 2)
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


@pytest.mark.parametrize("gate,expert", [("softmax", "linear"), ("softmax", "scalar"), ("tree", "linear"),
                                         ("tree", "scalar")])
@pytest.mark.parametrize("K", [4, 7, 16, 3, 45])
@pytest.mark.parametrize("loss,rf,train", [("sigmoid", False, True), ("l2", False, False), ("sigmoid", True, True)])
def test_gbst_epilogue_matches_torch(cuda, gate, expert, K, loss, rf, train):
    from ytk_learn_amd.ops._ext import hip, ptr, stream
    g = torch.Generator().manual_seed(K)
    n = 5000
    stride = 2 * K - 1 if expert == "linear" else K - 1
    A = torch.randn((n, stride), generator=g)
    z = torch.randn(n, generator=g) * 0.3
    y = (torch.rand(n, generator=g) < 0.5).float() if loss == "sigmoid" else torch.randn(n, generator=g)
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
    hip().gbst_epilogue(ptr(Ad), stride, ptr(zd), ptr(yd), ptr(wd), ptr(md), 1.0 / rate,
                        ptr(ld) if expert == "scalar" else 0, n, K, 1 if gate == "tree" else 0,
                        1 if expert == "linear" else 0, 0 if loss == "sigmoid" else 1, 1 if rf else 0, T, 1, ptr(D),
                        stride, ptr(pred), ptr(acc), stream(Ad))
    a = acc.cpu().numpy()
    np.testing.assert_allclose(a[0], ref[0], rtol=1e-10)
    np.testing.assert_allclose(a[1], ref[1], rtol=1e-10)
    torch.testing.assert_close(D.cpu().double(), ref[2].float().double(), rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(pred.cpu().double(), ref[3].float().double(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(a[2:2 + K], ref[4].numpy(), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(a[2 + K:2 + 2 * K], ref[5].numpy(), rtol=1e-9, atol=1e-12)
