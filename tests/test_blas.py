"""fp64-accumulated reductions (csrc/hip/blas.hip) against torch fp64."""
import pytest
import torch

from ytk_learn_amd.ops import blas


def test_blas_cpu():
    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(1001, generator=g), torch.randn(1001, generator=g)
    assert abs(blas.dot(a, b) - float(torch.dot(a.double(), b.double()))) < 1e-12
    assert abs(blas.sum_sq(a) - float((a.double() ** 2).sum())) < 1e-10
    assert abs(blas.sum_abs(a) - float(a.double().abs().sum())) < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_blas_gpu(cuda, n):
    g = torch.Generator().manual_seed(n)
    a, b = torch.randn(n + 1, generator=g), torch.randn(n + 1, generator=g)
    for off in (0, 1):  # aligned and misaligned (scalar path)
        x, y = a[off:off + n], b[off:off + n]
        xg, yg = a.to(cuda)[off:off + n], b.to(cuda)[off:off + n]
        ref = float(torch.dot(x.double(), y.double()))
        assert abs(blas.dot(xg, yg) - ref) <= 1e-12 * max(1.0, abs(ref)) + 1e-9
        assert abs(blas.sum_sq(xg) - float((x.double() ** 2).sum())) <= 1e-9 * n
        assert abs(blas.sum_abs(xg) - float(x.double().abs().sum())) <= 1e-9 * n
        assert blas.dot(xg, yg) == blas.dot(xg, yg)  # reproducible
