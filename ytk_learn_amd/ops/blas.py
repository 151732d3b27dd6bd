"""fp64-accumulated reductions of fp32 vectors (``csrc/hip/blas.hip``).

Used by the L-BFGS/OWL-QN driver for the two-loop dot products, line-search directional
derivatives and regularizer sums over the full model vector. On CPU: torch in fp64.
"""
from __future__ import annotations

import os

import torch

from ._ext import check_cuda, hip, ptr, stream

_scratch = {}


def _buffers(dev):
    key = (dev.type, dev.index)
    if key not in _scratch:
        _scratch[key] = torch.empty(1024 + 8, dtype=torch.float64, device=dev)
    return _scratch[key]


def _reduce(a: torch.Tensor, b, mode: int) -> float:
    if a.device.type != "cuda":
        a64 = a.reshape(-1).double()
        if mode == 0:
            return float(torch.dot(a64, b.reshape(-1).double()))
        if mode == 1:
            return float(torch.dot(a64, a64))
        return float(a64.abs().sum())
    a = a.reshape(-1)
    if not a.is_contiguous():
        a = a.contiguous()
    if b is not None:
        b = b.reshape(-1)
        if not b.is_contiguous():
            b = b.contiguous()
        if b.numel() != a.numel():
            raise ValueError("dot: size mismatch")
        check_cuda(a, b)
    else:
        check_cuda(a)
    if a.dtype != torch.float32 or (b is not None and b.dtype != torch.float32):
        raise TypeError("dot: float32 operands expected")
    buf = _buffers(a.device)
    hip().dot(ptr(a), ptr(b) if b is not None else 0, a.numel(), mode, ptr(buf), ptr(buf[1024:]), stream(a))
    return float(buf[1024])


def dot(a: torch.Tensor, b: torch.Tensor) -> float:
    return _reduce(a, b, 0)


def sum_sq(a: torch.Tensor) -> float:
    return _reduce(a, None, 1)


def sum_abs(a: torch.Tensor) -> float:
    return _reduce(a, None, 2)


def axpy_dot(p: torch.Tensor, x: torch.Tensor, alpha: float, scale: float, d: torch.Tensor) -> float:
    """p <- (p + alpha x) * scale in place (fp32, torch's add-then-scale order), returning
    d . p_new accumulated in fp64 -- one pass over the four vectors (the two-loop
    recursion's update + next dot product). GPU float32 contiguous operands."""
    if p.device.type != "cuda":
        p.add_(x, alpha=alpha)
        if scale != 1.0:
            p.mul_(scale)
        return float(torch.dot(p.reshape(-1).double(), d.reshape(-1).double()))
    for t in (p, x, d):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p.numel():
            raise TypeError("axpy_dot: contiguous float32 operands of one size expected")
    check_cuda(p, x, d)
    buf = _buffers(p.device)
    hip().axpy_dot(ptr(p), ptr(x), float(alpha), float(scale), ptr(d), p.numel(), ptr(buf), ptr(buf[1024:]),
                   stream(p))
    return float(buf[1024])


_ROW_LOSS = {"sigmoid": 0, "l2": 1}


def row_loss(loss, z0: torch.Tensor, y: torch.Tensor, wt: torch.Tensor, z1=None, want_grad: bool = True,
             want_loss: bool = True):
    """One fused pass over the rows of a single-output L-BFGS model (``row_loss_partial_kernel``):
    z = z0 (+ z1) in fp64 -> (sum weight * loss (fp64 float), pred fp32 [n], c = weight * l'(z)
    fp32 [n] or None). The formulas are the loss classes' fp64 ones
    (``losses/functions.py``, reference LinearHoagOptimizer.java:127-147). Returns None when the
    fused pass does not cover the case (CPU tensors, losses other than sigmoid / l2,
    YTK_ROW_LOSS=0): the caller runs the torch formulas then. ``want_loss=False``: the loss sum
    is not read back (None; no host synchronisation -- SGD batches)."""
    lid = _ROW_LOSS.get(getattr(loss, "name", None))
    if lid is None or z0.device.type != "cuda" or os.environ.get("YTK_ROW_LOSS", "1") == "0":
        return None
    n = z0.numel()
    if (z0.dim() != 1 or not z0.is_contiguous() or z0.dtype not in (torch.float32, torch.float64)
            or y.dim() != 1 or y.dtype != torch.float32 or y.numel() != n or wt.numel() != n):
        return None
    if z1 is not None and (z1.dtype != torch.float32 or not z1.is_contiguous() or z1.numel() != n):
        return None
    wt = wt.float().contiguous()
    check_cuda(z0, wt, *([z1] if z1 is not None else []))
    if not y.is_cuda or y.device != z0.device:
        raise ValueError("row_loss: labels on another device")
    pred = torch.empty(n, dtype=torch.float32, device=z0.device)
    c = torch.empty(n, dtype=torch.float32, device=z0.device) if want_grad else None
    buf = _buffers(z0.device)
    hip().row_loss(lid, ptr(z0), 1 if z0.dtype == torch.float64 else 0, ptr(z1) if z1 is not None else 0, ptr(y),
                   y.stride(0), ptr(wt), n, ptr(pred), ptr(c) if c is not None else 0, ptr(buf), ptr(buf[1024:]),
                   stream(z0))
    return (float(buf[1024]) if want_loss else None), pred, c


_MC_LOSS = {"softmax": 0, "multiclass_hinge": 1, "multiclass_l2_hinge": 2, "multiclass_smooth_hinge": 3,
            "hsoftmax": 4}
MC_MAX_BLOCKS = 4096  # grid cap of the multiclass epilogue (64-row tiles, grid-stride beyond)
_mc_scratch = {}


def multiclass_row_loss(loss, S: torch.Tensor, y: torch.Tensor, wt: torch.Tensor, want_grad: bool = True):
    """One fused pass over the rows of the multiclass linear model (``mc_row_loss_kernel``):
    scores S fp32 [n, K-1] (the K-th logit is the implicit 0), labels y [n, K], weights [n] ->
    (sum weight * loss (fp64 float), pred fp32 [n, K], D = weight * d1[:, :K-1] fp32 or None).
    The formulas are the loss classes' fp64 ones (``losses/functions.py``; reference
    MulticlassLinearHoagOptimizer.java:82-149). Returns None when the fused pass does not cover
    the case (CPU tensors, K > 64, another loss, YTK_ROW_LOSS=0): the caller runs torch then."""
    lid = _MC_LOSS.get(getattr(loss, "name", None))
    if lid is None or S.device.type != "cuda" or os.environ.get("YTK_ROW_LOSS", "1") == "0":
        return None
    n, J = S.shape
    K = J + 1
    if K < 2 or K > 64 or S.dtype != torch.float32 or tuple(y.shape) != (n, K) or wt.numel() != n:
        return None
    S = S.contiguous()
    y = y.float().contiguous()
    wt = wt.float().contiguous()
    check_cuda(S, y, wt)
    dev = S.device
    key = (dev.type, dev.index)
    if key not in _mc_scratch:
        _mc_scratch[key] = torch.empty(MC_MAX_BLOCKS + 8, dtype=torch.float64, device=dev)
    buf = _mc_scratch[key]
    pred = torch.empty((n, K), dtype=torch.float32, device=dev)
    D = torch.empty((n, J), dtype=torch.float32, device=dev) if want_grad else None
    hip().mc_row_loss(lid, ptr(S), K, ptr(y), ptr(wt), n, ptr(pred), ptr(D) if D is not None else 0, ptr(buf),
                      MC_MAX_BLOCKS, ptr(buf[MC_MAX_BLOCKS:]), stream(S))
    return float(buf[MC_MAX_BLOCKS]), pred, D
