"""Synthetic datasets with the shapes of the reference's benchmarks (no network).

* ``higgs_like``: Higgs-shaped dense binary classification -- 28 float features
  (21 "low level": positive heavy-tailed momenta, bounded pseudo-rapidities,
  uniform angles, 3-valued b-tags; 7 "high level": positive invariant-mass-like
  features) with a nonlinear logit, so trees have real structure to learn.
  The reference benchmark (docs/gbdt_experiments.md:9) is 10.5M train + 0.5M
  test rows x 28 features.
* ``criteo_like``: sparse CTR-shaped rows for the FM/FFM paths.

Generated directly on the target device with a seeded generator.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch


def _higgs_chunk(m: int, g: torch.Generator, dev: torch.device) -> Tuple[torch.Tensor, torch.Tensor]:
    Z = torch.randn((m, 28), generator=g, device=dev)
    U = torch.rand((m, 28), generator=g, device=dev)
    x = torch.empty((m, 28), device=dev)
    # 5 objects x (pT, eta, phi, btag)-ish + missing-energy magnitude/phi -> 21 low-level
    for j in range(21):
        k = j % 4
        if k == 0:
            x[:, j] = -torch.log(U[:, j].clamp_min(1e-7)) * 0.8 + 0.3   # pT ~ exponential
        elif k == 1:
            x[:, j] = torch.clamp(Z[:, j] * 1.0, -2.5, 2.5)             # eta
        elif k == 2:
            x[:, j] = (U[:, j] * 2.0 - 1.0) * math.pi                      # phi
        else:
            x[:, j] = torch.floor(U[:, j] * 3.0) * 1.1                    # b-tag {0,1.1,2.2}
    for j in range(21, 28):
        x[:, j] = torch.exp(0.35 * Z[:, j]) * (0.8 + 0.1 * (j - 21))     # masses ~ lognormal
    logit = (0.9 * (x[:, 25] - 1.0) - 0.7 * (x[:, 26] - 1.2) + 0.5 * torch.tanh(x[:, 0] - 1.0)
             + 0.4 * x[:, 4] * x[:, 8] / (1.0 + x[:, 4] + x[:, 8])
             + 0.3 * torch.cos(x[:, 2] - x[:, 6]) + 0.25 * (x[:, 3] > 1.0).float()
             - 0.35 * (x[:, 27] - 1.4) ** 2 + 0.2 * x[:, 1] * x[:, 5] + 0.3 * torch.sin(x[:, 22]))
    noise = torch.randn((m,), generator=g, device=dev) * 0.6
    p = torch.sigmoid(logit + noise)
    y = (torch.rand((m,), generator=g, device=dev) < p).float()
    return x, y


def higgs_like(n: int, seed: int = 0, device="cpu", chunk: int = 1 << 22) -> Tuple[torch.Tensor, torch.Tensor]:
    dev = torch.device(device)
    X = torch.empty((n, 28), dtype=torch.float32, device=dev)
    y = torch.empty((n, 1), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        x, yy = _higgs_chunk(m, g, dev)
        y[s:s + m, 0] = yy
        X[s:s + m] = x
    return X, y


def higgs_like_rows(n: int, lo: int, hi: int, seed: int = 0, device="cpu",
                    chunk: int = 1 << 20) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rows [lo, hi) of ONE global n-row Higgs-shaped dataset: chunk c (rows [c*chunk,
    (c+1)*chunk)) is drawn from its own generator seeded (seed, c), so every rank of a
    row-sharded job generates only the chunks that overlap its slice and any world size
    trains on the same global rows."""
    dev = torch.device(device)
    lo, hi = max(0, lo), min(n, hi)
    X = torch.empty((max(0, hi - lo), 28), dtype=torch.float32, device=dev)
    y = torch.empty((max(0, hi - lo), 1), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for c in range(lo // chunk, -(-hi // chunk)):
        s, e = c * chunk, min(n, (c + 1) * chunk)
        g.manual_seed(seed * 1_000_003 + c)
        x, yy = _higgs_chunk(e - s, g, dev)
        a, b = max(s, lo), min(e, hi)
        X[a - lo:b - lo] = x[a - s:b - s]
        y[a - lo:b - lo, 0] = yy[a - s:b - s]
    return X, y


def criteo_like(n: int, n_fields: int = 39, n_features: int = 1_000_000, seed: int = 0,
                device="cpu"):
    """CSR rows with one active feature per field (Criteo-shaped one-hot).

    Returns (indptr int64 [n+1], indices int32 [n*fields], values float32, fields int32, y [n,1]).
    Feature ids are drawn per field from a power-law so hot features exist.
    """
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    per_field = max(1, n_features // n_fields)
    u = torch.rand((n, n_fields), generator=g, device=dev)
    # Zipf-like: id = floor(per_field * u^3)
    loc = torch.floor(per_field * u.pow(3)).to(torch.int64).clamp_(max=per_field - 1)
    base = torch.arange(n_fields, device=dev, dtype=torch.int64) * per_field
    idx = (loc + base[None, :]).to(torch.int32)
    vals = torch.ones((n, n_fields), dtype=torch.float32, device=dev)
    fields = torch.arange(n_fields, device=dev, dtype=torch.int32).expand(n, n_fields)
    w = torch.randn((n_fields * per_field,), generator=g, device=dev) * 0.3
    logit = w[idx.long()].sum(1) - 1.0
    y = (torch.rand((n,), generator=g, device=dev) < torch.sigmoid(logit)).float()[:, None]
    indptr = torch.arange(0, n * n_fields + 1, n_fields, device=dev, dtype=torch.int64)
    return indptr, idx.reshape(-1).contiguous(), vals.reshape(-1), fields.reshape(-1).contiguous(), y
