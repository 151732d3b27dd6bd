"""Loader for the in-tree native extensions.

``torch`` is imported first on purpose: torch ships ``libamdhip64.so.7`` and our
HIP module links the same SONAME, so importing torch first makes both share one
HIP runtime instance (two runtimes in a process would not share streams).

GPU ops call :func:`hip` which raises loudly when the extension is missing --
there is no silent eager fallback for tensors that live on the GPU.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension import)

_HIP = None
_NATIVE = None
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class ExtensionMissing(RuntimeError):
    pass


def _try_build():
    if os.environ.get("YTK_NO_AUTOBUILD"):
        return
    import sys

    sys.path.insert(0, os.path.join(_ROOT, "csrc"))
    try:
        import build as _b  # type: ignore

        _b.build_all()
    finally:
        sys.path.pop(0)


HIST_FW = int(os.environ.get("YTK_HIST_FW", "32"))


# == kCurStride / kDoneWords (csrc/hip/gbdt_partition_atomic.h): split cursors of the
# GPU tree engines sit one 128-B line apart, followed by the fused partition kernels'
# done counters
CUR_STRIDE = 16
DONE_WORDS = 17 * CUR_STRIDE


def hist_cols(F: int) -> int:
    """Histogram staging columns per bin: F rounded up to the per-block feature group."""
    return -(-F // HIST_FW) * HIST_FW


def hip():
    """The HIP kernel module (gfx950). Raises if not built/loadable."""
    global _HIP
    if _HIP is None:
        try:
            _HIP = importlib.import_module("ytk_learn_amd.ops._ytk_hip")
        except ImportError:
            try:
                _try_build()
                _HIP = importlib.import_module("ytk_learn_amd.ops._ytk_hip")
            except Exception as e:  # pragma: no cover - depends on toolchain
                raise ExtensionMissing(
                    "HIP extension ytk_learn_amd.ops._ytk_hip is not built; run `python csrc/build.py`"
                ) from e
        # features per histogram block (YTK_HIST_FW = 32 | 16): see hist_fx_kernel
        _HIP.hist_set_fw(HIST_FW)
    return _HIP


def native():
    """The host C++ runtime module (parser, hashing, sketches)."""
    global _NATIVE
    if _NATIVE is None:
        try:
            _NATIVE = importlib.import_module("ytk_learn_amd._native._ytk_native")
        except ImportError:
            try:
                _try_build()
                _NATIVE = importlib.import_module("ytk_learn_amd._native._ytk_native")
            except Exception as e:  # pragma: no cover
                raise ExtensionMissing(
                    "native extension ytk_learn_amd._native._ytk_native is not built; run `python csrc/build.py`"
                ) from e
    return _NATIVE


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream(t: torch.Tensor) -> int:
    """Raw hipStream_t of the current torch stream for ``t``'s device (the raw query
    skips building a Stream object: ~1 us instead of ~7 us per launch from Python)."""
    if _raw_stream is not None:
        idx = t.device.index
        return _raw_stream(torch.cuda.current_device() if idx is None else idx)
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int:
    if t is None:
        return 0
    return t.data_ptr()


def check_cuda(*ts, rows_ok=()):
    """Every tensor on the same GPU and contiguous; those in ``rows_ok`` may be row-pitched
    2-D views (contiguous rows, any row stride >= the row length: padded row layouts)."""
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("expected a GPU tensor")
        pitched = any(t is r for r in rows_ok) and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]
        if not (t.is_contiguous() or pitched):
            raise ValueError("expected a contiguous tensor")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError("tensors on different devices")
    return dev
