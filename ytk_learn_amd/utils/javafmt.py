"""Java-compatible number formatting for byte-compatible model text files.

The reference writes GBDT trees with ``Float.toString`` (J/data/gbdt/Tree.java:274,282)
and headers with ``"" + float``; linear models with ``%f``. Python's repr differs
(``1e-05`` vs ``1.0E-5``), so writers use these helpers and loaders accept both.
"""
from __future__ import annotations

import numpy as np


def _java_fmt(digits: str, exp10: int, neg: bool) -> str:
    # digits: shortest significant digits without leading zeros, value = 0.d1d2.. * 10^exp10
    # (i.e. scientific exponent e = exp10 - 1)
    e = exp10 - 1
    sign = "-" if neg else ""
    if -3 <= e < 7:
        if e >= 0:
            ip = digits[: e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e - 1) + digits
        return f"{sign}{ip}.{fp}"
    mant = digits[0] + "." + (digits[1:] or "0")
    return f"{sign}{mant}E{e}"


def _shortest(x, is_float32: bool):
    v = np.float32(x) if is_float32 else np.float64(x)
    if np.isnan(v):
        return None, "NaN"
    if np.isinf(v):
        return None, "Infinity" if v > 0 else "-Infinity"
    if v == 0:
        return None, "-0.0" if np.signbit(v) else "0.0"
    s = np.format_float_scientific(v, unique=True, trim="-")
    neg = s.startswith("-")
    s = s.lstrip("-")
    mant, exp = s.split("e")
    digits = mant.replace(".", "").rstrip("0") or "0"
    return (digits, int(exp) + 1, neg), None


def java_float_str(x) -> str:
    """``Float.toString`` of a float32 value."""
    r, special = _shortest(x, True)
    if special is not None:
        return special
    return _java_fmt(*r)


def java_double_str(x) -> str:
    """``Double.toString`` of a float64 value."""
    r, special = _shortest(x, False)
    if special is not None:
        return special
    return _java_fmt(*r)


def parse_java_float(s: str) -> float:
    s = s.strip()
    if s in ("NaN",):
        return float("nan")
    if s in ("Infinity", "+Infinity"):
        return float("inf")
    if s == "-Infinity":
        return float("-inf")
    return float(s)
