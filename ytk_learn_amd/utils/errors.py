"""Framework exception (reference: J/exception/YtkLearnException.java)."""


class YtkLearnError(RuntimeError):
    """Raised for invalid configuration, malformed input beyond max_error_tol, or
    inconsistent model files (the reference's ``YtkLearnException``)."""
