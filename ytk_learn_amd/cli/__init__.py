"""Command-line entry points (``python -m ytk_learn_amd.cli.<train|predict|convert>``)."""
