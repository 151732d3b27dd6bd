"""ytk-learn on MI355X (gfx950): GBDT, linear / FM / FFM and soft-tree models over HIP kernels."""
import os as _os

# Kernel arguments in device memory: the host-launched engines (leaf-wise batches: ~5 launches
# per speculative batch, ~25 batches per tree) measured 3.43 -> 3.29 ms per 255-leaf tree with
# it (profiles/r5/leafab/); graph-replayed level-wise rounds are unchanged. Read by the HIP
# runtime at its first device call, so it only applies when the package is imported before
# anything touches the GPU; an explicit user setting wins. Single-process jobs only: the
# multi-GPU path (RCCL / peer exchanges) was not measured with it, and its graph-replayed
# level-wise rounds do not gain from it.
if _os.environ.get("WORLD_SIZE", "1") == "1":
    _os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
