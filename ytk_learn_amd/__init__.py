"""ytk-learn on MI355X (gfx950): GBDT, linear / FM / FFM and soft-tree models over HIP kernels.

Runtime note: single-process jobs that grow leaf-wise trees gain ~4 % with kernel arguments in
device memory (``HIP_FORCE_DEV_KERNARG=1`` in the environment before the first GPU call:
3.43 -> 3.29 ms per 255-leaf tree, profiles/r5/leafab/); ``bench.py`` sets it for its
one-GPU runs. The package does not set it: child processes inherit the environment, and the
multi-GPU RCCL paths were not measured with it.
"""
