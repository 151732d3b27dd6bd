"""Host time split of leaf-wise growth on the GPU (wall clock per phase, no syncs added):
wraps TreeBuilder methods with perf_counter accumulators. python tools/dbg_leaf_host.py"""
import runpy
import sys
import time
from functools import wraps

import torch

sys.path.insert(0, ".")
from ytk_learn_amd.models.gbdt import builder as B  # noqa: E402
from ytk_learn_amd.ops import gbdt as gops  # noqa: E402

acc = {}


def wrap(obj, name, key=None):
    f = getattr(obj, name)

    @wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[key or name] = acc.get(key or name, 0.0) + time.perf_counter() - t
    setattr(obj, name, g)


for n in ("_partition", "_build_and_find", "_count_children", "_grow_loss_guided", "build"):
    wrap(B.TreeBuilder, n)
for n in ("hist_build", "split_find", "partition_atomic", "segment_copy"):
    wrap(gops, n, "gops." + n)
_cpu = torch.Tensor.cpu


def cpu(self, *a, **k):
    t = time.perf_counter()
    r = _cpu(self, *a, **k)
    acc["tensor.cpu (sync wait)"] = acc.get("tensor.cpu (sync wait)", 0.0) + time.perf_counter() - t
    return r


torch.Tensor.cpu = cpu
sys.argv = ["bench.py", "--steps", "10", "--warmup", "2", "--policy", "loss"]
runpy.run_path("bench.py", run_name="__main__")
trees = 12
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"{v / trees * 1e3:8.3f} ms/tree  {k}")
