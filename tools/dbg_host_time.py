"""Where does the host time of gops.partition_atomic go? (wall-clock per statement,
no device syncs added). Usage: python tools/dbg_host_time.py"""
import sys
import time

import torch

sys.path.insert(0, ".")
from ytk_learn_amd.ops import gbdt as gops  # noqa: E402
from ytk_learn_amd.ops._ext import hip, ptr, stream  # noqa: E402

acc = {}


def tick(k, t0):
    t1 = time.perf_counter()
    acc[k] = acc.get(k, 0.0) + (t1 - t0)
    return t1


def timed_partition_atomic(binsT, rows, rows_out, ghp, gh_out, first_blk, hdr, nblocks, feat, thr,
                           node_begin, node_count):
    t = time.perf_counter()
    n = feat.shape[0]
    cursor = torch.zeros(max(n, 1), dtype=torch.int64, device=binsT.device)[:n]
    t = tick("zeros", t)
    hip().partition_atomic(ptr(binsT), 1, binsT.shape[1], ptr(rows), ptr(rows_out),
                           ptr(ghp), ptr(gh_out), ptr(first_blk), ptr(hdr), ptr(hdr) + 4, nblocks,
                           ptr(feat), ptr(thr), ptr(node_begin), ptr(node_count), ptr(cursor), 0,
                           stream(binsT))
    t = tick("launch", t)
    out = cursor & 0xFFFFFFFF
    tick("and", t)
    acc["calls"] = acc.get("calls", 0) + 1
    return out


gops.partition_atomic = timed_partition_atomic
sys.argv = ["bench.py", "--steps", "6", "--warmup", "1", "--policy", "loss"]
import runpy  # noqa: E402

runpy.run_path("bench.py", run_name="__main__")
n = acc.pop("calls")
print({k: round(v / n * 1e6, 1) for k, v in acc.items()}, "us per call over", n, "calls")
