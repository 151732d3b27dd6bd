"""Code-object resource guard (CPU: hipcc cross-compiles gfx950 device assembly).

Per-thread scratch in a streaming kernel multiplies its memory traffic: indexing a
kernel-argument array with a runtime value (``a.ordw[d & 1]``) copied the whole 368-byte
argument block to scratch in every thread of the exact-greedy partition (13.0 ms per level;
5.7 ms once the level parity became a template constant). Every kernel must run without
scratch except the listed ones, whose scratch is a known register-pressure spill on a
non-default or single-block path.
"""
import os
import re
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from kernel_resources import HIP_DIR, demangle, kernel_table  # noqa: E402

# (pattern on the demangled name, why scratch is tolerated there)
ALLOWED = [
    (r"lv_partition_children_kernel<true, \d+, 16, true, true", "YTK_PART_CHUNK=4096 prefetch variant (off by default)"),
    (r"tree_grad_hist_kernel<0, 2>", "sigmoid fused pass at the 128-VGPR cap of 1024-thread blocks: one dword per 2 rows"),
    (r"split_feat_kernel<\d+, 1024>", "wide-bin (> 1024 bins) split search, 1024-thread blocks"),
    (r"lw_plan_kernel<true>", "one-block leaf-wise planner, workspace mode (> 512 leaves) at 1024 threads"),
    (r"lw_subtree_kernel", "opt-in small-node subtree kernel (YTK_LW_SUB_ROWS, off by default): "
                           "split_node_block's register tiles at the 1024-thread VGPR cap"),
]

pytestmark = pytest.mark.skipif(not shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")),
                                reason="hipcc not available")


@pytest.fixture(scope="module")
def table():
    files = sorted(os.path.join(HIP_DIR, f) for f in os.listdir(HIP_DIR) if f.endswith(".hip"))
    rows = kernel_table(files, jobs=8)
    for r, n in zip(rows, demangle([r["name"] for r in rows])):
        r["demangled"] = n
    return rows


def test_every_source_has_kernels(table):
    files = {r["file"] for r in table}
    for f in os.listdir(HIP_DIR):
        if f.endswith(".hip"):
            assert f in files, f


def test_no_unexpected_scratch(table):
    bad = []
    for r in table:
        if r["private_segment_fixed_size"] == 0:
            continue
        if any(re.search(p, r["demangled"]) for p, _ in ALLOWED):
            continue
        bad.append((r["file"], r["demangled"][:120], r["private_segment_fixed_size"]))
    assert not bad, "kernels with per-thread scratch:\n" + "\n".join(map(str, bad))


@pytest.mark.parametrize("kern", ["ex_part_kernel", "ex_eval_kernel", "ex_gather_kernel",
                                  "lv_partition_children_kernel<true, 64, 8, true, true, false",
                                  "hist_fx_kernel", "hist_reduce_kernel"])
def test_hot_kernels_fit_registers(table, kern):
    rows = [r for r in table if kern in r["demangled"]]
    assert rows, kern
    for r in rows:
        assert r["private_segment_fixed_size"] == 0, r["demangled"]
        assert r["vgpr_spill_count"] == 0, r["demangled"]
