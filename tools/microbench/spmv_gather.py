"""Where does the J == 1 sparse product spend its time? Criteo-shape CSR (4M rows x 40 nnz,
1M columns): the tiled and the per-segment kernels with the real column indices, with every
index 0 (one cache line), and with sequential indices (i % ncols): isolates the x gathers
from the index stream."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import ytk_learn_amd.ops.sparse as sp  # noqa: E402
from ytk_learn_amd.data.synthetic import criteo_like  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0


dev = torch.device("cuda")
n, F = 4_000_000, 1_000_000
indptr, idx, vals, fields, y = criteo_like(n, 39, F, seed=11, device=dev)
out = {}
ref = None
for name, ix in (("real", idx), ("zero", torch.zeros_like(idx)),
                 ("seq", (torch.arange(idx.numel(), device=dev) % F).to(idx.dtype)),
                 ("sorted_rows", torch.sort(idx.view(n, -1) if idx.numel() % n == 0 else idx)[0].reshape(-1))):
    for tile in (True, False):
        sp.TILE_ON = sp.TILE_ROWS = tile
        X = sp.SparseMatrix(indptr, ix.to(torch.int32), torch.ones_like(vals), F, build_csc=False)
        w = torch.randn(F, device=dev)
        o = torch.empty(n, device=dev)
        tag = "tile" if tile else ("persist" if os.environ.get("YTK_SPMV_PERSIST", "1") != "0" else "seg")
        out[f"{name}_{tag}_us"] = round(timeit(lambda: X.matmul(w, out=o)), 1)
        del X
print(json.dumps(out))
