"""Micro-benchmark of the FFM backward kernels on the bench_sparse data shape (one GPU)."""
import os
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ytk_learn_amd.data.synthetic import criteo_like  # noqa: E402
from ytk_learn_amd.ops.ffm import ffm_backward_csc, ffm_forward  # noqa: E402
from ytk_learn_amd.ops.sparse import SparseMatrix  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    dev = torch.device("cuda")
    ip, idx, val, fld, _ = criteo_like(rows, 39, 1_000_000, seed=11, device=dev)
    F = 39 * (1_000_000 // 39)
    nf, k = 39, 4
    X = SparseMatrix(ip, idx, val, F)
    V = torch.randn(F * nf * k, device=dev) * 0.01
    c = torch.randn(rows, device=dev)
    gV = torch.zeros_like(V)
    for name, fn in [("fwd", lambda: ffm_forward(ip, idx, val, fld, V, nf, k)),
                     ("csc", lambda: ffm_backward_csc(X, fld, V, nf, k, c, gV))]:
        fn()
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"{name} dbg={os.environ.get('YTK_FFM_DBG', '0')}: {(time.time() - t) / 3 * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "sweep":
        for d in ["0", "1", "2", "3", "4", "8"]:
            env = dict(os.environ, YTK_FFM_DBG=d)
            subprocess.run([sys.executable, __file__, sys.argv[1]], env=env, check=True, timeout=300)
    else:
        main()
