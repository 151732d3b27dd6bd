#!/usr/bin/env python3
"""Secondary benchmark: L-BFGS loss+gradient evaluations of the sparse models on a
synthetic Criteo-shaped dataset (BASELINE.json configs 4/5: FM k=16, FFM 39 fields k=4,
45M rows x 1M features at 8 GPUs).

A "step" is one full loss + gradient evaluation over the local rows (the unit of work of
every L-BFGS line-search step, HoagOptimizer.calcLossAndGrad) INCLUDING the gradient
all-reduce over RCCL; the L-BFGS/OWL-QN vector algebra of one iteration is timed
separately (``lbfgs_iter_ms``). Data-parallel weak scaling: --rows is per GPU.

  python bench_sparse.py --model fm --rows 4000000 --steps 10
  python -m torch.distributed.run --nproc-per-node 8 ... bench_sparse.py --model ffm
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from ytk_learn_amd.config.params import CommonParams, LineSearchParams  # noqa: E402
from ytk_learn_amd.data.dataflow import SparseData  # noqa: E402
from ytk_learn_amd.data.synthetic import criteo_like  # noqa: E402
from ytk_learn_amd.models.continuous.base import LoadedData  # noqa: E402
from ytk_learn_amd.optim.lbfgs import HoagOptimizer  # noqa: E402
from ytk_learn_amd.parallel.comm import Comm  # noqa: E402
from ytk_learn_amd.utils.logging import YtkLogger  # noqa: E402


class _Names(list):
    """Lazy 'f<i>' feature names (the model only indexes them at dump time)."""

    def __init__(self, n):
        super().__init__()
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return f"f{i}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="fm", choices=["linear", "fm", "ffm", "gbmlr", "gbsdt", "gbhmlr", "gbhsdt", "multiclass"])
    ap.add_argument("--classes", type=int, default=10, help="multiclass: K classes (K-1 weight columns)")
    ap.add_argument("--loss", default=None, help="multiclass: softmax (default) | multiclass_hinge | ... | hsoftmax")
    ap.add_argument("--experts", type=int, default=16, help="soft-tree experts K (gbmlr/gbsdt/gbhmlr/gbhsdt)")
    ap.add_argument("--rows", type=int, default=4_000_000, help="rows per GPU")
    ap.add_argument("--features", type=int, default=1_000_000)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--k", type=int, default=0, help="latent dim (default fm 16, ffm 4)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--optimizer", default="lbfgs", choices=["lbfgs", "sgd"],
                    help="sgd: a step is one epoch of mini-batch Hogwild!-style SGD over the local rows")
    ap.add_argument("--batch", type=int, default=65536, help="sgd mini-batch rows")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="sgd: storage of the FM latent factors read by the row passes (fp32 master kept)")
    a = ap.parse_args()
    comm = Comm.from_env()
    dev = comm.device
    k = a.k or (16 if a.model == "fm" else 4)
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    indptr, idx, vals, fields, y = criteo_like(a.rows, a.fields, a.features, seed=11 + comm.rank, device=dev)
    F = a.fields * max(1, a.features // a.fields) + 1  # + bias column 0
    idx = idx + 1
    n = a.rows
    # append the bias (index 0) to every row
    ip2 = indptr + torch.arange(n + 1, device=dev, dtype=torch.int64)
    nnz = idx.numel() + n
    rows = torch.repeat_interleave(torch.arange(n, device=dev), indptr[1:] - indptr[:-1])
    pos = torch.arange(idx.numel(), device=dev, dtype=torch.int64) + rows  # shift by row index
    idx2 = torch.zeros(nnz, dtype=torch.int32, device=dev)
    val2 = torch.ones(nnz, dtype=torch.float32, device=dev)
    fld2 = torch.zeros(nnz, dtype=torch.int32, device=dev)
    idx2[pos] = idx
    val2[pos] = vals
    fld2[pos] = fields + 1
    del idx, vals, fields, rows, pos
    w = torch.ones(n, dtype=torch.float32, device=dev)
    if a.model == "multiclass":  # one-hot labels of a class drawn per row (the binary label picks the half)
        gen = torch.Generator(device=dev).manual_seed(5 + comm.rank)
        half = max(1, a.classes // 2)
        cls = torch.randint(0, half, (n,), device=dev, generator=gen) + (y[:, 0] > 0.5).long() * (a.classes - half)
        y = torch.nn.functional.one_hot(cls.clamp_max(a.classes - 1), a.classes).float()
        del cls
    tot = comm.allreduce_scalars([float(n)])[0]
    data = SparseData(ip2, idx2, val2, y, w, fld2 if a.model == "ffm" else None, None, tot, tot, float(n))
    params = CommonParams()
    params.loss.loss_function = (a.loss or "softmax") if a.model == "multiclass" else "sigmoid"
    params.loss.evaluate_metric = []
    params.model.need_bias = True
    params.model.data_path = "/tmp/ytk_bench_sparse_model"
    params.extra = {"k": [1, k], "bias_need_latent_factor": False}
    if a.model == "multiclass":
        params.extra = {"k": a.classes}
    if a.model.startswith("gb"):
        params.extra = {"k": a.experts, "tree_num": 1, "learning_rate": 1.0}
    log = YtkLogger(comm.rank, stream=sys.stderr)
    log.quiet = True
    loaded = LoadedData(data, None, _Names(F), {}, ["_bias_"] + [f"c{i}" for i in range(a.fields)])
    t0 = time.perf_counter()
    if a.model == "linear":
        from ytk_learn_amd.models.continuous.linear import LinearModel
        model = LinearModel(params, loaded, comm, log)
    elif a.model == "fm":
        from ytk_learn_amd.models.continuous.fm import FMModel
        model = FMModel(params, loaded, comm, log)
    elif a.model == "multiclass":
        from ytk_learn_amd.models.continuous.multiclass import MulticlassLinearModel
        model = MulticlassLinearModel(params, loaded, comm, log)
        k = a.classes
    elif a.model == "ffm":
        from ytk_learn_amd.models.continuous.ffm import FFMModel
        model = FFMModel(params, loaded, comm, log)
    else:  # gradient-boosted soft trees: one tree's L-BFGS evaluations (fused HIP epilogue)
        from ytk_learn_amd.models.gbst.model import GBSTModel
        model = GBSTModel(a.model, params, loaded, comm, log)
        model.init_w()
        model.next_sample(1.0, 1.0)
        k = a.experts
    setup_s = time.perf_counter() - t0
    if a.optimizer == "sgd":
        from ytk_learn_amd.optim.sgd import SGDOptimizer, SGDParams
        ng = model.ngroups if hasattr(model, "ngroups") else 1
        sgd = SGDOptimizer(model, SGDParams(learning_rate=0.05, batch_size=a.batch, epochs=1, dtype=a.dtype),
                           [0.0] * ng, [1e-6] * ng, comm, log, tot, tot)
        sgd._sync_copy(model.w)
        bounds = [(b, min(b + a.batch, n)) for b in range(0, n, a.batch)]

        t1 = time.perf_counter()
        batches = sgd._setup(bounds)  # per-batch column order, built once (not timed)
        sync()
        sgd_setup_s = time.perf_counter() - t1

        def epoch():
            for j, (b, e) in enumerate(bounds):
                sgd._step(model.w, b, e, 0.05, batches[j] if batches is not None else None)
            sgd._average(model.w)

        for _ in range(a.warmup):
            epoch()
        comm.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            epoch()
        sync()
        comm.barrier()
        el = time.perf_counter() - t0
        el = comm.allreduce_scalars([el], op="max")[0] if comm.is_dist else el
        pure, _ = sgd._losses(model.w)
        if comm.rank == 0:
            print(json.dumps({
                "metric": f"{a.model} SGD epoch (criteo-shape, {a.fields} fields, {a.features} features, k={k}, "
                          f"batch {a.batch})",
                "value": round(a.rows * comm.world / (el / a.steps), 1), "unit": "rows/s",
                "ms_per_step": round(1000.0 * el / a.steps, 3), "n_gpus": comm.world, "rows_per_gpu": a.rows,
                "dim": int(model.w.numel()), "nnz_per_row": a.fields + 1, "scaling": "weak", "dtype": a.dtype,
                "data": "synthetic Criteo-shape", "train_loss": pure / tot,
                "sgd_setup_s": round(sgd_setup_s, 3), "step": "column-ordered synchronous mini-batch",
            }), flush=True)
        comm.close()
        return
    ng = len(model.regular_groups()) if hasattr(model, "regular_groups") else getattr(model, "ngroups", 1)
    opt = HoagOptimizer(model, LineSearchParams(m=12), [0.0] * ng, [1e-6] * ng, comm, log, tot)
    g = torch.zeros_like(model.w)
    for _ in range(a.warmup):
        opt.loss_and_grad(model.w, g)
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    loss = 0.0
    for _ in range(a.steps):
        _, loss = opt.loss_and_grad(model.w, g)
    sync()
    comm.barrier()
    el = time.perf_counter() - t0
    el = comm.allreduce_scalars([el], op="max")[0] if comm.is_dist else el
    # one L-BFGS two-loop + direction update (history full: m pairs)
    # (history sharded over the ranks unless YTK_LBFGS_SHARD=0: this rank's slice of every pair,
    # the per-step dot partials all-reduced, p all-gathered once -- timed with that traffic)
    m = 12
    opt.setup_history(model.w.numel(), dev)
    if opt.shard and dev.type == "cuda":
        from ytk_learn_amd.parallel import peer as peer_mod
        P = comm.world
        opt._peer = peer_mod.make(comm, -(-max(model.w.numel(), P * opt.seg) * 4 // 8))
    opt.S.normal_(0.0, 1e-3)
    opt.Y.normal_(0.0, 1e-3)
    p = -g
    sync()
    t1 = time.perf_counter()
    opt.hv(p, 0, m, 1.0, 1.0)
    sync()
    hv_ms = (time.perf_counter() - t1) * 1000
    hist_mb = round(2 * opt.S.numel() * 4 / 2 ** 20, 1)
    # the local compute of one rank's sharded two-loop at P = 8: the same 12-pair recursion over
    # a 1/8 slice of the model vector (its 24 scalar all-reduces and the p all-gather excluded)
    seg8 = -(-(-(-model.w.numel() // 8)) // 4) * 4
    opt8 = HoagOptimizer(model, LineSearchParams(m=12), [0.0] * ng, [1e-6] * ng, None, log, tot)
    opt8.setup_history(seg8, dev)
    opt8.S.normal_(0.0, 1e-3)
    opt8.Y.normal_(0.0, 1e-3)
    p8 = torch.randn(seg8, device=dev)
    opt8.hv(p8, 0, m, 1.0, 1.0)  # warm
    sync()
    t1 = time.perf_counter()
    opt8.hv(p8, 0, m, 1.0, 1.0)
    sync()
    hv8_ms = (time.perf_counter() - t1) * 1000
    del opt8, p8
    if getattr(opt, "_peer", None) is not None:
        opt._peer.close()
    ms = 1000.0 * el / a.steps
    if comm.rank == 0:
        print(json.dumps({
            "metric": f"{a.model} L-BFGS loss+grad evaluation (criteo-shape, {a.fields} fields, "
                      f"{a.features} features, k={k})",
            "value": round(a.rows * comm.world / (el / a.steps), 1), "unit": "rows/s",
            "ms_per_step": round(ms, 3), "n_gpus": comm.world, "rows_per_gpu": a.rows, "dim": int(model.w.numel()),
            "nnz_per_row": a.fields + 1, "lbfgs_two_loop_ms": round(hv_ms, 3), "lbfgs_history_shard": bool(opt.shard),
            "lbfgs_two_loop_ms_local_at_1_8_slice": round(hv8_ms, 3),
            "lbfgs_history_mib_per_rank": hist_mb, "setup_s": round(setup_s, 2),
            "scaling": "weak", "dtype": "fp32", "data": "synthetic Criteo-shape", "loss": loss / tot,
            "gbst_fused": (os.environ.get("YTK_GBST_FUSED", "1") != "0") if a.model.startswith("gb") else None,
            "row_loss_fused": os.environ.get("YTK_ROW_LOSS", "1") != "0",
            "loss_function": params.loss.loss_function,
        }), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
