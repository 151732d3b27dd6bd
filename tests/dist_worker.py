"""Worker script for the multi-process tests (launched by torch.distributed.run).

usage: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
           --master-port P tests/dist_worker.py TASK OUT_DIR DEVICE
TASK: gbdt | gbdt_loss | linear | gbst | comm. Each task writes rank-0 results to OUT_DIR.
Row sharding: rank r takes rows r, r+N, ... of one fixed synthetic dataset, so any world
size sees the same global data.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("YTK_QUIET", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ytk_learn_amd.parallel.comm import Comm  # noqa: E402


def gbdt_data(n, F, seed, rank, world, device):
    g = np.random.default_rng(seed)
    X = g.integers(0, 40, size=(n, F)).astype(np.float32)  # < max_cnt distinct -> exact bins
    X[g.random((n, F)) < 0.05] = np.nan
    z = np.nansum(X[:, :4], axis=1) / 40.0 - 2.0 + 0.3 * g.normal(size=n)
    y = (z > 0).astype(np.float32)[:, None]
    sl = slice(rank, n, world)
    return torch.from_numpy(X[sl]).to(device), torch.from_numpy(y[sl]).to(device)


def run_gbdt(comm, out, device, policy, loss="sigmoid"):
    from ytk_learn_amd.models.gbdt.builder import TreeParams
    from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer
    X, y = gbdt_data(20000, 10, 7, comm.rank, comm.world, device)
    Xt, yt = gbdt_data(4000, 10, 8, comm.rank, comm.world, device)
    tp = TreeParams(max_depth=5 if policy == "level" else -1, max_leaf_cnt=32 if policy == "level" else 20,
                    min_child_hessian_sum=1.0, learning_rate=0.2, l2=1.0, grow_policy=policy,
                    feature_sample_rate=float(os.environ.get("YTK_TEST_FSAMPLE", "1.0")))
    p = GBDTParams(round_num=6, loss_function=loss, missing_value="value@0",
                   lad_refine_appr=os.environ.get("YTK_TEST_LAD_APPR", "0") == "1",
                   approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255}], tree=tp)
    tr = GBDTTrainer(p, GBDTData(X, y), GBDTData(Xt, yt), comm=comm)
    model = tr.train()
    tl, te = tr._losses()
    owner = bool(getattr(tr.builder, "owner", False))
    peer = getattr(tr.builder, "peer", None)
    if peer is not None:
        peer.check()
    peer_calls = peer.calls if peer is not None else 0
    slot_elems = int(getattr(tr.builder, "slot_elems", 0) or 0)
    peer_overlap = bool(getattr(tr.builder, "peer_overlap", False))
    overlap_times = getattr(tr.builder, "overlap_times", None)
    rccl_kcap = int(getattr(tr.builder, "RCCL_KCAP", 0) or 0)
    tr.close()
    if comm.log is not None:  # every rank's collective sequence (deadlock-freedom check)
        with open(os.path.join(out, f"comm_log_{comm.rank}.json"), "w") as f:
            json.dump(comm.log, f)
    if comm.rank == 0:
        with open(os.path.join(out, "model.txt"), "w") as f:
            f.write(model.dumps())
        with open(os.path.join(out, "res.json"), "w") as f:
            backend = torch.distributed.get_backend() if torch.distributed.is_initialized() else "none"
            json.dump({"train_loss": tl, "test_loss": te, "owner": owner, "comm": comm.stats,
                       "backend": backend, "is_dist": comm.is_dist,
                       "graph_replays": tr._graphs["n"] if isinstance(tr._graphs, dict) else 0,
                       "peer_calls": peer_calls, "slot_elems": slot_elems, "rccl_kcap": rccl_kcap,
                       "peer_overlap": peer_overlap, "overlap_times": overlap_times}, f)


def write_lines(path, n, seed, fields=False):
    """Sparse binary lines; fields=True names feature i "f<i % 3>@x<i>" (FFM field@name)."""
    w = np.random.default_rng(99).normal(size=30)
    g = np.random.default_rng(seed)
    name = (lambda i: f"f{i % 3}@x{i}") if fields else (lambda i: f"x{i}")
    with open(path, "w") as f:
        for _ in range(n):
            idx = np.unique(g.integers(0, 30, size=6))
            v = g.random(len(idx))
            y = int((w[idx] * v).sum() > 0)
            f.write("1###%d###%s\n" % (y, ",".join(f"{name(i)}:{x:.4f}" for i, x in zip(idx, v))))


def run_linear(comm, out, device, model_name, sgd=False):
    from ytk_learn_amd.config.hocon import parse_file
    from ytk_learn_amd.train import train
    tr_path, te_path = os.path.join(out, "train.txt"), os.path.join(out, "test.txt")
    ffm = model_name == "ffm"
    fd_path = os.path.join(out, "fields.txt")
    if comm.rank == 0 and not os.path.exists(tr_path):
        write_lines(tr_path, 4000, 1, fields=ffm)
        write_lines(te_path, 1000, 2, fields=ffm)
        with open(fd_path, "w") as f:
            f.write("f0\nf1\nf2\n")
    comm.barrier()
    cfg = parse_file(os.path.join(ROOT, "config", "model", f"{model_name}.conf")).with_overrides({
        "data.train.data_path": tr_path, "data.test.data_path": te_path,
        "model.data_path": os.path.join(out, f"{model_name}_w{comm.world}.model"),
        "optimization.line_search.lbfgs.convergence.max_iter": 10, "k": 4 if model_name != "fm" else [1, 4],
        "tree_num": 2})
    if ffm:
        cfg = cfg.with_overrides({"model.field_dict_path": fd_path, "k": [1, 4]})
    if sgd:
        cfg = cfg.with_overrides({"optimization.optimizer": "sgd", "optimization.sgd.learning_rate": 0.05,
                                  "optimization.sgd.batch_size": 128, "optimization.sgd.epochs": 4,
                                  "optimization.sgd.sync_every": 5})
    res = train(model_name, cfg, comm=comm)
    if comm.rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            if sgd:
                json.dump({"loss": res[0], "test_loss": res[1]}, f)
            else:
                json.dump({"loss": res.loss, "test_loss": res.test_loss}, f)


def run_comm(comm, out, device):
    t = torch.full((4,), float(comm.rank + 1), device=device)
    comm.allreduce_(t)
    m = comm.allreduce(torch.tensor([float(comm.rank)], device=device), op="max")
    g = comm.allgather(torch.tensor([comm.rank], device=device))
    o = comm.allreduce_object({f"k{comm.rank}": 1, "shared": 2}, lambda a, b: {k: a.get(k, 0) + b.get(k, 0)
                                                                               for k in set(a) | set(b)})
    rs = torch.empty(2, device=device)
    comm.reduce_scatter_(rs, torch.arange(2 * comm.world, dtype=torch.float32, device=device))
    # keyed merge: rank r holds names f0..f(10+r), "only_r", and unicode "xé" (sum, max, min)
    names = [f"f{i}" for i in range(10 + comm.rank)] + [f"only_{comm.rank}", "x\u00e9"]
    vals = [[1.0, float(comm.rank), float(comm.rank)] for _ in names]
    mn, mv = comm.merge_named(names, vals, ["sum", "max", "min"])
    if comm.rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            json.dump({"sum": t.tolist(), "max": m.tolist(), "gather": g.tolist(), "obj": o,
                       "rs": rs.tolist(), "range": list(comm.shard_range(10)),
                       "merged": dict(zip(mn, mv.tolist()))}, f)


def run_binning(comm, out, device):
    """Batched tensor-exchange binning vs the per-feature path (and the quantile fill)."""
    from ytk_learn_amd.models.gbdt import binning as bn
    g = torch.Generator().manual_seed(7 + comm.rank)
    n = 3000 + 500 * comm.rank
    cols = [torch.randint(0, 40, (n,), generator=g).float(),               # few distinct: union path
            torch.round(torch.randn(n, generator=g) * 100) / 10,           # many distinct: summaries
            torch.randn(n, generator=g),
            torch.full((n,), float(comm.rank))]
    X = torch.stack(cols, 1).to(device)
    w = (torch.rand(n, generator=g) + 0.5).to(device)
    specs = [bn.SamplerSpec(max_cnt=63), bn.SamplerSpec(max_cnt=31, use_sample_weight=True),
             bn.SamplerSpec(max_cnt=255, quantile_approximate_bin_factor=4), bn.SamplerSpec(max_cnt=8)]
    fit = bn.BinMapper.fit(X, w, specs, comm)
    per = [bn.feature_candidates(X[:, f].contiguous(), w, specs[f], comm) for f in range(4)]
    Xn = X.clone()
    Xn[::7, 1] = float("nan")
    fill = bn.compute_missing_fill(Xn, w, "quantile@0.3", comm)
    if comm.rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            json.dump({"fit": [c.tolist() for c in fit.cands], "per": [c.tolist() for c in per],
                       "fill": fill.tolist()}, f)


def run_samplers(comm, out, device):
    """Non-quantile samplers (no_sample, sample_by_precision, sample_by_cnt, sample_by_rate) on
    row shards of one global dataset: candidates through ragged tensor all-gathers."""
    from ytk_learn_amd.models.gbdt import binning as bn
    g = np.random.default_rng(5)
    n = 6000
    X = np.stack([g.integers(0, 300, n).astype(np.float32),
                  np.round(g.normal(size=n) * 50, 2).astype(np.float32),
                  np.exp(g.normal(size=n)).astype(np.float32)], 1)
    Xs = torch.from_numpy(X[comm.rank::comm.world]).to(device)
    res = {}
    res["no_sample"] = bn.feature_candidates(Xs[:, 0].contiguous(), None, bn.SamplerSpec(type="no_sample"),
                                             comm).tolist()
    res["precision"] = bn.feature_candidates(
        Xs[:, 2].contiguous(), None, bn.SamplerSpec(type="sample_by_precision", dot_precision=2, use_log=True,
                                                    use_min_max=True), comm).tolist()
    # random samplers: the result must be the union of what every rank selected
    for t, kw in (("sample_by_cnt", {"max_cnt": 100}), ("sample_by_rate", {"sample_rate": 0.3, "min_cnt": 10})):
        got = bn.feature_candidates(Xs[:, 1].contiguous(), None, bn.SamplerSpec(type=t, **kw), comm, seed=3)
        res[t + "_size"] = len(got)
        res[t + "_sorted_unique"] = bool(np.all(np.diff(got) > 0))
    res["ops"] = sorted({op for op, _, _ in (comm.log or [])})
    if comm.rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            json.dump(res, f)


def run_peer_ops(comm, out, device):
    """The peer-memory exchange primitives against their definitions, every dtype and both
    exchange shapes: all-reduce (one-shot / two-shot by size), reduce-scatter and all-gather
    of P equal segments (int64 exact, floats summed in rank order)."""
    from ytk_learn_amd.parallel import peer as peer_mod
    P, r = comm.world, comm.rank
    pr = peer_mod.make(comm, 1 << 19)  # 4 MiB slabs: the 2.5 MB message runs two-shot
    res = {"peer": pr is not None, "ok": []}
    if pr is not None:
        for dt in (torch.int64, torch.float64, torch.float32):
            for n in (4 * P, 4099 * 4 * P, 160000 * 4 * P):  # P segments of whole 16-B units
                n = min(n, pr.cap_bytes // torch.tensor([], dtype=dt).element_size() // (4 * P) * (4 * P))

                def val(q):  # rank q's contribution, exactly representable in every dtype
                    return (torch.arange(n, dtype=torch.float64, device=device) % 97 + 3 * q).to(dt)

                want = sum(val(q).double() for q in range(P))
                t = val(r).clone()
                pr.allreduce_(t)
                ok_ar = bool(torch.equal(t.double(), want))
                t = val(r).clone()
                seg = pr.reduce_scatter_(t)
                ok_rs = bool(torch.equal(seg.double(), want.view(P, -1)[r]))
                g = val(0).view(P, -1).clone()
                g[r] = val(r).view(P, -1)[r] * 2
                pr.allgather_(g.view(-1))
                expect = torch.stack([val(q).view(P, -1)[q] * 2 for q in range(P)])
                ok_ag = bool(torch.equal(g, expect))
                res["ok"].append([str(dt), n, ok_ar, ok_rs, ok_ag])
        torch.cuda.synchronize(device)
        pr.check()
        pr.close()
    if comm.rank == 0:
        with open(os.path.join(out, "res.json"), "w") as f:
            json.dump(res, f)


def main():
    task, out, device = sys.argv[1], sys.argv[2], sys.argv[3]
    comm = Comm.from_env(device)
    dev = comm.device
    try:
        if task == "gbdt":
            run_gbdt(comm, out, dev, "level")
        elif task == "gbdt_loss":
            run_gbdt(comm, out, dev, "loss")
        elif task == "gbdt_l1":  # l1 loss: leaf refine by the exact distributed weighted median
            run_gbdt(comm, out, dev, "level", loss="l1")
        elif task in ("linear", "fm", "ffm", "gbmlr", "gbhsdt", "multiclass_linear"):
            run_linear(comm, out, dev, task)
        elif task in ("fm_sgd", "linear_sgd", "ffm_sgd"):
            run_linear(comm, out, dev, task.split("_")[0], sgd=True)
        elif task == "binning":
            run_binning(comm, out, dev)
        elif task == "samplers":
            run_samplers(comm, out, dev)
        elif task == "comm":
            run_comm(comm, out, dev)
        elif task == "peer_ops":
            run_peer_ops(comm, out, dev)
        else:
            raise SystemExit(f"unknown task {task}")
    finally:
        comm.close()


if __name__ == "__main__":
    main()
