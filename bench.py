#!/usr/bin/env python3
"""Headline benchmark: Higgs-shaped GBDT, sec/tree, on 1..8 MI355X (one rank per GPU).

Config (BASELINE.json / BASELINE.md target (b)): 10.5M train + 0.5M test rows x 28
features (the Higgs split, docs/gbdt_experiments.md:9), level-wise depth 6
(max_leaf_cnt 255 -> min(255, 2^6) = 64 leaves), 255 quantile bins (alpha 0.5),
lr 0.1, l1 = l2 = 0, min_child_hessian_sum 100 -- the reference's
experiment/higgs/local_gbdt.conf with tree_grow_policy=level, max_depth=6.
``--policy loss`` runs the reference-identical leaf-wise 255-leaf shape (a).

A "step" is one whole reference boosting round (GBDTOptimizer.java:406-462): one
tree + train-score update + train loss/gradients for the next tree + incremental
test-set scoring and test loss + the round's model conversion (convertModel: slot ->
raw threshold, feature names, default directions, :431 / :663-690) + the per-round
(train, test) loss readback (:457-462). Conversion and readback are pipelined one
round behind the GPU (pinned buffers + events); the timed region ends only after
every timed tree is a host model tree and every loss has landed.
Scaling is STRONG: the 10.5M rows are sharded over the N ranks.

``vs_baseline`` is null: the reference publishes no depth-6 level-wise number. The
reference-identical shape (leaf-wise, 255 leaves) is timed separately on the same
data (every N) and reported as ``leafwise_s_per_tree`` / ``leafwise_vs_reference``
(÷ 1.136 s/tree, docs/gbdt_experiments.md:104).

Multi-GPU design A/B (N > 1, ``--variants auto``): after the headline, short extra timed runs
(2 untimed + ``--variant-steps`` timed level-wise trees each, a fresh trainer per variant) of
the choices a one-GPU box cannot measure -- the half-level exchange overlapped with the build
forced on / off (``overlap_on`` / ``overlap_off``; the headline's default ``auto`` times both on
trees 1-4 and keeps the faster, reported as ``overlap_auto_us``), the other histogram sync mode (``owner`` / ``allreduce``), RCCL instead of
the peer-memory exchange (``rccl``) and RCCL with its half-level overlap (``rccl_overlap``) --
reported under ``variants`` in the same JSON line. Each runs in its own try block followed by
an all-rank vote: a variant that fails on any rank is reported as ``{"error": ...}``, ends the
variant list and leaves the headline intact.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N>1 the driver launches it under torch.distributed.run (RANK/WORLD_SIZE env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import traceback
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
if os.environ.get("WORLD_SIZE", "1") == "1" and os.environ.get("YTK_FORCE_DIST") != "1":
    os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see ytk_learn_amd/__init__.py

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ytk_learn_amd.data.synthetic import higgs_like_rows  # noqa: E402
from ytk_learn_amd.models.gbdt.builder import TreeParams  # noqa: E402
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer  # noqa: E402
from ytk_learn_amd.parallel import peer as peer_mod  # noqa: E402
from ytk_learn_amd.parallel.comm import Comm  # noqa: E402
from ytk_learn_amd.utils.fault import fault_point  # noqa: E402
from ytk_learn_amd.utils.logging import YtkLogger  # noqa: E402

BASELINE_SEC_PER_TREE = 1.136  # ytk-learn 567.83 s / 500 trees (docs/gbdt_experiments.md:104)
METRIC = "Higgs-11M GBDT: sec/tree (500 trees, depth 6, 255 bins) at 1/2/4/8 MI355X"


def timed_rounds(tr, comm, dev, warmup: int, steps: int) -> float:
    """W untimed + K timed whole rounds; returns the max-over-ranks wall time of the K."""
    for i in range(warmup):
        tr.run_round(i)
    tr.materialize()
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    comm.reset_stats()
    peer = getattr(tr.builder, "peer", None)
    x0 = peer.timing() if peer is not None else (0, 0.0)
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        fault_point("bench", i, comm.rank)  # YTK_FAULT_INJECT=bench:<rank>:<round>:stall (tests)
        tr.run_round(i)
    tr.materialize()  # the last round's trees and losses land inside the timed region
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    comm.barrier()
    el = time.perf_counter() - t0
    timed_stats = dict(comm.stats)
    if peer is not None:  # device-timed peer exchanges of the timed rounds (outside the timing)
        x1 = peer.timing()
        timed_stats["peer_exchanges"] = x1[0] - x0[0]
        timed_stats["peer_us"] = x1[1] - x0[1]
    el = comm.allreduce_scalars([el], op="max")[0] if comm.is_dist else el
    comm.stats = timed_stats  # the timed rounds' collectives only
    return el


def _transport(comm, builder) -> str:
    if not comm.is_dist:
        return "none"
    if getattr(builder, "peer", None) is not None:
        return "peer"
    return dist.get_backend(comm.group) if comm.group is not None else "none"


# (name, environment of the variant's trainer); "sync_alt" is the histogram sync mode the
# headline did not use (owner <-> allreduce)
VARIANTS = [
    ("overlap_on", {"YTK_PEER_OVERLAP": "1"}),
    ("overlap_off", {"YTK_PEER_OVERLAP": "0"}),
    ("sync_alt", {}),
    ("rccl", {"YTK_PEER_REDUCE": "0"}),
    ("rccl_overlap", {"YTK_PEER_REDUCE": "0", "YTK_HIST_OVERLAP_MIN_ROWS": "0"}),
]
VARIANT_NAMES = [v[0] for v in VARIANTS]


def _exchange_keys(coll, steps):
    """Per-tree collective / device-timed exchange accounting of a timed run."""
    n_x = coll.get("peer_exchanges", coll["calls"])
    out = {"collectives_per_tree": round(coll["calls"] / steps, 2),
           "exchanges_per_tree": round(n_x / steps, 2),
           "exchange_us_per_tree": (round(coll["peer_us"] / steps, 2) if "peer_us" in coll else None),
           # device wall time of one exchange (a built level's histogram message, or the round
           # vector) -- the per-level exchange cost at this N
           "exchange_us_per_level": (round(coll["peer_us"] / n_x, 2) if "peer_us" in coll and n_x else None)}
    return out


class _Env:
    """Temporarily set environment variables (identical on every rank)."""

    def __init__(self, kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_variants(a, comm, dev, data, params, headline_sync, log):
    """The multi-GPU design A/B (module docstring): each variant is a fresh trainer, 2 untimed
    + a.variant_steps timed trees; an all-rank vote after each one stops the list on a failure
    anywhere (the ranks then agree on the collectives they issue next)."""
    if a.variants == "none" or (a.variants == "auto" and comm.world <= 1):
        return None
    names = VARIANT_NAMES if a.variants in ("auto", "all") else [v for v in a.variants.split(",") if v]
    X, y, Xt, yt = data
    out = {}
    t_start = time.perf_counter()
    for name in names:
        # bounded: the variants never cost the headline more than --variant-budget seconds
        # (agreed over the ranks, so every rank stops at the same variant)
        spent = time.perf_counter() - t_start
        if comm.is_dist:
            spent = comm.allreduce_scalars([spent], op="max")[0]
        if spent > a.variant_budget:
            out[name] = {"skipped": f"variant time budget ({a.variant_budget:.0f} s) spent"}
            continue
        env = dict(dict(VARIANTS).get(name, {}))
        # a stuck peer exchange fails the variant in seconds, not the job's 120 s
        env.setdefault("YTK_PEER_TIMEOUT_S", "30")
        if name == "sync_alt":
            env["YTK_HIST_SYNC"] = "owner" if headline_sync != "owner" else "allreduce"
        t0 = time.perf_counter()
        res, err = None, None
        try:
            with _Env(env):
                if os.environ.get("YTK_BENCH_FAIL_VARIANT") == name:  # tests: a variant that fails
                    raise RuntimeError(f"injected failure in variant {name}")
                pv = GBDTParams(round_num=2 + a.variant_steps, loss_function="sigmoid", eval_metric=[],
                                missing_value="value@0", approximate=params.approximate, tree=params.tree)
                trv = GBDTTrainer(pv, GBDTData(X, y), GBDTData(Xt, yt), comm=comm, log=log)
                trv.prepare()
                trv.init_gradients()
                el = timed_rounds(trv, comm, dev, 2, a.variant_steps)
                coll = dict(comm.stats)
                res = {"s_per_tree": round(el / a.variant_steps, 6), "env": env,
                       "transport": _transport(comm, trv.builder),
                       "hist_sync": "owner" if getattr(trv.builder, "owner", False) else "allreduce",
                       "overlap": _overlap(comm, trv.builder),
                       "graph_replays": trv._graphs["n"] if isinstance(trv._graphs, dict) else 0}
                res.update(_exchange_keys(coll, a.variant_steps))
                trv.close()
                del trv
        except Exception as e:  # noqa: BLE001 -- reported in the line; the headline stands
            traceback.print_exc()
            err = f"{type(e).__name__}: {e}"[:300]
            peer = getattr(getattr(locals().get("trv"), "builder", None), "peer", None)
            if peer is not None:
                peer.abort()
        ok = comm.allreduce_scalars([0.0 if err is not None else 1.0], op="min")[0] > 0.5 if comm.is_dist \
            else err is None
        if not ok:
            out[name] = {"error": err or "failed on another rank", "env": env}
            break
        res["wall_s"] = round(time.perf_counter() - t0, 2)
        out[name] = res
    return out


def _overlap(comm, builder) -> bool:
    """Half-level exchange / all-reduce overlapped with the other half's build."""
    return bool(getattr(builder, "peer_overlap", False)
                or (getattr(builder, "overlap", False) and comm.is_dist and getattr(builder, "peer", None) is None))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--train-rows", type=int, default=10_500_000)
    ap.add_argument("--test-rows", type=int, default=500_000)
    ap.add_argument("--policy", default="level", choices=["level", "loss"])
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--leaves", type=int, default=255)
    ap.add_argument("--bins", type=int, default=255)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--device", default=None)
    ap.add_argument("--profile", action="store_true", help="sync per phase and print time stats")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--leafwise-steps", type=int, default=None,
                    help="extra timed leaf-wise 255-leaf rounds on the same data (default 10)")
    ap.add_argument("--variants", default="auto",
                    help="multi-GPU design A/B after the headline: auto (N > 1 only) | none | all | "
                         "comma list of " + ",".join(VARIANT_NAMES))
    ap.add_argument("--variant-steps", type=int, default=8, help="timed level-wise trees per variant")
    ap.add_argument("--variant-budget", type=float, default=90.0,
                    help="seconds after which the remaining variants are skipped")
    a = ap.parse_args()

    # a stuck rank must fail the job well inside the driver's bench timeout: every collective
    # (and peer-exchange flag wait) times out after YTK_COMM_TIMEOUT seconds (default 120)
    os.environ.setdefault("YTK_PEER_TIMEOUT_S", os.environ.get("YTK_COMM_TIMEOUT", "120"))
    comm = Comm.from_env(device=a.device, timeout_s=120)
    try:
        run(a, comm)
    except BaseException as e:  # noqa: BLE001 -- report, then exit non-zero (never re-exec)
        traceback.print_exc()
        print(f"[bench] rank {comm.rank} failed: {type(e).__name__}: {e}; last collective issued: "
              f"{comm.last_op}", file=sys.stderr, flush=True)
        os._exit(1)
    comm.close()


def run(a, comm):
    dev = comm.device
    world, rank = comm.world, comm.rank
    if world != a.gpus and rank == 0:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    # strong scaling: ONE global dataset (chunk-seeded), rank r keeps rows
    # [r * n / N, (r + 1) * n / N) -- every N trains and tests on the same rows
    t0 = time.perf_counter()
    X, y = higgs_like_rows(a.train_rows, *comm.shard_range(a.train_rows), seed=a.seed * 1000, device=dev)
    Xt, yt = higgs_like_rows(a.test_rows, *comm.shard_range(a.test_rows), seed=a.seed * 1000 + 500, device=dev)
    gen_s = time.perf_counter() - t0

    tp = TreeParams(max_depth=a.depth if a.policy == "level" else -1, max_leaf_cnt=a.leaves,
                    min_child_hessian_sum=100.0, min_split_loss=0.0, min_split_samples=-1,
                    learning_rate=0.1, l1=0.0, l2=0.0, grow_policy=a.policy)
    if a.policy == "level":
        tp.max_leaf_cnt = min(a.leaves, 1 << a.depth)  # GBDTOptimizationParams.java:148-154
    total_rounds = a.warmup + a.steps
    params = GBDTParams(round_num=total_rounds, loss_function="sigmoid", eval_metric=["auc"],
                        missing_value="value@0",
                        approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": a.bins,
                                      "use_sample_weight": False, "alpha": 0.5}],
                        tree=tp)
    log = YtkLogger(rank, stream=sys.stderr, every=10)
    if a.quiet:
        log.quiet = True
    tr = GBDTTrainer(params, GBDTData(X, y), GBDTData(Xt, yt), comm=comm, log=log, profile=a.profile)
    t0 = time.perf_counter()
    tr.prepare()
    tr.init_gradients()  # initial prediction + gradients (GBDTOptimizer.initPred)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    prep_s = time.perf_counter() - t0
    # multi-GPU: the histogram-exchange overlap is auto-tuned on trees 1-4 (eager, event-timed;
    # DeviceLevelBuilder.OVERLAP_TRIAL) and the round graphs are captured on the tree after
    # them (with the RCCL watchdog drain before it, ~100 ms: Comm.drain_pending), so those
    # trees are always untimed: a warmup below 6 gets the missing rounds added when the
    # engine tunes (reported as warmup_autotune_extra)
    need = max(getattr(tr.builder, "OVERLAP_TRIAL", (4,))) + 2
    extra = max(0, need - a.warmup) if getattr(tr.builder, "tuning", False) else 0
    warmup = a.warmup + extra
    total_rounds += extra

    el_max = timed_rounds(tr, comm, dev, warmup, a.steps)
    assert len(tr.model.trees) == total_rounds, "every timed tree must be a converted host tree"
    coll = dict(comm.stats)
    replays = tr._graphs["n"] if isinstance(tr._graphs, dict) else 0
    # quality check after the timed rounds (outside timing): losses and AUC over the GLOBAL
    # train / test rows (the evaluators all-reduce their bucket histograms)
    auc = tr.eval_test.evals[0].compute(yt, tr.te_pred, None, comm)[0]
    train_auc = tr.eval_train.evals[0].compute(y, tr.pred, None, comm)[0]
    train_loss, test_loss = tr.round_losses[total_rounds - 1]
    sec_per_tree = el_max / a.steps
    transport = _transport(comm, tr.builder)
    if a.profile and rank == 0:
        print(tr.timer.report() if tr.use_device_builder else tr.builder.total_stats, file=sys.stderr)
    if rank == 0 and hasattr(tr.builder, "prof_report") and os.environ.get("YTK_LW_PROF") == "1":
        print("leafwise planner profile (warmup + timed trees): " + json.dumps(tr.builder.prof_report()),
              file=sys.stderr)
    tr_builder = tr.builder
    leaf_steps = a.leafwise_steps if a.leafwise_steps is not None else 10
    leaf = leaf_transport = leaf_error = None
    leaf_coll = {}
    tr.close()
    if leaf_steps > 0 and a.policy == "level":
        del tr
        tpl = TreeParams(max_depth=-1, max_leaf_cnt=255, min_child_hessian_sum=100.0, min_split_loss=0.0,
                         min_split_samples=-1, learning_rate=0.1, l1=0.0, l2=0.0, grow_policy="loss")
        pl = GBDTParams(round_num=3 + leaf_steps, loss_function="sigmoid", eval_metric=["auc"],
                        missing_value="value@0", approximate=params.approximate, tree=tpl)
        # an extra key: a failure here is reported in the line instead of losing the headline
        try:
            trl = GBDTTrainer(pl, GBDTData(X, y), GBDTData(Xt, yt), comm=comm, log=log)
            trl.prepare()
            trl.init_gradients()
            leaf = timed_rounds(trl, comm, dev, 3, leaf_steps) / leaf_steps
            leaf_coll = dict(comm.stats)
            assert len(trl.model.trees) == 3 + leaf_steps
            leaf_transport = _transport(comm, trl.builder)
            trl.close()
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            leaf, leaf_error = None, f"{type(e).__name__}: {e}"[:300]
            peer = getattr(getattr(locals().get("trl"), "builder", None), "peer", None)
            if peer is not None:
                peer.abort()  # queued exchanges return at once: the device drains, the job ends
    headline_sync = ("owner" if getattr(tr_builder, "owner", False) else "allreduce") if comm.is_dist else "none"
    variants = run_variants(a, comm, dev, (X, y, Xt, yt), params, headline_sync, log) if a.policy == "level" else None
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(sec_per_tree, 6),
            "unit": "s/tree",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_autotune_extra": extra,
            "ms_per_step": round(1000.0 * sec_per_tree, 4),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": (round(sec_per_tree / BASELINE_SEC_PER_TREE, 6) if a.policy == "loss"
                            and a.leaves == 255 else None),
            "dtype": "fp32",
            "data": "synthetic Higgs-shape (10.5M train + 0.5M test x 28 dense float features, random-init trees)",
            "config": {
                "model": f"gbdt {a.policy}-wise depth{a.depth if a.policy == 'level' else '-unlimited'} leaves{tp.max_leaf_cnt} bins{a.bins} sigmoid lr0.1",
                "global_batch": a.train_rows,
                "seq_len": 28,
                "parallelism": f"dp{world}",
                "test_rows": a.test_rows,
                "rounds_timed": a.steps,
                "device": str(dev),
            },
            "train_loss": round(float(train_loss), 6),
            "test_loss": round(float(test_loss), 6),
            "train_auc": round(float(train_auc), 6),
            "test_auc": round(float(auc), 6),
            "quality_on": "global train / test rows (identical data at every N)",
            "prep_s": round(prep_s, 3),
            "datagen_s": round(gen_s, 3),
            "timed_region": "step + convertModel + per-round loss readback (pipelined), all trees landed",
            "collectives_per_tree": round(coll["calls"] / a.steps, 2),
            "collective_bytes_per_tree": int(coll["bytes"] / a.steps),
            "hist_sync": headline_sync,
            "hist_transport": transport,
            # half-level exchange / all-reduce overlapped with the other half's build
            "overlap": _overlap(comm, tr_builder),
            # auto-tuned overlap: (off, on) device us per trial tree, max over ranks
            "overlap_auto_us": getattr(tr_builder, "overlap_times", None),
            "graph_replays": replays,
            "trees_converted": total_rounds,
            # multi-GPU diagnostics: the start-up self-test of the peer-memory path (on a vote
            # for RCCL, the reason) and the device-timed exchanges of the timed trees
            "peer_selftest": (peer_mod.LAST_STATUS["state"] + (": " + peer_mod.LAST_STATUS["reason"]
                                                               if peer_mod.LAST_STATUS["reason"] else ""))
            if comm.is_dist else "n/a",
        }
        res.update({k: v for k, v in _exchange_keys(coll, a.steps).items() if k != "collectives_per_tree"})
        if leaf is not None:
            res["leafwise_s_per_tree"] = round(leaf, 6)
            res["leafwise_vs_reference"] = round(leaf / BASELINE_SEC_PER_TREE, 6)
            res["leafwise_rounds_timed"] = leaf_steps
            res["leafwise_transport"] = leaf_transport
            if "peer_us" in leaf_coll:
                res["leafwise_exchanges_per_tree"] = round(leaf_coll["peer_exchanges"] / leaf_steps, 2)
                res["leafwise_exchange_us_per_tree"] = round(leaf_coll["peer_us"] / leaf_steps, 2)
        if leaf_error is not None:
            res["leafwise_error"] = leaf_error
        if variants is not None:
            res["variants"] = variants
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
