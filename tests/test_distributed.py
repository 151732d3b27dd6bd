"""Multi-process tests of the distributed paths (torch.distributed.run, 127.0.0.1).

CPU: gloo, world 1 vs world 2 -- GBDT must produce the IDENTICAL model text (exact int64
histograms, feature-ownership-free all-reduce), L-BFGS models must reach the same loss.
GPU (@gpu): two ranks share the one GPU of the test box over gloo (YTK_DIST_BACKEND=gloo),
exercising the GPU-resident level builder's collectives (root count, max |g|/|h|, per-level
left counts and histogram slabs) -- RCCL itself needs one GPU per rank.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _head_tail(text, n=4000):
    if len(text) <= 2 * n:
        return text
    return text[:n] + f"\n[... {len(text) - 2 * n} characters ...]\n" + text[-n:]


def _run(task, out, world, device="cpu", timeout=600, extra_env=None):
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    env["OMP_NUM_THREADS"] = "2"
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER, task, str(out), device]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    with open(os.path.join(out, "stderr.log"), "w") as f:  # the whole worker stderr, kept with the run
        f.write(r.stderr)
    # the head of stderr holds an abort's what() message, the tail the launcher's report
    assert r.returncode == 0, r.stdout[-3000:] + _head_tail(r.stderr)
    with open(os.path.join(out, "res.json")) as f:
        return json.load(f)


def test_comm_collectives_gloo(tmp_path):
    res = _run("comm", tmp_path, 2)
    assert res["sum"] == [3.0] * 4
    assert res["max"] == [1.0]
    assert res["gather"] == [0, 1]
    assert res["obj"] == {"k0": 1, "k1": 1, "shared": 4}
    assert res["rs"] == [0.0, 2.0]  # rank 0 gets elements [0, 2) summed over 2 ranks
    assert res["range"] == [0, 5]
    mg = res["merged"]
    assert mg["f0"] == [2.0, 1.0, 0.0] and mg["f10"] == [1.0, 1.0, 1.0]
    assert mg["only_0"] == [1.0, 0.0, 0.0] and mg["only_1"] == [1.0, 1.0, 1.0]
    assert mg["x\u00e9"] == [2.0, 1.0, 0.0] and len(mg) == 14


@pytest.mark.parametrize("world", [1, 3])
def test_binning_tensor_exchange_matches_per_feature(tmp_path, world):
    """BinMapper.fit's batched exchange (one distinct-count all-reduce + one ragged tensor
    all-gather of device-pruned summaries / distinct values) == the per-feature path."""
    res = _run("binning", tmp_path, world, extra_env={"YTK_COMM_LOG": "1"})
    for a, b in zip(res["fit"], res["per"]):
        assert np.array_equal(np.float32(a), np.float32(b))
    assert all(np.isfinite(res["fill"]))


@pytest.mark.parametrize("world", [2, 4])
def test_non_quantile_samplers_tensor_union_world_n(tmp_path, world):
    """no_sample / sample_by_precision candidates over row shards == the single-rank ones
    (the union travels as ragged tensors, not pickled objects); the random samplers return a
    sorted union."""
    r1 = _run("samplers", tmp_path / "w1", 1, extra_env={"YTK_COMM_LOG": "1"})
    rn = _run("samplers", tmp_path / f"w{world}", world, extra_env={"YTK_COMM_LOG": "1"})
    assert rn["no_sample"] == r1["no_sample"]
    np.testing.assert_allclose(rn["precision"], r1["precision"], rtol=1e-6)
    for t in ("sample_by_cnt", "sample_by_rate"):
        assert rn[t + "_sorted_unique"] and rn[t + "_size"] > 0
    assert "allgather_object" not in rn["ops"]  # no pickled collectives


@pytest.mark.parametrize("task", ["gbdt", "gbdt_loss"])
def test_gbdt_world2_identical_to_world1(tmp_path, task):
    r1 = _run(task, tmp_path / "w1", 1)
    r2 = _run(task, tmp_path / "w2", 2)
    m1 = open(tmp_path / "w1" / "model.txt").read()
    m2 = open(tmp_path / "w2" / "model.txt").read()
    assert m1 == m2
    np.testing.assert_allclose(r2["train_loss"], r1["train_loss"], rtol=1e-9)
    np.testing.assert_allclose(r2["test_loss"], r1["test_loss"], rtol=1e-9)


@pytest.mark.parametrize("task,world,mode,fs", [
    ("gbdt", 2, "owner", "1.0"), ("gbdt", 4, "owner", "0.6"), ("gbdt", 8, "owner", "1.0"),
    ("gbdt", 8, "allreduce", "0.6"), ("gbdt_loss", 4, "owner", "1.0"), ("gbdt_loss", 8, "allreduce", "1.0"),
    ("gbdt_loss", 8, "owner", "0.6")])
def test_gbdt_world_n_both_sync_modes(tmp_path, task, world, mode, fs):
    """World 2/4/8 (gloo, CPU) == world 1 byte for byte, with the histogram all-reduce
    and with owner-computes (reduce-scatter by feature block + allgather of split records;
    with 10 features and 8 ranks some ranks own one feature, with feature sampling some
    own no sampled feature at all)."""
    env = {"YTK_HIST_SYNC": mode, "YTK_TEST_FSAMPLE": fs, "YTK_COMM_LOG": "1"}
    _run(task, tmp_path / "w1", 1, extra_env=env)
    r = _run(task, tmp_path / f"w{world}", world, extra_env=env)
    assert r["owner"] == (mode == "owner")
    assert open(tmp_path / "w1" / "model.txt").read() == open(tmp_path / f"w{world}" / "model.txt").read()
    _same_collective_sequence(tmp_path / f"w{world}", world)


def _same_collective_sequence(out, world):
    """Every rank issued the identical collective sequence (op, dtype, size): under RCCL a
    mismatch would hang, so this is the CPU-checkable form of the ordering contract."""
    logs = [json.load(open(os.path.join(out, f"comm_log_{r}.json"))) for r in range(world)]
    assert len(logs[0]) > 0
    for r in range(1, world):
        assert logs[r] == logs[0], f"rank {r} collective sequence differs from rank 0"


@pytest.mark.parametrize("world", [2, 4])
def test_gbdt_l1_exact_refine_world_n(tmp_path, world):
    """TreeRefiner exact mode (lad_refine_appr = false) across ranks: the bucketed
    distributed weighted median gives the world-1 (single sort) leaf values."""
    _run("gbdt_l1", tmp_path / "w1", 1)
    _run("gbdt_l1", tmp_path / f"w{world}", world,
         extra_env={"YTK_COMM_LOG": "1", "YTK_MEDIAN_GATHER_MAX": "64" if world == 4 else "8192"})
    assert open(tmp_path / "w1" / "model.txt").read() == open(tmp_path / f"w{world}" / "model.txt").read()
    _same_collective_sequence(tmp_path / f"w{world}", world)


@pytest.mark.parametrize("task,world,shard", [("linear", 2, "1"), ("gbmlr", 2, "1"), ("linear", 8, "1"),
                                              ("gbmlr", 4, "1"), ("fm", 2, "1"), ("fm", 4, "1"), ("ffm", 2, "1"),
                                              ("ffm", 4, "1"), ("linear", 4, "1"), ("linear", 2, "0"),
                                              ("ffm", 2, "0")])
def test_lbfgs_world_n_matches_world1(tmp_path, task, world, shard):
    """L-BFGS at world N (gloo) reaches the world-1 losses: with the (s, y) history sharded
    over the ranks (shard "1", the default: per-step dot partials all-reduced, p all-gathered;
    HoagOptimizer.java:441-449,904-929) and replicated (YTK_LBFGS_SHARD=0)."""
    r1 = _run(task, tmp_path / "w1", 1)
    r2 = _run(task, tmp_path / f"w{world}", world, extra_env={"YTK_LBFGS_SHARD": shard})
    np.testing.assert_allclose(r2["loss"], r1["loss"], rtol=1e-4)
    np.testing.assert_allclose(r2["test_loss"], r1["test_loss"], rtol=1e-3)
    if task == "linear":
        parts = os.listdir(tmp_path / f"w{world}" / f"linear_w{world}.model")
        assert sorted(parts) == [f"model-{r:05d}" for r in range(world)]  # each rank dumps its feature range


@pytest.mark.gpu
@pytest.mark.parametrize("task,world,mode", [("gbdt", 2, "allreduce"), ("gbdt", 4, "allreduce"),
                                             ("gbdt_loss", 3, "allreduce"), ("gbdt", 3, "owner"),
                                             ("gbdt", 4, "owner"), ("gbdt_loss", 2, "owner"),
                                             ("gbdt", 2, "peer"), ("gbdt_loss", 2, "peer"), ("gbdt", 3, "peer"),
                                             ("gbdt_loss", 3, "peer"), ("gbdt", 4, "peer"), ("gbdt", 2, "peer_owner"),
                                             ("gbdt", 3, "peer_owner"), ("gbdt", 4, "peer_owner"),
                                             ("gbdt_loss", 2, "peer_owner"), ("gbdt_loss", 3, "peer_owner"),
                                             ("gbdt", 2, "peer_overlap"), ("gbdt", 3, "peer_overlap"),
                                             ("gbdt", 2, "peer_auto")])
def test_gpu_builders_multi_rank_one_gpu(tmp_path, task, world, mode):
    """Several ranks share the one GPU over gloo: the GPU level engine (fused count slots,
    overlapped half-level all-reduce, global gradient bound; or owner-computes:
    reduce-scatter by feature block + device split-record argmax) and the leaf-wise
    speculative builder (scattered slot all-reduce / reduce-scatter) must give the world-1
    model byte for byte. "peer": every level / batch message and the round vector go through
    the one-kernel IPC peer-memory exchange (leaf-wise: sized on the device, no host wait per
    batch); level-wise rounds are then graph-captured even over gloo, so the replays check
    that the device-resident exchange epochs stay in step across graph replays. "peer_owner":
    owner-computes with the level's reduce-scatter and the split-record all-gather as one
    peer kernel each (leaf-wise: the batch's reduce-scatter sized on the device)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    peer = mode.startswith("peer")
    sync = {"peer": "allreduce", "peer_owner": "owner", "peer_overlap": "allreduce",
            "peer_auto": "allreduce"}.get(mode, mode)
    env = {"YTK_DIST_BACKEND": "gloo", "YTK_HIST_SYNC": sync,
           "YTK_TEST_FSAMPLE": "0.7" if world == 3 else "1.0", "YTK_PEER_REDUCE": "1" if peer else "0",
           "YTK_COMM_LOG": "1", "YTK_HIST_OVERLAP_MIN_ROWS": "0",  # small shards: keep the overlap covered
           "YTK_PEER_OVERLAP": {"peer_overlap": "1", "peer_auto": "auto_force"}.get(mode, "0"),
           # the first levels / batches reserve partition chunks by count + scan at these small
           # shards too (splits with no local rows give empty chunk ranges)
           "YTK_PART_SCAN_MIN_ROWS": os.environ.get("YTK_TEST_PART_SCAN_MIN_ROWS", "0")}
    _run(task, tmp_path / "w1", 1, "cuda", extra_env=env)
    res = _run(task, tmp_path / f"w{world}", world, "cuda", extra_env=env)
    if peer:
        assert res["peer_calls"] > 0
        assert res["owner"] == (mode == "peer_owner")
        if mode == "peer_auto":  # trees 1-4 timed off / on, the faster mode kept (either is fine)
            off_us, on_us = res["overlap_times"]
            assert off_us > 0 and on_us > 0 and res["peer_overlap"] == (on_us < off_us)
        else:
            assert res["peer_overlap"] == (mode == "peer_overlap")
        if task == "gbdt" and world != 3:  # no feature sampling: graph-eligible rounds
            assert res["graph_replays"] > 0
    assert open(tmp_path / "w1" / "model.txt").read() == open(tmp_path / f"w{world}" / "model.txt").read()
    _same_collective_sequence(tmp_path / f"w{world}", world)


@pytest.mark.gpu
def test_leafwise_rccl_loop_fixed_messages(tmp_path):
    """The leaf-wise batch loop over the process group (YTK_PEER_REDUCE=0, two ranks on the one
    GPU over gloo): every batch message has the size of the host's cap schedule
    min(2^batch, YTK_LW_RCCL_KCAP) x (slot + cursors) -- the host never reads a batch's split
    count from the device to size its collective (round 4 waited on each batch's planner for
    it) -- and the model is the world-1 model byte for byte, the capped batches included."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_DIST_BACKEND": "gloo", "YTK_HIST_SYNC": "allreduce", "YTK_PEER_REDUCE": "0", "YTK_COMM_LOG": "1",
           "YTK_LW_RCCL_KCAP": "4"}
    _run("gbdt_loss", tmp_path / "w1", 1, "cuda", extra_env=env)
    res = _run("gbdt_loss", tmp_path / "w2", 2, "cuda", extra_env=env)
    assert open(tmp_path / "w1" / "model.txt").read() == open(tmp_path / "w2" / "model.txt").read()
    S, cap = res["slot_elems"], res["rccl_kcap"]
    assert S > 0 and cap == 4
    sched = [min(cap, 1 << i) * (S + 16) for i in range(64)]  # CUR_STRIDE 16 words per split
    log = json.load(open(tmp_path / "w2" / "comm_log_0.json"))
    sizes = [n for op, dt, n in log if op == "allreduce_sum" and dt == "torch.int64" and n >= S]
    roots = [i for i, n in enumerate(sizes) if n == S]  # each tree's root slot message
    assert len(roots) >= 6
    for a, b in zip(roots, roots[1:] + [len(sizes)]):
        batch = sizes[a + 1:b]
        assert batch and batch == sched[:len(batch)], batch[:8]
    _same_collective_sequence(tmp_path / "w2", 2)


@pytest.mark.parametrize("task,mode", [("gbdt", "allreduce"), ("gbdt_loss", "owner")])
def test_forced_dist_world1_gloo(tmp_path, task, mode):
    """YTK_FORCE_DIST=1 at world 1 takes every multi-rank code path (collectives issued to a
    one-rank group) and must give the plain world-1 model byte for byte."""
    env = {"YTK_HIST_SYNC": mode}
    _run(task, tmp_path / "plain", 1, extra_env=env)
    res = _run(task, tmp_path / "forced", 1, extra_env=dict(env, YTK_FORCE_DIST="1"))
    assert res["is_dist"] and res["backend"] == "gloo" and res["comm"]["calls"] > 0
    assert res["owner"] == (mode == "owner")
    assert open(tmp_path / "plain" / "model.txt").read() == open(tmp_path / "forced" / "model.txt").read()


@pytest.mark.gpu
@pytest.mark.parametrize("task,mode", [("gbdt", "allreduce"), ("gbdt", "owner"), ("gbdt_loss", "allreduce"),
                                       ("gbdt_loss", "owner")])
def test_rccl_world1_forced_dist(tmp_path, task, mode):
    """The real nccl (= RCCL) backend on the one GPU of the test box: a world-1 process group
    with YTK_FORCE_DIST=1 runs the multi-GPU engines' RCCL calls (init with device_id, async
    all-reduce work handles waited on the compute stream, reduce-scatter + all-gather of the
    owner mode, the gloo side group for host scalars) -- RCCL refuses two ranks on one GPU,
    so this is the RCCL-semantics check available here; the model must equal the plain
    world-1 run byte for byte. Level-wise rounds replay as graphs that contain the RCCL calls
    (one capture, then graph replays; YTK_GRAPH_DIST=0 variant: eager rounds)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_HIST_SYNC": mode, "YTK_COMM_LOG": "1", "YTK_HIST_OVERLAP_MIN_ROWS": "0", "YTK_PEER_REDUCE": "0"}
    if task == "gbdt" and mode == "allreduce":
        eager = _run(task, tmp_path / "eager", 1, "cuda", extra_env=dict(env, YTK_FORCE_DIST="1", YTK_GRAPH_DIST="0"))
        assert eager["graph_replays"] == 0
    _run(task, tmp_path / "plain", 1, "cuda", extra_env=env)
    res = _run(task, tmp_path / "rccl", 1, "cuda", extra_env=dict(env, YTK_FORCE_DIST="1"))
    assert res["is_dist"] and res["backend"] == "nccl" and res["comm"]["calls"] > 0
    assert res["owner"] == (mode == "owner")
    if task == "gbdt":  # level-wise rounds are captured WITH their RCCL calls and replayed as graphs
        assert res["graph_replays"] > 0 and res["comm"]["calls"] >= 5 * 6
    assert open(tmp_path / "plain" / "model.txt").read() == open(tmp_path / "rccl" / "model.txt").read()
    if task == "gbdt" and mode == "allreduce":
        assert open(tmp_path / "eager" / "model.txt").read() == open(tmp_path / "rccl" / "model.txt").read()


@pytest.mark.gpu
def test_capture_after_eager_rccl_drains_watchdog(tmp_path):
    """Forced interleaving of the round-5 abort: eager RCCL all-reduces, then a GLOBAL-mode
    capture held open ~0.8 s (8 watchdog polls) that also records captured all-reduces. Without
    a drain this aborts the process from the watchdog's event query (tools/
    probe_capture_watchdog.py global_nodrain, profiles/r6/watchdog_probe/); with
    Comm.drain_pending -- what GBDTTrainer._graph_round calls before capturing -- the watchdog
    holds no eager work during the capture and the process runs clean."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_capture_watchdog.py"), str(tmp_path),
                        "global_comm"], capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    log = open(tmp_path / "global_comm.log").read() if (tmp_path / "global_comm.log").exists() else ""
    assert r.returncode == 0, r.stdout + _head_tail(log)
    assert "PROBE_OK" in log and "Comm.drain_pending" in log


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["1", "2"])
def test_rccl_world1_capture_failure_falls_back(tmp_path, where):
    """A round capture that fails (injected after the capture, "1", or inside it with the
    round's kernels and RCCL calls half captured, "2") is voted down and the job continues
    with eager rounds -- same model, no graph replays, the captured collectives not counted."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_HIST_SYNC": "allreduce", "YTK_HIST_OVERLAP_MIN_ROWS": "0", "YTK_PEER_REDUCE": "0"}
    _run("gbdt", tmp_path / "plain", 1, "cuda", extra_env=env)
    good = _run("gbdt", tmp_path / "graph", 1, "cuda", extra_env=dict(env, YTK_FORCE_DIST="1"))
    bad = _run("gbdt", tmp_path / "fail", 1, "cuda", extra_env=dict(env, YTK_FORCE_DIST="1", YTK_FAULT_CAPTURE=where))
    assert good["graph_replays"] > 0 and bad["graph_replays"] == 0
    assert bad["comm"]["calls"] == good["comm"]["calls"]  # eager rounds issue what replays count
    assert open(tmp_path / "plain" / "model.txt").read() == open(tmp_path / "fail" / "model.txt").read()


@pytest.mark.gpu
@pytest.mark.parametrize("task", ["gbdt", "gbdt_loss"])
def test_peer_world1_forced_dist(tmp_path, task):
    """YTK_FORCE_DIST=1 on the nccl backend with the default (single-node) peer path: every
    level / batch message and the round vector is one peer exchange kernel, level-wise rounds
    replay as graphs, and the model equals the plain world-1 run byte for byte. Level-wise:
    one exchange per built level plus the round vector, no RCCL call per round."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_HIST_SYNC": "allreduce", "YTK_COMM_LOG": "1"}
    _run(task, tmp_path / "plain", 1, "cuda", extra_env=env)
    res = _run(task, tmp_path / "peer", 1, "cuda", extra_env=dict(env, YTK_FORCE_DIST="1"))
    assert res["is_dist"] and res["backend"] == "nccl" and res["peer_calls"] > 0
    if task == "gbdt":
        assert res["graph_replays"] > 0
        # the captured round: its level messages + round vector are peer exchanges only
        log = json.load(open(tmp_path / "peer" / "comm_log_0.json"))
        assert sum(1 for op, _, _ in log if op == "peer_allreduce") >= 5
    assert open(tmp_path / "plain" / "model.txt").read() == open(tmp_path / "peer" / "model.txt").read()


@pytest.mark.gpu
@pytest.mark.parametrize("task,two_shot", [("linear", "0"), ("fm", "1"), ("gbmlr", "0"), ("ffm", "1")])
def test_lbfgs_peer_gradient_allreduce_one_gpu(tmp_path, task, two_shot):
    """Two ranks on the one GPU: the L-BFGS gradient all-reduce over the peer-memory exchange
    (fp32, rank-order sums; two_shot "0": every message two-shot reduce-scatter + all-gather,
    "1": the default size split) reaches the gloo run's losses to 1e-6. The sharded (s, y)
    history's dot partials and the p all-gather ride the peer exchange too."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_DIST_BACKEND": "gloo"}
    ref = _run(task, tmp_path / "gloo", 2, "cuda", extra_env=dict(env, YTK_PEER_REDUCE="0"))
    peer_env = dict(env, YTK_PEER_REDUCE="1")
    if two_shot == "0":
        peer_env["YTK_PEER_TWO_SHOT_BYTES"] = "0"
    got = _run(task, tmp_path / "peer", 2, "cuda", extra_env=peer_env)
    np.testing.assert_allclose(got["loss"], ref["loss"], rtol=1e-6)
    np.testing.assert_allclose(got["test_loss"], ref["test_loss"], rtol=1e-6)


@pytest.mark.gpu
def test_lbfgs_peer_dropped_exchange_raises(tmp_path):
    """Rank 1 silently drops one L-BFGS gradient exchange (fault mode ``skip``): rank 0's flag
    wait times out and the error word must surface as an exception -- not as training on
    stale peer sums -- so the job exits non-zero naming the timed-out wait."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", YTK_DIST_BACKEND="gloo",
               YTK_PEER_REDUCE="1", YTK_PEER_TIMEOUT_S="5", YTK_COMM_TIMEOUT="30",
               YTK_FAULT_INJECT="peer:1:4:skip")
    os.makedirs(tmp_path, exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), WORKER, "linear", str(tmp_path), "cuda"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "injected fault at peer step 4 (skip)" in r.stderr, r.stderr[-3000:]
    assert "flag wait timed out" in r.stderr, r.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_peer_primitives_one_gpu(tmp_path, world):
    """Ranks sharing the one GPU: the peer exchange's all-reduce (one-shot and two-shot
    sizes), reduce-scatter and all-gather equal their definitions exactly for int64, fp64
    and fp32 (values exactly representable, so rank-order float sums are exact too)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run("peer_ops", tmp_path, world, "cuda", extra_env={"YTK_DIST_BACKEND": "gloo", "YTK_PEER_REDUCE": "1"})
    res = json.load(open(tmp_path / "res.json"))
    assert res["peer"] and len(res["ok"]) == 9
    for dt, n, ok_ar, ok_rs, ok_ag in res["ok"]:
        assert ok_ar and ok_rs and ok_ag, (dt, n, ok_ar, ok_rs, ok_ag)


@pytest.mark.parametrize("task", ["linear_sgd", "fm_sgd", "ffm_sgd"])
def test_sgd_world2_model_averaging(tmp_path, task):
    """SGD on 2 ranks (shards differ in size: uneven step counts must still meet at every
    averaging point) learns like the single-rank run."""
    r1 = _run(task, tmp_path / "w1", 1)
    r2 = _run(task, tmp_path / "w2", 2)
    assert r2["test_loss"] < 0.6 and r1["test_loss"] < 0.6
    assert abs(r2["test_loss"] - r1["test_loss"]) < 0.1


@pytest.mark.parametrize("mode", ["allreduce", "owner"])
def test_bench_under_torchrun_world2(tmp_path, mode):
    """bench.py as the driver launches it for N > 1 (torch.distributed.run, one JSON line from
    rank 0, max-over-ranks time, per-tree collective accounting)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", YTK_HIST_SYNC=mode)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--device", "cpu", "--train-rows", "8000", "--test-rows", "1000",
           "--depth", "3", "--quiet"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2" and res["steps"] == 2
    assert res["collectives_per_tree"] > 0 and res["collective_bytes_per_tree"] > 0
    assert res["hist_sync"] == mode and res["trees_converted"] == 3
    # multi-GPU diagnostics carried by every multi-rank line (CPU: no peer-memory path)
    assert res["peer_selftest"].startswith("off") and res["overlap"] is False
    assert res["exchanges_per_tree"] == res["collectives_per_tree"] and res["exchange_us_per_tree"] is None


def _bench(world, extra_args=(), env_extra=None, timeout=600):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **(env_extra or {}))
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "3", "--warmup", "1", "--device", "cpu",
            "--train-rows", "12000", "--test-rows", "3000", "--depth", "4", "--quiet", "--leafwise-steps", "0",
            *extra_args]
    if world == 1:
        cmd = [sys.executable] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


def _bench_json(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 4])
def test_bench_global_rows_match_world1(world):
    """Every rank generates the same global data and keeps its contiguous row slice, so the
    world-N bench trains on the world-1 rows: losses agree to 1e-3 and AUCs to 3e-3 (the
    quantile sketches merged over ranks may move a bin candidate; 12k rows), and the JSON
    line names the sync mode."""
    r1 = _bench_json(_bench(1))
    rn = _bench_json(_bench(world))
    assert r1["hist_sync"] == "none" and r1["hist_transport"] == "none"
    assert rn["hist_sync"] in ("allreduce", "owner") and rn["hist_transport"] == "gloo"
    assert rn["quality_on"].startswith("global")
    for k in ("train_loss", "test_loss"):
        assert abs(rn[k] - r1[k]) < 1e-3, (k, r1[k], rn[k])
    for k in ("train_auc", "test_auc"):
        assert abs(rn[k] - r1[k]) < 3e-3, (k, r1[k], rn[k])


def test_bench_stalled_rank_fails_fast():
    """A rank that stops issuing (injected stall at timed round 2) makes the world-2 bench
    exit non-zero within the collective timeout, naming the last collective."""
    import time
    t0 = time.time()
    r = _bench(2, env_extra={"YTK_FAULT_INJECT": "bench:1:2:stall", "YTK_COMM_TIMEOUT": "15"}, timeout=300)
    assert r.returncode != 0
    assert time.time() - t0 < 200
    assert "failed" in r.stderr and "last collective issued" in r.stderr, r.stderr[-2000:]


VARIANT_KEYS = {"s_per_tree", "env", "transport", "hist_sync", "overlap", "graph_replays", "collectives_per_tree",
                "exchanges_per_tree", "exchange_us_per_tree", "exchange_us_per_level", "wall_s"}


def test_bench_variants_world2_failing_variant_keeps_headline():
    """bench.py at N > 1 runs the multi-GPU design A/B after the headline (overlap, the other
    sync mode, RCCL, RCCL + overlap): every variant reports its keys, and a variant that fails
    (injected into the last one) is reported as an error without losing the headline line."""
    r = _bench(2, extra_args=("--variant-steps", "2"), env_extra={"YTK_BENCH_FAIL_VARIANT": "rccl_overlap"})
    res = _bench_json(r)
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["hist_sync"] in ("allreduce", "owner")
    v = res["variants"]
    assert list(v) == ["overlap_on", "overlap_off", "sync_alt", "rccl", "rccl_overlap"]
    for name in ("overlap_on", "overlap_off", "sync_alt", "rccl"):
        assert VARIANT_KEYS <= set(v[name]), (name, v[name])
        assert v[name]["s_per_tree"] > 0 and v[name]["collectives_per_tree"] > 0
    assert v["sync_alt"]["hist_sync"] != res["hist_sync"]
    assert v["rccl_overlap"]["error"].startswith("RuntimeError: injected failure")
    assert "exchange_us_per_level" in res


def test_bench_variant_budget_skips():
    """Past --variant-budget seconds the remaining variants are skipped (every rank agrees)."""
    res = _bench_json(_bench(2, extra_args=("--variant-budget", "0", "--variants", "overlap_on,rccl")))
    assert all("skipped" in v for v in res["variants"].values()) and len(res["variants"]) == 2


def test_bench_world1_has_no_variants():
    res = _bench_json(_bench(1))
    assert "variants" not in res


@pytest.mark.gpu
def test_bench_variants_two_ranks_one_gpu():
    """Two ranks share the one GPU (gloo process group, forced peer-memory path): the bench
    line carries every variant's keys with the peer transport device-timed."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"YTK_DIST_BACKEND": "gloo", "YTK_PEER_REDUCE": "1", "YTK_PEER_TIMEOUT_S": "60"}
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--train-rows", "200000",
            "--test-rows", "20000", "--quiet", "--leafwise-steps", "0", "--variant-steps", "2",
            "--variants", "overlap_on,overlap_off,sync_alt"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port())] + args
    r = subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **env),
                       capture_output=True, text=True, timeout=300)
    res = _bench_json(r)
    assert res["hist_transport"] == "peer" and res["exchange_us_per_level"] is not None
    for name in ("overlap_on", "overlap_off", "sync_alt"):
        assert VARIANT_KEYS <= set(res["variants"][name]), res["variants"][name]
        assert res["variants"][name]["transport"] == "peer"
    assert res["variants"]["overlap_on"]["overlap"] is True and res["variants"]["overlap_off"]["overlap"] is False
