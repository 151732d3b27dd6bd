"""Failure detection + resume: a worker killed mid-training (test-only fault injection,
``YTK_FAULT_INJECT``) leaves the last complete dump behind; ``continue_train`` (by hand or
through ``bin/local_optimizer.sh MAX_RESTARTS``) finishes the job from it.

Reference behaviour being exercised: models are the checkpoints (GBDT dump every
``dump_freq`` rounds, L-BFGS every ``dump_freq`` iterations, soft trees per finished tree;
SURVEY.md §5 "Checkpoint / resume"), and a failing rank takes the whole job down.
"""
import os
import subprocess
import sys

import pytest

from test_models_e2e import write_binary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONF = os.path.join(ROOT, "config", "model")


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, YTK_QUIET="0")
    env.pop("YTK_FAULT_INJECT", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-m", "ytk_learn_amd.cli.train"] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("fault")
    write_binary(str(d / "train.txt"), 1500, seed=1)
    write_binary(str(d / "test.txt"), 300, seed=2)
    return d


def _final_loss(stdout):
    vals = [float(l.split("=")[1]) for l in stdout.splitlines() if l.startswith("train loss = ")]
    return vals[-1]


def test_gbdt_fault_then_resume_matches_uninterrupted(data, tmp_path):
    base = ["gbdt", os.path.join(CONF, "gbdt.conf"), "--device", "cpu",
            "--set", f"data.train.data_path={data / 'train.txt'}", "--set", f"data.test.data_path={data / 'test.txt'}",
            "--set", "data.max_feature_dim=40", "--set", "optimization.round_num=6",
            "--set", "optimization.max_depth=3", "--set", "model.dump_freq=1"]
    full = _run(base + ["--set", f"model.data_path={tmp_path / 'full.model'}"])
    assert full.returncode == 0, full.stderr[-2000:]
    m = str(tmp_path / "m.model")
    crashed = _run(base + ["--set", f"model.data_path={m}"], {"YTK_FAULT_INJECT": "gbdt:0:3"})
    assert crashed.returncode == 75, crashed.stderr[-2000:]
    text = open(m).read()
    assert "tree_num=3\n" in text  # the dump after round 3 is complete; round 4 never ran
    assert not [f for f in os.listdir(tmp_path) if f.startswith(".m.model.tmp")]
    resumed = _run(base + ["--set", f"model.data_path={m}", "--set", "model.continue_train=true"])
    assert resumed.returncode == 0, resumed.stderr[-2000:]
    assert "old model round_num=3" in resumed.stdout
    assert "tree_num=6\n" in open(m).read()
    # the resumed run re-scores the dumped trees (text thresholds / leaf values) -> same path
    assert abs(_final_loss(resumed.stdout) - _final_loss(full.stdout)) < 1e-5


def test_lbfgs_fault_then_resume(data, tmp_path):
    m = str(tmp_path / "lr.model")
    base = ["linear", os.path.join(CONF, "linear.conf"), "--device", "cpu",
            "--set", f"data.train.data_path={data / 'train.txt'}", "--set", f"data.test.data_path={data / 'test.txt'}",
            "--set", f"model.data_path={m}", "--set", "model.dump_freq=1",
            "--set", "optimization.line_search.lbfgs.convergence.max_iter=12"]
    crashed = _run(base, {"YTK_FAULT_INJECT": "lbfgs:0:4"})
    assert crashed.returncode == 75
    assert os.path.exists(os.path.join(m, "model-00000"))
    loss_at_crash = _final_loss(crashed.stdout)
    resumed = _run(base + ["--set", "model.continue_train=true"])
    assert resumed.returncode == 0, resumed.stderr[-2000:]
    first = [float(l.split("=")[1]) for l in resumed.stdout.splitlines() if l.startswith("train loss = ")][0]
    assert first <= loss_at_crash + 1e-9  # restarts from the dumped weights, not from zero
    assert _final_loss(resumed.stdout) <= first


def test_gbst_fault_then_resume(data, tmp_path):
    m = str(tmp_path / "gbmlr.model")
    base = ["gbmlr", os.path.join(CONF, "gbmlr.conf"), "--device", "cpu",
            "--set", f"data.train.data_path={data / 'train.txt'}", "--set", f"data.test.data_path={data / 'test.txt'}",
            "--set", f"model.data_path={m}", "--set", "k=4", "--set", "tree_num=3",
            "--set", "optimization.line_search.lbfgs.convergence.max_iter=5"]
    crashed = _run(base, {"YTK_FAULT_INJECT": "gbst:0:1"})
    assert crashed.returncode == 75
    assert "finished_tree_num:1\n" in open(os.path.join(m, "tree-info")).read()
    resumed = _run(base + ["--set", "model.continue_train=true"])
    assert resumed.returncode == 0, resumed.stderr[-2000:]
    assert "finished tree num:1" in resumed.stdout


def test_raise_mode_takes_error_path(data, tmp_path):
    r = _run(["linear", os.path.join(CONF, "linear.conf"), "--device", "cpu",
              "--set", f"data.train.data_path={data / 'train.txt'}", "--set", f"model.data_path={tmp_path / 'x'}"],
             {"YTK_FAULT_INJECT": "lbfgs:0:1:raise"})
    assert r.returncode != 0 and "injected fault" in r.stderr


def test_launcher_restart_resumes_two_ranks(data, tmp_path):
    """2 gloo ranks under torchrun: rank 1 dies at round 2, torchrun tears the group down,
    bin/local_optimizer.sh relaunches with continue_train and the job completes."""
    m = str(tmp_path / "g.model")
    env = dict(os.environ, MAX_RESTARTS="1", MASTER_PORT="29641", YTK_FAULT_INJECT="gbdt:1:2",
               YTK_FAULT_ONCE=str(tmp_path / "fault.once"), PYTHONPATH=ROOT, YTK_COMM_TIMEOUT="120")
    cmd = ["bash", "bin/local_optimizer.sh", "gbdt", os.path.join(CONF, "gbdt.conf"), "2", "", "--",
           "--device", "cpu", "--set", f"data.train.data_path={data / 'train.txt'}",
           "--set", "data.max_feature_dim=40", "--set", "optimization.round_num=4",
           "--set", "optimization.max_depth=3", "--set", f"model.data_path={m}", "--set", "model.dump_freq=1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "restart 1/1 with model.continue_train=true" in r.stdout
    assert "tree_num=4\n" in open(m).read()


def test_profile_and_metrics_jsonl(data, tmp_path):
    import json
    js = tmp_path / "m.jsonl"
    r = _run(["gbdt", os.path.join(CONF, "gbdt.conf"), "--device", "cpu", "--profile", "--metrics-jsonl", str(js),
              "--set", f"data.train.data_path={data / 'train.txt'}", "--set", f"data.test.data_path={data / 'test.txt'}",
              "--set", "data.max_feature_dim=40", "--set", "optimization.round_num=2",
              "--set", f"model.data_path={tmp_path / 'p.model'}"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[GBDT] time stats tree 2:" in r.stdout
    rows = [json.loads(l) for l in open(js)]
    assert [x["round"] for x in rows] == [1, 2] and rows[0]["test_loss"] is not None
    assert rows[1]["time_stats"]["build_tree"] > 0
