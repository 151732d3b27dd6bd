"""Graph-replayed boosting rounds (level engine, one GPU): the captured round must build the
same trees and losses as the eager launch sequence, for an odd and an even number of
replays, and an eager round after graph mode must continue from the right ping-pong buffers."""
import pytest
import torch

from ytk_learn_amd.data.synthetic import higgs_like
from ytk_learn_amd.models.gbdt.builder import TreeParams
from ytk_learn_amd.models.gbdt.trainer import GBDTData, GBDTParams, GBDTTrainer

pytestmark = pytest.mark.gpu


def _trainer(dev, rounds, depth=6):
    X, y = higgs_like(60000, seed=3, device=dev)
    Xt, yt = higgs_like(6000, seed=4, device=dev)
    tp = TreeParams(max_depth=depth, max_leaf_cnt=1 << depth, min_child_hessian_sum=1.0, learning_rate=0.1,
                    grow_policy="level")
    p = GBDTParams(round_num=rounds, loss_function="sigmoid", missing_value="value@0",
                   approximate=[{"cols": "default", "type": "sample_by_quantile", "max_cnt": 255, "alpha": 0.5}],
                   tree=tp)
    tr = GBDTTrainer(p, GBDTData(X, y), GBDTData(Xt, yt))
    tr.prepare()
    tr.init_gradients()
    return tr


def _model_text(tr):
    return "\n".join(t.dump(i) if hasattr(t, "dump") else repr(t.__dict__) for i, t in enumerate(tr.model.trees))


@pytest.mark.parametrize("rounds,depth", [(6, 6), (7, 6), (5, 5)])
def test_graph_rounds_match_eager(cuda, monkeypatch, rounds, depth):
    monkeypatch.setenv("YTK_GRAPH", "0")
    ref = _trainer(cuda, rounds, depth)
    for i in range(rounds):
        ref.run_round(i)
    ref.materialize()
    monkeypatch.setenv("YTK_GRAPH", "1")
    tr = _trainer(cuda, rounds, depth)
    for i in range(rounds):
        tr.run_round(i)
    tr.materialize()
    assert isinstance(tr._graphs, dict) and tr._graphs["n"] == rounds - 1  # round 0 eager, then replays
    assert _model_text(tr) == _model_text(ref)
    for i in range(rounds):
        assert tr.round_losses[i] == ref.round_losses[i]
    assert torch.equal(tr.score, ref.score) and torch.equal(tr.te_score, ref.te_score)


def test_eager_round_after_odd_replays(cuda, monkeypatch):
    """3 graph rounds (odd replays: 2 after the eager first), then eager rounds: the engine's
    buffer parity must follow the device."""
    rounds = 7
    monkeypatch.setenv("YTK_GRAPH", "0")
    ref = _trainer(cuda, rounds)
    for i in range(rounds):
        ref.run_round(i)
    ref.materialize()
    monkeypatch.setenv("YTK_GRAPH", "1")
    tr = _trainer(cuda, rounds)
    for i in range(4):  # round 0 eager, rounds 1-3 replayed (3 replays: odd)
        tr.run_round(i)
    assert tr._graphs["n"] == 3
    monkeypatch.setenv("YTK_GRAPH", "0")
    for i in range(4, rounds):
        tr.run_round(i)
    tr.materialize()
    assert tr._graphs is False
    assert _model_text(tr) == _model_text(ref)
    assert torch.equal(tr.score, ref.score)
