"""RCCL-facing semantics of the communicator, checked without a multi-GPU box.

* ``Comm.from_env`` must bind the rank to its GPU before the process group exists and hand
  that device to ``init_process_group(device_id=...)`` for the nccl (= RCCL) backend, with
  a separate gloo group for host tensors / objects.
* An ``async_op=True`` all-reduce returns a work handle: the result is only defined after
  ``wait()``, which the level engine's overlapped half-level all-reduce relies on
  (``device_builder.py``: first half async, second half built, ``work.wait()``, second
  half all-reduced). Exercised for real over gloo, world 2.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ytk_learn_amd.parallel import comm as comm_mod
from ytk_learn_amd.parallel.comm import Comm


def test_from_env_nccl_binds_device_and_passes_device_id(monkeypatch):
    calls = {}
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    monkeypatch.setenv("LOCAL_RANK", "2")
    monkeypatch.delenv("YTK_DIST_BACKEND", raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "set_device", lambda i: calls.setdefault("set_device", i))
    monkeypatch.setattr(dist, "is_initialized", lambda: False)

    def fake_init(backend, rank, world_size, timeout, **kw):
        calls["init"] = dict(backend=backend, rank=rank, world_size=world_size, **kw)
        # the device must already be bound when the group is created
        assert "set_device" in calls

    monkeypatch.setattr(dist, "init_process_group", fake_init)
    monkeypatch.setattr(dist, "new_group", lambda backend: calls.setdefault("new_group", backend) or "cpu_group")
    monkeypatch.setattr(dist, "get_rank", lambda: 2)
    monkeypatch.setattr(dist, "get_world_size", lambda: 4)
    c = Comm.from_env(device="cuda")
    assert calls["set_device"] == 2
    assert calls["init"]["backend"] == "nccl"
    assert calls["init"]["device_id"] == torch.device("cuda", 2)
    assert calls["init"]["rank"] == 2 and calls["init"]["world_size"] == 4
    assert calls["new_group"] == "gloo"  # host tensors / objects never go through RCCL
    assert c.device == torch.device("cuda", 2) and c.world == 4 and c.rank == 2


def test_from_env_gloo_override_has_no_device_id(monkeypatch):
    """YTK_DIST_BACKEND=gloo (several ranks on one GPU): no device_id, one group."""
    calls = {}
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("YTK_DIST_BACKEND", "gloo")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(torch.cuda, "set_device", lambda i: calls.setdefault("set_device", i))
    monkeypatch.setattr(dist, "is_initialized", lambda: False)
    monkeypatch.setattr(dist, "init_process_group",
                        lambda backend, rank, world_size, timeout, **kw: calls.setdefault("init", (backend, kw)))
    monkeypatch.setattr(dist, "new_group", lambda backend: pytest.fail("no second group for gloo"))
    monkeypatch.setattr(dist, "get_rank", lambda: 1)
    monkeypatch.setattr(dist, "get_world_size", lambda: 2)
    c = Comm.from_env(device="cuda")
    assert calls["set_device"] == 0  # both ranks on the one GPU
    assert calls["init"] == ("gloo", {})
    assert c.cpu_group is c.group


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _async_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    c = Comm.from_env(device="cpu")
    try:
        a = torch.full((1000,), float(rank + 1), dtype=torch.float64)
        b = torch.full((10,), float(10 * (rank + 1)), dtype=torch.float64)
        work = c.allreduce_(a, async_op=True)
        assert work is not None  # a handle, not an eager no-op
        c.allreduce_(b)  # a second collective may be issued while the first is in flight
        work.wait()
        q.put((rank, float(a[0]), float(a[-1]), float(b[0]), dict(c.stats)))
    finally:
        c.close()


def test_async_allreduce_work_handle_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, a0, a1, b0, stats in out:
        assert a0 == a1 == 3.0 and b0 == 30.0
        assert stats["calls"] == 2 and stats["bytes"] == (1000 + 10) * 8


def test_local_comm_collectives_are_noops():
    c = Comm.local()
    t = torch.arange(4.0)
    assert c.allreduce_(t, async_op=True) is None
    assert torch.equal(t, torch.arange(4.0)) and c.stats["calls"] == 0
    assert comm_mod.Comm.local().feature_blocks(10) == (10, [(0, 10)])
