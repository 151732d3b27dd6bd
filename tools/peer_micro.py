"""Peer-exchange micro-benchmark: time per exchange kernel (HIP events, back-to-back) for a
few message sizes. World 1 (forced dist over gloo) by default; several ranks on one GPU:
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/peer_micro.py
Env: YTK_PEER_SYS_FENCE, YTK_PEER_BLOCK_ELEMS (variants of csrc/hip/gbdt_comm.hip)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("YTK_FORCE_DIST", "1")
os.environ.setdefault("YTK_DIST_BACKEND", "gloo")
os.environ["YTK_PEER_REDUCE"] = "1"
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

from ytk_learn_amd.parallel import peer  # noqa: E402
from ytk_learn_amd.parallel.comm import Comm  # noqa: E402


def main():
    comm = Comm.from_env("cuda")
    pr = peer.make(comm, 1 << 21)
    assert pr is not None
    out = {"world": comm.world, "sys_fence": os.environ.get("YTK_PEER_SYS_FENCE", "1"),
           "block_elems": os.environ.get("YTK_PEER_BLOCK_ELEMS", "2048")}
    for n in (64, 57344, 262144, 1 << 20):
        t = torch.full((n,), comm.rank + 1, dtype=torch.int64, device=comm.device)
        for _ in range(20):
            pr.allreduce_(t)
        torch.cuda.synchronize()
        comm.barrier()
        reps = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            pr.allreduce_(t)
        e1.record()
        torch.cuda.synchronize()
        out[f"us_n{n}"] = round(e0.elapsed_time(e1) / reps * 1000.0, 2)
        # correctness: one exchange of known data
        t.fill_(comm.rank + 1)
        pr.allreduce_(t)
        torch.cuda.synchronize()
        assert int(t[0]) == comm.world * (comm.world + 1) // 2 and int(t[-1]) == int(t[0]), int(t[0])
    pr.check()
    pr.close()
    if comm.rank == 0:
        print(json.dumps(out), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
