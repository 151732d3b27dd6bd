"""RCCL probe: can several ranks share one GPU under the nccl (= RCCL) backend?

Run under torch.distributed.run on a 1-GPU box:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py
Each rank all-reduces a device tensor (sync and async work handle) and prints the result.
"""
import datetime
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev,
                        timeout=datetime.timedelta(seconds=60))
t = torch.full((1 << 20,), float(rank + 1), device=dev)
dist.all_reduce(t)
w = dist.all_reduce(t, async_op=True)
w.wait()
torch.cuda.synchronize()
expect = 2.0 * world * (world + 1) / 2
print(f"rank {rank}: sum {float(t[0])} expect {expect} ok={float(t[0]) == expect}", flush=True)
dist.barrier()
dist.destroy_process_group()
