#!/usr/bin/env python3
"""Forced-interleaving probe: ProcessGroupNCCL watchdog vs. a HIP graph capture.

Round-5 finding: test_rccl_world1_forced_dist[gbdt-allreduce] aborted once with SIGABRT raised
from ProcessGroupNCCL::Watchdog::run (gpurun_out/dist_final.log:53-63). The trainer captures
its level-wise rounds right after eager rounds that issued RCCL all-reduces; the watchdog
thread polls its list of eager work handles every ~100 ms and queries their end events
(hipEventQuery). Whether that query lands inside the capture is a timing accident -- which is
what an intermittent abort looks like.

This probe forces the interleaving: an eager all-reduce, then a capture that stays open for
~0.8 s (8 watchdog polls) while it records kernels and captured all-reduces. Each variant runs
in its own child process (a watchdog abort kills the process) and its FULL stderr is kept.

  variants: <capture mode>_<drain>
    capture mode: global | thread_local | relaxed
    drain: nodrain (capture right after torch.cuda.synchronize), drain (also wait until the
           process group's watchdog has retired every eager work: ProcessGroup._wait_for_pending_works),
           comm (the package's Comm.drain_pending, which the GBDT trainer calls before its captures)

Measured on MI355X (profiles/r6/watchdog_probe/): global_nodrain aborts with the round-5
signature -- "Process group watchdog thread terminated with exception: HIP error: operation not
permitted when stream is capturing", raised from the event query (HIPEvent.h:109) and rethrown
at ProcessGroupNCCL.cpp:2099 -- while global_drain, thread_local_nodrain and thread_local_drain
run clean.

Usage: python tools/probe_capture_watchdog.py [outdir] [variant ...]
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

# safe-expected variants first: a child that aborts ends the probe (no further GPU step after an abort)
VARIANTS = ["thread_local_drain", "global_drain", "thread_local_nodrain"]


def child(variant: str) -> None:
    import torch
    import torch.distributed as dist
    mode, drain = variant.rsplit("_", 1)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    pg = dist.group.WORLD
    x = torch.ones(1 << 20, device=dev)
    for _ in range(4):  # eager collectives: work handles the watchdog tracks
        dist.all_reduce(x, async_op=True).wait()
    torch.cuda.synchronize(dev)
    if drain == "comm":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from ytk_learn_amd.parallel.comm import Comm
        c = Comm(0, 1, dev, pg, pg)
        assert c.is_dist
        t0 = time.perf_counter()
        c.drain_pending()
        print(f"[probe] Comm.drain_pending in {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr, flush=True)
    if drain == "drain":
        t0 = time.perf_counter()
        pg._wait_for_pending_works()
        print(f"[probe] drained pending works in {1e3 * (time.perf_counter() - t0):.1f} ms", file=sys.stderr,
              flush=True)
    g = torch.cuda.CUDAGraph()
    t0 = time.perf_counter()
    with torch.cuda.graph(g, capture_error_mode=mode):
        for k in range(80):
            x.mul_(1.0)
            if k % 10 == 0:
                dist.all_reduce(x)
            time.sleep(0.01)  # the capture stays open ~0.8 s: the watchdog polls ~8 times inside it
    print(f"[probe] capture open {1e3 * (time.perf_counter() - t0):.0f} ms", file=sys.stderr, flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize(dev)
    time.sleep(0.3)  # let the watchdog poll again after the capture
    ok = bool(torch.all(x == 1.0).item())
    print(f"[probe] {variant}: replays done, values ok={ok}", file=sys.stderr, flush=True)
    dist.destroy_process_group()
    print("PROBE_OK", flush=True)


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return 0
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/watchdog_probe"
    variants = sys.argv[2:] or VARIANTS
    os.makedirs(out, exist_ok=True)
    summary = []
    for v in variants:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   TORCH_NCCL_ASYNC_ERROR_HANDLING="1")
        t0 = time.time()
        try:
            r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", v], env=env,
                               capture_output=True, text=True, timeout=120)
            rc, so, se = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired as e:
            rc, so, se = "timeout", str(e.stdout or ""), str(e.stderr or "")
        with open(os.path.join(out, f"{v}.log"), "w") as f:
            f.write(f"# variant {v} rc={rc} wall={time.time() - t0:.1f}s\n# ---- stdout\n{so}\n# ---- stderr\n{se}")
        what = [ln for ln in se.splitlines() if "what()" in ln or "HIP error" in ln or "terminated with" in ln]
        summary.append(f"{v}: rc={rc} ok={'PROBE_OK' in so} {what[:2]}")
        print(summary[-1], flush=True)
        if rc != 0:  # an abort / fault / time limit: start nothing more on the GPU
            break
    with open(os.path.join(out, "summary.txt"), "w") as f:
        f.write("\n".join(summary) + "\n")
    return 0 if all(" rc=0 " in ln for ln in summary) and len(summary) == len(variants) else 3


if __name__ == "__main__":
    sys.exit(main())
