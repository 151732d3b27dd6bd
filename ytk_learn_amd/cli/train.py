"""Training CLI.

Reference: ``J/worker/LocalTrainWorker.java:30-81`` (positional ``model conf pyScript
needPy user host port threads``) and ``bin/local_optimizer.sh``. Multi-GPU: run under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 -m
ytk_learn_amd.cli.train ...`` -- every rank reads RANK / WORLD_SIZE / LOCAL_RANK.

  python -m ytk_learn_amd.cli.train MODEL CONF [--transform-script transform.py]
         [--device cuda|cpu] [--threads N] [--set key=value ...]
The reference's positional form is also accepted:
  python -m ytk_learn_amd.cli.train MODEL CONF PY_SCRIPT NEED_PY [user host port threads]
"""
from __future__ import annotations

import argparse
import os
import sys

from ..config.hocon import parse_override_value
from ..utils.errors import YtkLearnError


def parse_args(argv):
    ap = argparse.ArgumentParser(prog="ytk_learn_amd.cli.train")
    ap.add_argument("model")
    ap.add_argument("conf")
    ap.add_argument("legacy", nargs="*", help="reference positional args: py_script need_py [user host port threads]")
    ap.add_argument("--transform-script", default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--profile", action="store_true",
                    help="per-phase device timers (TimeStats) per tree / iteration and in total")
    ap.add_argument("--metrics-jsonl", default=None, metavar="PATH",
                    help="append per-round / per-iteration metrics as JSON lines (rank 0)")
    a = ap.parse_args(argv)
    if a.legacy:
        py_script = a.legacy[0]
        need_py = len(a.legacy) > 1 and a.legacy[1].lower() == "true"
        if need_py and a.transform_script is None:
            a.transform_script = py_script
        if len(a.legacy) >= 6 and a.threads == 0:
            try:
                a.threads = int(a.legacy[5])
            except ValueError:
                pass
    return a


def main(argv=None) -> int:
    a = parse_args(sys.argv[1:] if argv is None else argv)
    overrides = {}
    for kv in a.set:
        if "=" not in kv:
            raise YtkLearnError(f"--set expects KEY=VALUE, got {kv}")
        k, v = kv.split("=", 1)
        overrides[k.strip()] = parse_override_value(v)
    if a.profile:
        os.environ["YTK_PROFILE"] = "1"
    if a.metrics_jsonl:
        os.environ["YTK_METRICS_JSONL"] = a.metrics_jsonl
    from ..train import train
    from ..parallel.comm import Comm
    comm = Comm.from_env(a.device)
    code = 0
    try:
        train(a.model, a.conf, overrides, a.transform_script, comm=comm, threads=a.threads)
    except Exception as e:  # reference: comm.exception(e); comm.close(1); exit(1)
        sys.stderr.write(f"[rank {comm.rank}] training failed: {e!r}\n")
        code = 1
        raise
    finally:
        comm.close()
        print(f"exit code:{code}", flush=True) if comm.rank == 0 else None
    return code


if __name__ == "__main__":
    sys.exit(main())
