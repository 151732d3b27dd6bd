"""Rank-aware logging that keeps the reference's log grammar.

Reference: ``J/utils/LogUtils.java:41-65`` -- ``importantInfo`` prints on rank 0 /
thread 0 only, ``verboseInfo`` is gated by the config ``verbose`` flag, errors go
to every rank. The reference ships slave logs to a master process; here every
rank writes to stderr/its own file and rank 0 owns the user-facing stream.
An optional JSONL metrics sink records per-round numbers.
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from typing import Optional


class YtkLogger:
    def __init__(self, rank: int = 0, verbose: bool = False, stream=None, jsonl_path: Optional[str] = None,
                 every: int = 1):
        self.rank = rank
        self.verbose = verbose
        self.stream = stream or sys.stdout
        self.every = max(1, every)
        self.jsonl = open(jsonl_path, "a") if (jsonl_path and rank == 0) else None
        self.quiet = os.environ.get("YTK_QUIET", "0") == "1"

    def info(self, msg: str, all_ranks: bool = False):
        if self.quiet:
            return
        if self.rank == 0 or all_ranks:
            ts = time.strftime("%Y-%m-%d %H:%M:%S")
            self.stream.write(f"{ts} [rank {self.rank}] {msg}\n")
            self.stream.flush()

    def verbose_info(self, msg: str):
        if self.verbose:
            self.info(msg)

    def error(self, msg: str):
        sys.stderr.write(f"[rank {self.rank}] ERROR {msg}\n")
        sys.stderr.flush()

    def metric(self, **kv):
        if self.jsonl is not None:
            self.jsonl.write(json.dumps(kv) + "\n")
            self.jsonl.flush()

    def enabled_for_round(self, i: int) -> bool:
        return ((i + 1) % self.every) == 0


def get_logger(comm=None, verbose: bool = False, **kw) -> YtkLogger:
    rank = comm.rank if comm is not None else 0
    return YtkLogger(rank, verbose, **kw)
