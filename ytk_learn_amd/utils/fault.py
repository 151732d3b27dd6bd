"""Test-only fault injection ("kill rank r at round n to verify resume").

``YTK_FAULT_INJECT=<loop>:<rank>:<step>[:<mode>]`` makes rank ``<rank>`` fail when loop
``<loop>`` (``gbdt`` boosting round, ``lbfgs`` iteration, ``gbst`` soft tree, ``bench``
timed round) is about to run step ``<step>`` (0-based). ``mode`` = ``exit`` (default: the
process dies with status 75 without cleanup, like a killed worker), ``raise`` (a Python
exception, so the normal error path runs), ``skip`` (:func:`fault_point` returns True and the
caller silently drops that step -- e.g. loop ``peer``: one peer-memory exchange this rank never
issues, so its peers' flag waits must time out and raise) or ``stall`` (the rank hangs without exiting, like
a wedged worker: the other ranks' collectives must time out and fail the job). Several specs can be given separated by ``;``. With ``YTK_FAULT_ONCE=<file>``
a spec fires only while ``<file>`` does not exist (it is created when the fault fires), so a
restarted job runs through. Unset: no cost beyond a dictionary lookup per step.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Tuple

FAULT_EXIT_CODE = 75
_cache: Dict[str, Tuple] = {}


class InjectedFault(RuntimeError):
    pass


def _specs():
    raw = os.environ.get("YTK_FAULT_INJECT", "")
    if _cache.get("raw") == raw:
        return _cache["specs"]
    specs = []
    for part in filter(None, (p.strip() for p in raw.split(";"))):
        f = part.split(":")
        if len(f) < 3:
            raise ValueError(f"YTK_FAULT_INJECT: expected loop:rank:step[:mode], got {part!r}")
        specs.append((f[0], int(f[1]), int(f[2]), f[3] if len(f) > 3 else "exit"))
    _cache["raw"], _cache["specs"] = raw, specs
    return specs


def fault_point(loop: str, step: int, rank: int = 0) -> bool:
    """Fire the matching spec, if any; True only for a ``skip`` spec (the caller drops the step)."""
    for lp, r, st, mode in _specs():
        if lp == loop and r == rank and st == step:
            once = os.environ.get("YTK_FAULT_ONCE")
            if once:  # fire only the first time (a restarted job then runs through)
                if os.path.exists(once):
                    continue
                open(once, "w").close()
            msg = f"[rank {rank}] injected fault at {loop} step {step}"
            if mode == "skip":
                sys.stderr.write(msg + " (skip)\n")
                sys.stderr.flush()
                return True
            if mode == "raise":
                raise InjectedFault(msg)
            if mode == "stall":
                sys.stderr.write(msg + " (stall)\n")
                sys.stderr.flush()
                import time
                while True:
                    time.sleep(60)
            sys.stderr.write(msg + " (exit)\n")
            sys.stderr.flush()
            os._exit(FAULT_EXIT_CODE)
    return False
