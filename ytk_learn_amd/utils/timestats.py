"""Per-phase timers for the training loops (reference: ``J/data/gbdt/TimeStats.java:30-78``:
BuildHist (compute / communicate), InitStats, FindBestSplit, SyncBestSplit per tree and in
total, printed per round when ``verbose``).

On the GPU the timer records a HIP event at every phase boundary on the current stream
(no synchronisation inside the round, so the asynchronous device builder keeps its
overlap) and resolves the elapsed times once per tree in :meth:`PhaseTimer.end`. On the CPU
it uses ``perf_counter``. Collective phases measure from the stream's point of view: the
time the compute stream waited for RCCL. Disabled timers cost nothing.

Enable with ``--profile`` on the CLI / bench (or ``YTK_PROFILE=1``).
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch


def profiling_enabled(flag: Optional[bool] = None) -> bool:
    if flag is not None:
        return bool(flag)
    return os.environ.get("YTK_PROFILE", "0") not in ("", "0", "false", "False")


class PhaseTimer:
    def __init__(self, device: Optional[torch.device] = None, enabled: bool = False):
        self.device = device if device is not None else torch.device("cpu")
        self.enabled = enabled
        self.cuda = self.enabled and self.device.type == "cuda"
        self._marks: List[Tuple[str, object]] = []
        self.totals: "OrderedDict[str, float]" = OrderedDict()
        self.last: "OrderedDict[str, float]" = OrderedDict()
        self.count = 0

    def _now(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def begin(self):
        """Start a new unit (tree / iteration)."""
        if self.enabled:
            self._marks = [("", self._now())]

    def mark(self, phase: str):
        """Attribute the time since the previous mark to ``phase``."""
        if self.enabled:
            if not self._marks:
                self.begin()
            self._marks.append((phase, self._now()))

    def end(self) -> Dict[str, float]:
        """Resolve this unit's phase times (ms); one device synchronisation on the GPU."""
        if not self.enabled or len(self._marks) < 2:
            self._marks = []
            return {}
        if self.cuda:
            self._marks[-1][1].synchronize()
        per: "OrderedDict[str, float]" = OrderedDict()
        for (_, a), (name, b) in zip(self._marks[:-1], self._marks[1:]):
            ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
            per[name] = per.get(name, 0.0) + ms
        for k, v in per.items():
            self.totals[k] = self.totals.get(k, 0.0) + v
        self.count += 1
        self.last = per
        self._marks = []
        return per

    @staticmethod
    def fmt(d: Dict[str, float]) -> str:
        tot = sum(d.values())
        parts = ", ".join(f"{k}:{v:.3f}ms" for k, v in d.items())
        return f"{parts} (sum {tot:.3f}ms)"

    def report(self) -> str:
        if not self.count:
            return ""
        avg = OrderedDict((k, v / self.count) for k, v in self.totals.items())
        return (f"time stats over {self.count} units, total: {self.fmt(self.totals)}\n"
                f"time stats per unit (avg): {self.fmt(avg)}")
