"""Tracing helpers (absent in the reference).

* :func:`profiled` - torch.profiler around a region, Chrome trace to a dir;
* :class:`StepTimer` - HIP-event step timing without host syncs inside the
  loop (events are read back once at the end);
* :func:`range_push` / :func:`range_pop` - roctx ranges (visible in
  ``rocprofv3 --marker-trace``) when available.
"""

from __future__ import annotations

import contextlib
import os
from typing import List

import torch


@contextlib.contextmanager
def profiled(outdir: str, wait: int = 2, warmup: int = 2, active: int = 5):
    os.makedirs(outdir, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False,
                                on_trace_ready=torch.profiler.tensorboard_trace_handler(outdir)) as p:
        yield p


def range_push(name: str) -> None:
    try:
        torch.cuda.nvtx.range_push(name)
    except Exception:
        pass


def range_pop() -> None:
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


class StepTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.events: List[torch.cuda.Event] = []

    def mark(self):
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append(e)

    def times_ms(self) -> List[float]:
        if len(self.events) < 2:
            return []
        self.events[-1].synchronize()
        return [a.elapsed_time(b) for a, b in zip(self.events[:-1], self.events[1:])]

    def percentiles(self, qs=(50, 90, 99)):
        t = sorted(self.times_ms())
        if not t:
            return {}
        return {q: t[min(len(t) - 1, int(round(q / 100 * (len(t) - 1))))] for q in qs}
