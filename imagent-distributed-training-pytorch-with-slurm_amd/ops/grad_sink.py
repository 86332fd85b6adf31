"""Gradient-ready notifications from kernels to the bucketed reducer.

Native backward kernels write each parameter gradient straight into the
parameter's slot of the flat gradient arena (``param.grad`` is a view into
it) and then call :func:`notify_ready`. The data-parallel wrapper
(:mod:`imagent_amd.parallel.ddp`) installs a sink that maps the parameter to
its bucket and launches the bucket's all-reduce as soon as the bucket is
complete - the analogue of the c10d Reducer's autograd hooks
([torch] reducer.hpp:275-285), without an extra copy into a bucket buffer.
"""

from __future__ import annotations

from typing import Callable, Optional

_sink: Optional[Callable] = None


def set_sink(fn: Optional[Callable]) -> Optional[Callable]:
    global _sink
    prev, _sink = _sink, fn
    return prev


def notify_ready(param) -> None:
    if _sink is not None:
        _sink(param)
