"""Gradient-ready notifications from kernels to the bucketed reducer.

Native backward kernels write each parameter gradient straight into the
parameter's slot of the flat gradient arena (``param.grad`` is a view into
it) and then call :func:`notify_ready`. The data-parallel wrapper
(:mod:`imagent_amd.parallel.ddp`) attaches ``param._imagent_ready`` which
maps the parameter to its bucket and launches the bucket's all-reduce as
soon as the bucket is complete - the analogue of the c10d Reducer's
autograd hooks ([torch] reducer.hpp:275-285), without an extra copy into a
bucket buffer. Without a wrapper (single-process use) this is a no-op.
"""

from __future__ import annotations


def notify_ready(param) -> None:
    fn = getattr(param, "_imagent_ready", None)
    if fn is not None:
        fn(param)
