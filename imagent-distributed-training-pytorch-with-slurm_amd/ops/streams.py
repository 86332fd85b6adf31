"""Side stream for weight-gradient kernels (backward overlap).

In backward, a conv's dgrad (feeds the next layer's backward: critical path)
and its wgrad (feeds only the gradient arena and the all-reduce) both consume
the same upstream gradient and are independent. Queuing every wgrad on a
second HIP stream lets it fill the CUs the critical-path kernels leave idle
(wave-quantisation tails, small late-stage grids) instead of serialising.

Dependencies that make this safe:
* the side stream waits for the main stream before each wgrad (its inputs);
* tensors read on the side stream are held (:func:`protect`) until the
  end-of-backward join, then released in main-stream order, so the caching
  allocator cannot recycle them while a side-stream kernel still reads them
  (``record_stream`` instead measured the same img/s at 2.4x the reserved HBM);
* the data-parallel reducer makes each bucket's all-reduce wait for the side
  stream as well as the main one (``parallel/ddp.py``), and the end of
  backward joins the side stream into the main one (the optimizer reads the
  gradient arena).
"""

from __future__ import annotations

from typing import Dict, Optional

import torch

_enabled = False
_streams: Dict[int, torch.cuda.Stream] = {}


def set_wgrad_overlap(on: bool) -> None:
    global _enabled
    _enabled = bool(on)


def overlap_enabled() -> bool:
    return _enabled


def side_stream(device: Optional[torch.device] = None) -> Optional[torch.cuda.Stream]:
    """The wgrad stream of ``device`` (None when the overlap is off or on CPU)."""
    if not _enabled or not torch.cuda.is_available():
        return None
    idx = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    s = _streams.get(idx)
    if s is None:
        s = _new_stream(idx)
        _streams[idx] = s
    return s


def side_cumask() -> int:
    """IMAGENT_SIDE_CUMASK = q in 1..4: the side stream runs on q / 4 of the CUs (a CU-masked HIP stream,
    ``imk_stream_create_cumask``); 0 (default): a plain stream over every CU. Measured at the 4096 default
    (scripts/runs/cumask_ab.sh, one box): plain 17,500 / 17,471 img/s, q = 3 13,664 / 13,628, q = 2 13,310 / 13,314,
    q = 1 10,434 -- the weight-gradient grids are sized for one wave over all 256 CUs, and the side stream's work is
    90 ms of the 233 ms step: confined, it becomes the step's tail. Kept as an A/B switch only."""
    import os
    return int(os.environ.get("IMAGENT_SIDE_CUMASK", "0"))


def _new_stream(idx: int):
    """A torch pool stream (normal priority: the alternatives measured slower, ``parallel/comm.py``
    :func:`stream_mode`), or a CU-masked one (:func:`side_cumask`), kept for the process lifetime."""
    q = side_cumask()
    if q:
        import ctypes as C
        from . import _lib
        ptr = C.c_void_p()
        with torch.cuda.device(idx):
            _lib.check(_lib.kernels().imk_stream_create_cumask(q, C.byref(ptr)), "CU-masked side stream")
        return torch.cuda.ExternalStream(ptr.value, device=torch.device("cuda", idx))
    return torch.cuda.Stream(device=idx)


def active_side_stream() -> Optional[torch.cuda.Stream]:
    """The side stream if one has been used on the current device."""
    if not _enabled or not torch.cuda.is_available():
        return None
    return _streams.get(torch.cuda.current_device())


_keep: list = []
# events of the fork / join edges recorded while a HIP graph is being captured: held until the capture has ended
# (GraphedStep clears them). torch's Stream.wait_stream records a TEMPORARY event that is destroyed as soon as the
# wait is enqueued; inside a two-stream capture on ROCm 7 that destroyed event is still referenced by the capture
# and hipStreamEndCapture segfaulted (tests/test_model_gpu.py::test_graphed_two_stream_step_matches_eager)
_capture_events: list = []


def wait(dst: torch.cuda.Stream, src: torch.cuda.Stream) -> None:
    """``dst`` waits for everything issued so far on ``src`` (Stream.wait_stream with an event that outlives a
    capture in progress). A stream never waits on itself: eagerly that is a no-op, but inside a HIP graph capture
    ROCm 7 turns the event wait into a self-edge of the captured graph, and hipStreamEndCapture's recursive walk
    of the graph then recurses without end (the two-stream capture segfault of rounds 1 and 5: the reducer's
    ``depend_on(side)`` issued from a weight-gradient launch already running ON the side stream; native
    backtrace and HIP API log in profiles/r50_small_batch_graph_r6.md)."""
    if dst.cuda_stream == src.cuda_stream:
        return
    ev = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)
    if torch.cuda.is_current_stream_capturing():
        _capture_events.append(ev)


def release_capture_events() -> None:
    _capture_events.clear()
# Side-stream operands are held until the end-of-backward join, then freed in
# main-stream order (immediately reusable), rather than record_stream'ed (freed
# only once the allocator sees the side stream pass them, so with the CPU ahead
# of the GPU every step got fresh blocks). Measured at R50 / 1024 img
# (profiles/r50_b1024_allocator.md): reserved HBM 129 -> 52.7 GiB, peak 40.6 -> 45.9 GiB,
# img/s unchanged.


def protect(*tensors: torch.Tensor) -> None:
    """Keep tensors read on the side stream from being recycled too early: a
    reference is held until the side stream has been joined back into the
    main stream (default, and always while a HIP graph is being captured,
    where ``record_stream`` is not usable; the join is also the dependency
    edge a captured graph needs)."""
    if active_side_stream() is None:
        return
    _keep.extend(tensors)


def join_side_into_current() -> None:
    s = active_side_stream()
    if s is not None:
        wait(torch.cuda.current_stream(), s)
    _keep.clear()


_join_queued = False
_deferred: list = []


def defer(fn) -> None:
    """Queue a weight-gradient launch to be issued by the NEXT backward node,
    after its memory-bound BN pass (so the side stream overlaps that node's
    dgrad instead). Runs right away when the side stream is off."""
    if active_side_stream() is None:
        fn()
    else:
        _deferred.append(fn)


def flush_deferred() -> None:
    """Issue the queued weight-gradient launches (in order)."""
    while _deferred:
        _deferred.pop(0)()


def deferred() -> int:
    return len(_deferred)


def held() -> int:
    """Number of side-stream operands currently held (0 after every join)."""
    return len(_keep)


def reset() -> None:
    """Start-of-step / failure-path reset: join anything still outstanding and
    forget a join callback that a failed backward never ran (otherwise later
    backwards would never queue their own join and ``_keep`` would grow)."""
    global _join_queued
    _join_queued = False
    _deferred.clear()
    if _keep:
        join_side_into_current()


def _join_cb() -> None:
    global _join_queued
    _join_queued = False
    join_side_into_current()


def ensure_join_after_backward() -> None:
    """Queue (once per backward pass) a join of the side stream into the main
    stream, so whoever reads ``.grad`` after ``backward()`` sees finished
    gradients even without the data-parallel reducer."""
    global _join_queued
    if _join_queued:
        return
    try:
        torch.autograd.Variable._execution_engine.queue_callback(_join_cb)
        _join_queued = True
    except RuntimeError:  # not inside a backward pass: join right away
        join_side_into_current()
