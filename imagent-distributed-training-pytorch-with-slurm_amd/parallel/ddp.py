"""Bucketed data parallelism over the flat gradient arena.

Capabilities of ``DistributedDataParallel(model, device_ids=[local_rank])``
as the reference uses it (``imagenet.py:316``):

* init: parameter-shape verification across ranks + broadcast of parameters
  and buffers from rank 0 ([torch] distributed.py:862-864);
* backward: gradients are averaged across ranks by bucketed all-reduces that
  start while the rest of the backward is still running;
* iteration 1 observes the real gradient-ready order and the buckets are
  rebuilt once from it ([torch] distributed.py:1551);
* BatchNorm buffers: the reference broadcasts them from rank 0 before EVERY
  forward (``broadcast_buffers=True``). Default here is ``'eval'``: broadcast
  only before validation / checkpointing (the per-step 40-tensor latency-bound
  broadcast buys nothing for per-GPU BN statistics); ``'always'`` restores
  the reference's behaviour exactly.

MI355X design:
* the gradients ARE the buckets (contiguous slices of the arena, in bucket
  order) - the native wgrad / BN-backward kernels accumulate straight into
  them and call :func:`~imagent_amd.ops.grad_sink.notify_ready`;
* bookkeeping (bucket plan, ready tracking, in-order launch) is the C++
  runtime (``csrc/runtime/reducer.cpp``);
* each complete bucket is all-reduced (``ncclAvg``) on the communicator's
  own comm stream (normal priority: a high-priority one measured -15 %,
  profiles/r50_b1024_comm_stream_study.md), ordered after the producing
  kernels by an event;
  the compute stream joins once at the end of backward. Bucket sizes target
  xGMI: a small first bucket (fc grads are ready first) and mid-size caps
  so several collectives overlap the remaining backward.
* ``grad_reduce_dtype='bf16'``: each bucket is rounded into a bf16 copy, the
  copy is all-reduced (half the xGMI bytes of the fp32 buckets; SURVEY §5.8
  sizes the plan at bf16) and written back into the fp32 arena -- on the comm
  stream for RCCL, so the casts overlap the backward like the collective. The
  fp32 masters, momentum and SGD are unchanged.
"""

from __future__ import annotations

import contextlib
import time
import zlib
import ctypes as C
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from ..models.arena import ParamArena
from ..ops import _lib, streams
from .comm import Communicator, LocalCommunicator

MB = 1024 * 1024


def plan_buckets(nbytes: List[int], first_cap: int, cap: int, last_cap: int = 0) -> List[int]:
    """Bucket id per tensor (tensors given in bucket/layout order): greedy, the first bucket capped at
    ``first_cap`` bytes, the others at ``cap``; ``last_cap`` > 0 splits the trailing tensors (at most that many
    bytes, at least one tensor) off the last bucket -- the all-reduce issued after the last gradient, which
    nothing overlaps."""
    n = len(nbytes)
    if n == 0:
        return []
    try:
        L = _lib.runtime()
        arr = (C.c_int64 * n)(*nbytes)
        out = (C.c_int32 * n)()
        L.imr_plan_buckets(n, arr, first_cap, cap, last_cap, out)
        return list(out)
    except _lib.NativeLibraryMissing:
        ids, b, acc, lim = [], 0, 0, first_cap if first_cap > 0 else cap
        for i, s in enumerate(nbytes):
            ids.append(b)
            acc += s
            if acc >= lim and i + 1 < n:
                b, acc, lim = b + 1, 0, cap
        if last_cap > 0:
            start, tail = n - 1, nbytes[-1]
            while start > 0 and ids[start - 1] == b and tail + nbytes[start - 1] <= last_cap:
                start -= 1
                tail += nbytes[start]
            if start > 0 and ids[start - 1] == b:
                ids[start:] = [b + 1] * (n - start)
        return ids


class _Tracker:
    """ctypes wrapper of the native ready tracker (pure-Python fallback)."""

    def __init__(self, bucket_of: List[int], nbuckets: int):
        self.n, self.nb = len(bucket_of), nbuckets
        try:
            self.L = _lib.runtime()
            arr = (C.c_int32 * self.n)(*bucket_of)
            self.h = self.L.imr_tracker_new(self.n, arr, nbuckets)
            self._first, self._count = C.c_int32(), C.c_int32()
        except _lib.NativeLibraryMissing:
            self.L = None
            self.bucket_of = list(bucket_of)
            self.size = [0] * nbuckets
            for b in bucket_of:
                self.size[b] += 1
            self._reset()

    def _reset(self):
        self.pending = list(self.size)
        self.marked = [False] * self.n
        self.next = 0
        self.order: List[int] = []

    def mark(self, i: int):
        if self.L is not None:
            rc = self.L.imr_tracker_mark(self.h, i, C.byref(self._first), C.byref(self._count))
            if rc == -1:
                raise RuntimeError(f"parameter {i} marked ready twice in one iteration (used twice "
                                   "in the forward?)")
            if rc != 0:
                raise RuntimeError(f"tracker error {rc}")
            return self._first.value, self._count.value
        if self.marked[i]:
            raise RuntimeError(f"parameter {i} marked ready twice in one iteration")
        self.marked[i] = True
        self.order.append(i)
        self.pending[self.bucket_of[i]] -= 1
        first = self.next
        while self.next < self.nb and self.pending[self.next] == 0:
            self.next += 1
        return first, self.next - first

    def finalize(self):
        if self.L is not None:
            unready = (C.c_uint8 * self.n)()
            missing = self.L.imr_tracker_finalize(self.h, unready)
            order = (C.c_int32 * self.n)()
            k = self.L.imr_tracker_last_order(self.h, order)
            return missing, [i for i in range(self.n) if unready[i]], list(order)[:k]
        missing = self.nb - self.next
        unready = [i for i in range(self.n) if not self.marked[i]]
        order = list(self.order)
        self._reset()
        return missing, unready, order

    def __del__(self):
        if getattr(self, "L", None) is not None and getattr(self, "h", None):
            self.L.imr_tracker_free(self.h)
            self.h = None


class CommTimeline:
    """How one step's bucketed all-reduces overlap its backward (what an N-GPU run that disappoints needs
    to say why; bench.py reports it as ``comm_overlap``).

    On a GPU communicator with its own comm stream every mark is a timing event: ``begin`` on the compute
    stream at the end of forward, per bucket ``issue`` on the comm stream once it has waited for the bucket's
    producers (main AND weight-gradient side stream: the moment the all-reduce can start on the device) and
    ``done`` after it, ``compute_end`` on the compute stream after the side stream joined (the last backward
    kernel), ``joined`` after the compute stream waited for the comm stream. Without device events (gloo / CPU)
    the marks are host clock readings at the same program points.

    ``stats()`` (synchronises): ``exposed_comm_ms`` = compute_end -> joined (communication the optimizer waits
    for after the last backward kernel), ``comm_stream_busy_ms`` = sum over buckets of issue -> done (device
    only), ``bucket_issue_ms`` / ``bucket_done_ms`` relative to ``begin``, ``backward_ms`` = begin ->
    compute_end, ``issue_order`` = bucket ids in issue order."""

    def __init__(self, ddp: "DataParallel"):
        self.ddp = ddp
        s = getattr(ddp.comm, "stream", None)
        self.dev = s is not None and ddp.arena.G.is_cuda and torch.cuda.is_available()
        self.stream = s
        self._reset()

    def _reset(self):
        self.t0 = self.tc = self.tj = None
        self.iss, self.dn, self.order = {}, {}, []

    def _mark(self, stream=None):
        if not self.dev:
            return time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream if stream is not None else torch.cuda.current_stream())
        return e

    def begin(self):
        self._reset()
        self.t0 = self._mark()

    def issue(self, b: int):
        if self.t0 is None:
            return
        if self.dev:  # the comm stream waits for the bucket's producers first: the event marks the device start
            self.ddp.comm.depend_on(torch.cuda.current_stream())
        self.iss[b] = self._mark(self.stream)
        self.order.append(b)

    def done(self, b: int):
        if self.t0 is not None:
            self.dn[b] = self._mark(self.stream)

    def compute_end(self):
        if self.t0 is not None:
            self.tc = self._mark()

    def joined(self):
        if self.t0 is not None:
            self.tj = self._mark()

    def _ms(self, a, b) -> float:
        if self.dev:
            return float(a.elapsed_time(b))
        return 1000.0 * (b - a)

    def stats(self) -> dict:
        if self.t0 is None or self.tj is None:
            return {}
        if self.dev:
            torch.cuda.synchronize()
        nb = len(self.ddp.buckets)
        out = {
            "exposed_comm_ms": round(self._ms(self.tc, self.tj), 3),
            "backward_ms": round(self._ms(self.t0, self.tc), 3),
            "bucket_issue_ms": [round(self._ms(self.t0, self.iss[b]), 3) if b in self.iss else None for b in range(nb)],
            "bucket_done_ms": ([round(self._ms(self.t0, self.dn[b]), 3) if b in self.dn else None for b in range(nb)]
                               if self.dev else None),
            "comm_stream_busy_ms": (round(sum(self._ms(self.iss[b], self.dn[b]) for b in self.iss if b in self.dn), 3)
                                    if self.dev else None),
            "issue_order": list(self.order),
            "clock": "device events" if self.dev else "host",
        }
        return out


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, arena: ParamArena, comm: Optional[Communicator] = None,
                 bucket_cap_mb: float = 16.0, first_bucket_mb: float = 2.0, last_bucket_mb: float = 1.0,
                 broadcast_buffers: str = "eval", rebuild_buckets: bool = True,
                 find_unused_parameters: bool = False, use_autograd_hooks: Optional[bool] = None,
                 probe_order: bool = False, grad_reduce_dtype: str = "fp32"):
        super().__init__()
        self.module = module
        self.arena = arena
        self.comm = comm or LocalCommunicator()
        self.cap = int(bucket_cap_mb * MB)
        self.first_cap = int(first_bucket_mb * MB)
        self.last_cap = int(last_bucket_mb * MB)
        # per-step record of how the bucket all-reduces overlap backward (comm_timeline(), bench JSON); off
        # unless asked for: a few event records per bucket
        self.timeline: Optional["CommTimeline"] = None
        self.broadcast_buffers = broadcast_buffers
        self.rebuild_pending = rebuild_buckets
        self.find_unused = find_unused_parameters
        self.sync_enabled = True
        self.iteration = 0
        self._callback_queued = False
        self._in_backward = False
        self.last_order: List[int] = []
        # ordering probe (race detector): a checksum of every bucket taken ON
        # the comm stream right after its all-reduce; see verify_order()
        self.probe_order = probe_order
        self._probe_sums: Optional[torch.Tensor] = None
        if grad_reduce_dtype not in ("fp32", "bf16"):
            raise ValueError(f"grad_reduce_dtype must be fp32 or bf16, not {grad_reduce_dtype!r}")
        self.grad_reduce_dtype = grad_reduce_dtype
        # bf16 bucket copies: one buffer shaped like the arena (bucket b = the same slice)
        self._g16 = (torch.empty(self.arena.G.numel(), dtype=torch.bfloat16, device=self.arena.G.device)
                     if grad_reduce_dtype == "bf16" else None)
        self._g16_pending: List[int] = []  # buckets to write back after join (no comm stream)

        self._verify_and_broadcast()
        self._plan()
        for i, p in enumerate(self.arena.params):
            p._imagent_ready = self._mark_param
            p._imagent_index = i
        if use_autograd_hooks is None:
            use_autograd_hooks = getattr(module, "backend", "torch") not in ("hip", "hip_f32")
        self.hooks = []
        if use_autograd_hooks:
            for p in self.arena.params:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._mark_param))

    # ----------------------------------------------------------- set-up
    def _verify_and_broadcast(self):
        ws = self.comm.world_size
        if ws <= 1:
            return
        # shape verification (X2): every rank must hold the same parameter list
        desc = repr([(n, s) for n, s in zip(self.arena.names, self.arena.shapes)]).encode()
        sig = torch.tensor([zlib.crc32(desc), len(self.arena.names)], dtype=torch.int64,
                           device=self.arena.P.device)
        allsig = self.comm.allgather(sig)
        if not bool((allsig == allsig[0]).all()):
            raise RuntimeError("DataParallel: parameter shapes differ across ranks")
        # parameters + buffers from rank 0 (X3), one flat broadcast each
        self.comm.broadcast_(self.arena.P, 0)
        self.sync_buffers()

    def _plan(self):
        order = self.arena.order
        nbytes = [self.arena.nbytes_of(i) for i in order]
        bid_in_order = plan_buckets(nbytes, self.first_cap, self.cap, self.last_cap)
        nb = (max(bid_in_order) + 1) if bid_in_order else 0
        bucket_of = [0] * len(order)
        for pos, i in enumerate(order):
            bucket_of[i] = bid_in_order[pos]
        self.bucket_of = bucket_of
        # contiguous slices of G per bucket
        self.buckets = []
        for b in range(nb):
            members = [i for i in order if bucket_of[i] == b]
            lo = self.arena.offsets[members[0]]
            last = members[-1]
            hi = self.arena.offsets[last] + self.arena.numels[last]
            self.buckets.append((lo, hi, members))
        self.tracker = _Tracker(bucket_of, nb)

    @torch.no_grad()
    def check_consistency(self, raise_on_mismatch: bool = True) -> bool:
        """Race / divergence detector: after identical averaged
        gradients every rank must hold bit-identical parameters. A bucket read
        by RCCL before its producing kernel finished, or a compute kernel
        overwriting a bucket during its all-reduce, shows up here as a
        checksum mismatch. Costs one tiny all-gather; call it every N steps."""
        if self.comm.world_size <= 1:
            return True
        P = self.arena.P
        sig = torch.stack([P.double().sum(), (P.double() * torch.arange(P.numel(), device=P.device,
                                                                         dtype=torch.float64).remainder_(977)).sum()])
        allsig = self.comm.allgather(sig)
        ok = bool((allsig == allsig[0]).all())
        if not ok and raise_on_mismatch:
            raise RuntimeError(f"DataParallel: parameters diverged across ranks: {allsig.tolist()}")
        return ok

    def bucket_sizes_mb(self) -> List[float]:
        return [(hi - lo) * 4 / MB for lo, hi, _ in self.buckets]

    def sync_buffers(self):
        """Broadcast every buffer (BN running stats, counters) from rank 0."""
        if self.comm.world_size <= 1:
            return
        bufs = [b for b in self.module.buffers()]
        if not bufs:
            return
        dev = self.arena.P.device
        f = [b for b in bufs if b.dtype == torch.float32]
        o = [b for b in bufs if b.dtype != torch.float32]
        if f:
            flat = torch.cat([b.reshape(-1) for b in f]).to(dev)
            self.comm.broadcast_(flat, 0)
            off = 0
            for b in f:
                b.copy_(flat[off:off + b.numel()].view_as(b))
                off += b.numel()
        if o:
            flat = torch.cat([b.reshape(-1).to(torch.int64) for b in o]).to(dev)
            self.comm.broadcast_(flat, 0)
            off = 0
            for b in o:
                b.copy_(flat[off:off + b.numel()].view_as(b))
                off += b.numel()

    # ---------------------------------------------------------- forward
    def forward(self, *args, **kw):
        if self.broadcast_buffers == "always" and self.module.training:
            self.sync_buffers()
        out = self.module(*args, **kw)
        if self.timeline is not None and self.module.training and torch.is_grad_enabled():
            self.timeline.begin()  # end of forward ~ start of backward (the loss kernel is microseconds)
        return out

    def comm_timeline(self, on: bool = True) -> None:
        """Record the next steps' bucket timing (:class:`CommTimeline`); read it with ``timeline.stats()``."""
        self.timeline = CommTimeline(self) if on else None

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: skip communication inside the context."""
        prev = self.sync_enabled
        self.sync_enabled = False
        try:
            yield
        finally:
            self.sync_enabled = prev

    # --------------------------------------------------------- backward
    def _mark_param(self, p):
        if not self.sync_enabled:
            return
        i = p._imagent_index
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize_backward)
        first, count = self.tracker.mark(i)
        for b in range(first, first + count):
            self._launch(b)

    def _launch(self, b: int):
        lo, hi, _ = self.buckets[b]
        side = streams.active_side_stream()
        if side is not None:
            # bucket members may have been produced on the wgrad side stream:
            # the all-reduce waits for it too (main stream not blocked)
            self.comm.depend_on(side)
        tl = self.timeline
        if tl is not None:
            tl.issue(b)
        if self._g16 is None:
            self.comm.allreduce_(self.arena.G[lo:hi], "avg")
        else:
            self._launch_bf16(b, lo, hi)
        if tl is not None:
            tl.done(b)
        if self.probe_order:
            self._probe(b, lo, hi)

    def _launch_bf16(self, b: int, lo: int, hi: int) -> None:
        g, h = self.arena.G[lo:hi], self._g16[lo:hi]
        s = getattr(self.comm, "stream", None) if g.is_cuda else None
        if s is not None:
            from ..ops.misc import cast_bf16, uncast_bf16
            self.comm.depend_on(torch.cuda.current_stream(g.device))  # after the producers
            with torch.cuda.stream(s):  # cast, reduce, write back: all ordered on the comm stream
                cast_bf16(g, h)
                self.comm.allreduce_(h, "avg")
                uncast_bf16(h, g)
        else:
            h.copy_(g)
            self.comm.allreduce_(h, "avg")
            self._g16_pending.append(b)  # the collective may still be in flight: write back after join

    def _probe(self, b: int, lo: int, hi: int) -> None:
        s = getattr(self.comm, "stream", None)
        if s is None or not self.arena.G.is_cuda:
            return
        if self._probe_sums is None or self._probe_sums.numel() != len(self.buckets):
            self._probe_sums = torch.full((len(self.buckets),), float("nan"), dtype=torch.float64,
                                          device=self.arena.G.device)
        with torch.cuda.stream(s):
            torch.sum(self.arena.G[lo:hi].view(1, -1), dim=1, dtype=torch.float64,
                      out=self._probe_sums.narrow(0, b, 1))

    @torch.no_grad()
    def verify_order(self) -> List[int]:
        """Buckets whose all-reduce saw different data than the finished
        gradient (call after the step, before the next ``zero_grad``).

        The probe sums each bucket on the comm stream right after its
        collective. If the collective was ordered after every kernel that
        writes the bucket (main stream AND wgrad side stream), that checksum
        equals the one of the final gradient bit for bit (same data, same
        deterministic reduction); a bucket reduced before a producer finished
        shows up as a mismatch. Returns the mismatching bucket ids."""
        if self._probe_sums is None:
            return []
        torch.cuda.synchronize(self.arena.G.device)
        got = self._probe_sums.clone()
        want = torch.stack([self.arena.G[lo:hi].view(1, -1).sum(dim=1, dtype=torch.float64)[0]
                            for lo, hi, _ in self.buckets])
        self._probe_sums.fill_(float("nan"))
        return [b for b in range(len(self.buckets)) if not bool(got[b] == want[b])]

    def abandon_backward(self) -> None:
        """A backward raised part-way: forget its ready marks and queued callback."""
        if self._callback_queued:
            self._callback_queued = False
            self.tracker.finalize()

    def _finalize_backward(self):
        self._callback_queued = False
        missing, unready, order = self.tracker.finalize()
        if missing:
            if not self.find_unused:
                names = [self.arena.names[i] for i in unready][:8]
                raise RuntimeError(
                    "DataParallel: expected to have finished reduction in the prior iteration; "
                    f"{len(unready)} parameters never produced a gradient (e.g. {names}). "
                    "Pass find_unused_parameters=True if this is intended.")
            # unused parameters contribute zeros: launch the remaining buckets in order
            for b in range(len(self.buckets) - missing, len(self.buckets)):
                self._launch(b)
        streams.join_side_into_current()  # the optimizer reads the gradient arena
        if self.timeline is not None:
            self.timeline.compute_end()
        self.comm.join()
        if self.timeline is not None:
            self.timeline.joined()
        for b in self._g16_pending:
            lo, hi, _ = self.buckets[b]
            self.arena.G[lo:hi].copy_(self._g16[lo:hi])
        self._g16_pending.clear()
        self.iteration += 1
        self.last_order = order
        if self.rebuild_pending and self.iteration == 1 and order:
            self.rebuild_pending = False
            self._maybe_rebuild(order)

    def _maybe_rebuild(self, ready_order: List[int]):
        """Rebuild the layout once from the observed ready order (torch DDP
        rebuilds its buckets after the first iteration). The optimizer
        must not own arena-shaped state yet (it is created lazily)."""
        seen = set(ready_order)
        order = list(ready_order) + [i for i in self.arena.order if i not in seen]
        if self.comm.world_size > 1:
            # every rank must use the SAME layout: take rank 0's observed order
            t = torch.tensor(order, dtype=torch.int64, device=self.arena.P.device)
            self.comm.broadcast_(t, 0)
            order = t.tolist()
        if order == list(self.arena.order):
            return
        self.pending_relayout = order

    def apply_pending_relayout(self, flats=()):
        order = getattr(self, "pending_relayout", None)
        if order is None:
            return list(flats)
        self.pending_relayout = None
        out = self.arena.relayout(order, flats)
        self._plan()
        return out
