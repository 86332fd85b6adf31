"""Communicators: native RCCL (GPU) and torch.distributed (gloo/CPU, or c10d).

The reference's collectives are the DDP bucket all-reduce, the DDP init /
per-forward buffer broadcasts and three scalar metric all-reduces per step
(``imagenet.py:84-86,137-139``).

:class:`RcclCommunicator` owns its own RCCL communicator (bootstrapped through
the c10d TCPStore) and its own HIP comm stream: collectives are ordered
after the producing compute stream by an event and the compute stream joins
back with one event wait before the optimizer step. :class:`TorchCommunicator`
offers the same interface over ``torch.distributed`` (``gloo`` for CPU runs
and tests). :class:`LocalCommunicator` is the world-of-one no-op.
"""

from __future__ import annotations

import ctypes as C
import os
import time
import warnings
from typing import List, Optional

import torch
import torch.distributed as dist

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4,
       torch.uint8: 5, torch.float64: 6}
_OP = {"sum": 0, "avg": 1, "max": 2, "min": 3}


class Communicator:
    rank: int = 0
    world_size: int = 1
    name = "base"
    collectives: int = 0  # collectives actually issued (0 for a world of one that skips them)

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> None:
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        raise NotImplementedError

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def join(self) -> None:
        """Make the caller's current stream wait for every issued collective."""

    def synchronize(self) -> None:
        self.join()

    def healthy(self) -> bool:
        return True

    def abort(self) -> None:
        """Failure path: unblock collectives waiting on dead peers."""

    def close(self) -> None:
        pass

    def depend_on(self, stream) -> None:
        """Collectives issued after this call also wait for ``stream``."""
        if torch.cuda.is_available():
            from ..ops.streams import wait
            wait(torch.cuda.current_stream(), stream)


def stream_mode() -> int:
    """Kind of HIP stream for the comm stream: plain, normal priority (0). The alternatives the native
    library still implements measured slower on one MI355X at R50 / 1024 img with RCCL self collectives:

    * highest-priority comm stream (1): 10.2k vs 12.1k img/s. The comm stream spends the backward parked on
      barrier packets (waiting for the next bucket's producers); while a high-priority queue holds work the
      lower-priority queues' wave launches are throttled, and the main-stream forward / BN kernels ran
      10-40 % slower (stats_finalize 5x);
    * full-CU-mask streams (2, a hardware queue each): 8.9k img/s.

    Study: ``profiles/r50_b1024_comm_stream_study.md``."""
    return 0


class LocalCommunicator(Communicator):
    name = "local"

    def allreduce_(self, t, op="sum"):
        return None

    def broadcast_(self, t, root=0):
        return None

    def allgather(self, t):
        return t.unsqueeze(0).clone()


class TorchCommunicator(Communicator):
    """torch.distributed collectives (async), joined in :meth:`join`."""

    name = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self._pending: List[tuple] = []

    def allreduce_(self, t, op="sum"):
        if self.world_size == 1:
            return
        self.collectives += 1
        if op == "avg" and self.backend != "nccl":
            w = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._pending.append((w, t))
            return
        rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        w = dist.all_reduce(t, op=rop, group=self.group, async_op=True)
        self._pending.append((w, None))

    def broadcast_(self, t, root=0):
        if self.world_size > 1:
            dist.broadcast(t, root, group=self.group)

    def allgather(self, t):
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return torch.stack(out)

    def join(self):
        for w, div in self._pending:
            w.wait()
            if div is not None:
                div.div_(self.world_size)
        self._pending.clear()

    def abort(self):
        try:
            dist.distributed_c10d._abort_process_group()
        except Exception:  # best effort: the process exits right after
            pass


class RcclCommunicator(Communicator):
    """Our own RCCL communicator on its own HIP comm stream (normal priority:
    see :func:`stream_mode`).

    Bootstrap (multi-rank): rank 0 publishes the ncclUniqueId through the c10d
    store; every rank starts a NON-BLOCKING ``ncclCommInitRankConfig`` and polls
    it while watching the store for a failure flag. A rank whose init fails
    (or times out) raises the flag before raising, so its peers abort their
    half-built communicators instead of waiting in the RCCL bootstrap, and all
    ranks fall back together (:func:`make_communicator`). A rank that finished
    also waits until every rank reports success, so no rank starts issuing
    RCCL collectives while another has fallen back to c10d.

    ``self_collectives`` (default on, ``IMAGENT_RCCL_SELF=0`` turns it off):
    at world size 1 the collectives are still issued to RCCL (a one-rank
    communicator), so the single-GPU run exercises exactly the comm-stream
    ordering, events and buffer lifetimes of the multi-GPU one.
    """

    name = "rccl"
    _instances = 0  # per-process creation counter: every rank creates communicators in the same order
    live = 0        # communicators currently open in this process

    def __init__(self, rank: int, world_size: int, device: torch.device, store=None,
                 key: Optional[str] = None, self_collectives: Optional[bool] = None,
                 nonblocking: Optional[bool] = None, init_timeout: Optional[float] = None):
        from ..ops import _lib
        self._lib = _lib
        self.L = _lib.comm()
        self.rank, self.world_size = rank, world_size
        self.device = torch.device(device)
        self.h = None
        if self_collectives is None:
            self_collectives = os.environ.get("IMAGENT_RCCL_SELF", "1") != "0"
        if nonblocking is None:
            nonblocking = os.environ.get("IMAGENT_RCCL_NONBLOCKING", "1") != "0"
        if init_timeout is None:  # a stuck bootstrap falls back to c10d after this long (IMAGENT_RCCL_INIT_TIMEOUT)
            init_timeout = float(os.environ.get("IMAGENT_RCCL_INIT_TIMEOUT", "180"))
        self.active = world_size > 1 or bool(self_collectives)
        self.collectives = 0  # collectives handed to RCCL so far
        self._held: List[torch.Tensor] = []
        RcclCommunicator._instances += 1
        key = key or f"imagent/rccl/{RcclCommunicator._instances}"
        multi = store is not None and world_size > 1
        if world_size > 1 and store is None:
            raise RuntimeError("RcclCommunicator needs a c10d store to bootstrap a multi-rank job")
        fail_key = f"{key}/fail"

        def fail(msg: str):
            if multi:
                store.set(fail_key, f"rank {rank}: {msg}")  # peers abort instead of waiting on us
            raise RuntimeError(msg)

        nbytes = self.L.imc_unique_id_bytes()
        if rank == 0:
            buf = C.create_string_buffer(nbytes)
            rc = self.L.imc_get_unique_id(buf)
            uid = buf.raw if rc == 0 else b""
            if multi:
                store.set(f"{key}/uid", uid)  # an empty id tells the other ranks to fail with us
            if rc != 0:
                fail(f"ncclGetUniqueId: {self.L.imc_last_error().decode()}")
        else:
            store.wait([f"{key}/uid"])
            uid = store.get(f"{key}/uid")
            if len(uid) != nbytes:
                raise RuntimeError("rank 0 could not create an RCCL unique id")
        h = C.c_void_p()
        rc = self.L.imc_comm_init_start(uid, world_size, rank, self.device.index or 0, 64, int(nonblocking),
                                        C.byref(h))
        if rc != 0:
            fail(f"ncclCommInitRank: {self.L.imc_last_error().decode()} (rc={rc})")
        self.h = h
        self.L.imc_comm_set_stream_mode(h, stream_mode())
        t0 = time.monotonic()
        delay = 1e-4
        while True:  # non-blocking init: poll, and watch for a peer's failure
            rc = self.L.imc_comm_poll(h)
            if rc == 0:
                break
            if rc < 0:
                msg = self.L.imc_last_error().decode()
                self.abort()
                fail(f"{msg} (rc={rc})")
            if multi and store.check([fail_key]):
                self.abort()
                raise RuntimeError(f"RCCL init abandoned: {store.get(fail_key).decode()}")
            if time.monotonic() - t0 > init_timeout:
                self.abort()
                fail(f"ncclCommInitRank did not finish within {init_timeout:.0f} s")
            time.sleep(delay)
            delay = min(delay * 2, 0.01)
        if multi:  # agreement: nobody proceeds until every rank holds a working communicator
            store.add(f"{key}/ok", 1)
            while store.add(f"{key}/ok", 0) < world_size:
                if store.check([fail_key]):
                    self.abort()
                    raise RuntimeError(f"RCCL init abandoned: {store.get(fail_key).decode()}")
                if time.monotonic() - t0 > init_timeout:
                    self.abort()
                    fail(f"RCCL ranks did not all come up within {init_timeout:.0f} s")
                time.sleep(0.001)
        self.stream = torch.cuda.ExternalStream(self.L.imc_comm_stream(h), device=self.device)
        RcclCommunicator.live += 1

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.L.imc_last_error().decode()} (rc={rc})")

    def _cur(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    @property
    def nranks(self) -> int:
        """Ranks in the RCCL communicator as RCCL itself reports them."""
        return int(self.L.imc_comm_nranks(self.h)) if self.h else 0

    def allreduce_(self, t, op="sum"):
        assert t.is_cuda and t.is_contiguous()
        if not self.active:
            return  # self collectives off: a one-rank all-reduce is the identity
        self._chk(self.L.imc_allreduce(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op], self._cur()),
                  "allreduce")
        self.collectives += 1
        self._held.append(t)  # alive until the caller's stream has joined the comm stream

    def broadcast_(self, t, root=0):
        assert t.is_cuda and t.is_contiguous()
        if not self.active:
            return
        self._chk(self.L.imc_broadcast(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], root, self._cur()),
                  "broadcast")
        self.collectives += 1
        self._held.append(t)
        self.join()

    def allgather(self, t):
        t = t.contiguous()
        if not self.active:
            return t.unsqueeze(0).clone()
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._chk(self.L.imc_allgather(self.h, t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype],
                                       self._cur()), "allgather")
        self.collectives += 1
        self._held.extend((t, out))
        self.join()
        return out

    def depend_on(self, stream) -> None:
        if self.active:  # the comm stream waits; the compute stream keeps going
            self._chk(self.L.imc_stream_join_from(self.h, stream.cuda_stream), "join_from")

    def join(self):
        if self.h:
            self._chk(self.L.imc_stream_join_into(self.h, self._cur()), "join")
        # Operands are held rather than record_stream'ed on the comm stream: once the caller's
        # stream waits for the comm stream, freeing them in the caller's stream order is safe,
        # and no allocator block ever refers to the comm stream (which close() destroys).
        self._held.clear()

    def synchronize(self):
        self._chk(self.L.imc_synchronize(self.h), "sync")

    def healthy(self) -> bool:
        return bool(self.h) and self.L.imc_async_error(self.h) == 0

    def abort(self) -> None:
        """Tear the communicator down without waiting for peers (failure path):
        any collective blocked on a dead rank returns with an error."""
        if getattr(self, "h", None):
            self.L.imc_abort(self.h)

    def close(self):
        if getattr(self, "h", None):
            self.L.imc_comm_destroy(self.h)  # synchronises the comm stream first
            self.h = None
            if hasattr(self, "stream"):
                RcclCommunicator.live -= 1
        self._held.clear()


def _default_store():
    try:
        from torch.distributed.distributed_c10d import _get_default_store
        return _get_default_store()
    except Exception:
        return None


def _fallback_group(ctx):
    """The group the c10d fallback reduces over. GPU jobs bootstrap c10d over gloo
    (:mod:`.dist`), so their fallback creates a ``ProcessGroupNCCL`` HERE, lazily, on
    every rank together (all ranks reach the fallback together); CPU jobs use the
    default group."""
    if getattr(ctx, "device", torch.device("cpu")).type == "cuda" and dist.get_backend() != "nccl":
        return dist.new_group(backend="nccl")
    return None


def rccl_communicators() -> int:
    """RCCL communicators this process holds: the own ones plus c10d's NCCL groups."""
    n = RcclCommunicator.live
    if dist.is_initialized():
        try:
            from torch.distributed.distributed_c10d import _world
            n += sum(1 for pg in _world.pg_map if dist.get_backend(pg) == "nccl")
        except Exception:  # private c10d layout moved: count ours only
            pass
    return n


def make_communicator(ctx, kind: str = "auto") -> Communicator:
    """Pick the communicator for a :class:`~.dist.DistContext`.

    ``auto``: RCCL on GPUs (also at world size 1, so the bucket path runs the
    same code), torch.distributed on CPU, local when single-process on CPU.
    """
    if kind == "auto":
        if ctx.device.type == "cuda":
            kind = "rccl"
        elif ctx.world_size > 1:
            kind = "torch"
        else:
            kind = "local"
    kind = os.environ.get("IMAGENT_COMM", kind)  # operator override: rccl | torch | local
    if kind == "rccl":
        store = _default_store() if ctx.world_size > 1 else None
        try:
            return RcclCommunicator(ctx.rank, ctx.world_size, ctx.device, store)
        except RuntimeError as e:
            if ctx.world_size == 1 or not dist.is_initialized():
                raise
            # the bootstrap's failure flag makes every rank fail together (RcclCommunicator),
            # so all of them fall back to the c10d group together
            warnings.warn(f"own RCCL communicator unavailable ({e}); using the c10d process group")
            return TorchCommunicator(_fallback_group(ctx))
    if kind == "torch":
        if not dist.is_initialized():  # single process without a c10d group: nothing to reduce over
            return LocalCommunicator()
        return TorchCommunicator()
    return LocalCommunicator()
