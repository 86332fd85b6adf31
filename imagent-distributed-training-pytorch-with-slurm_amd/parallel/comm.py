"""Communicators: native RCCL (GPU) and torch.distributed (gloo/CPU, or c10d).

The reference's collectives are the DDP bucket all-reduce, the DDP init /
per-forward buffer broadcasts and three scalar metric all-reduces per step
(``imagenet.py:84-86,137-139``).

:class:`RcclCommunicator` owns its own RCCL communicator (bootstrapped through
the c10d TCPStore) and a highest-priority HIP stream: collectives are ordered
after the producing compute stream by an event and the compute stream joins
back with one event wait before the optimizer step. :class:`TorchCommunicator`
offers the same interface over ``torch.distributed`` (``gloo`` for CPU runs
and tests). :class:`LocalCommunicator` is the world-of-one no-op.
"""

from __future__ import annotations

import ctypes as C
import os
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

    def close(self) -> None:
        pass

    def depend_on(self, stream) -> None:
        """Collectives issued after this call also wait for ``stream``."""
        if torch.cuda.is_available():
            torch.cuda.current_stream().wait_stream(stream)


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


class RcclCommunicator(Communicator):
    """Our own RCCL communicator on a dedicated high-priority HIP stream."""

    name = "rccl"

    def __init__(self, rank: int, world_size: int, device: torch.device, store=None,
                 key: str = "imagent/rccl_uid"):
        from ..ops import _lib
        self._lib = _lib
        self.L = _lib.comm()
        self.rank, self.world_size = rank, world_size
        self.device = torch.device(device)
        nbytes = self.L.imc_unique_id_bytes()
        if rank == 0:
            buf = C.create_string_buffer(nbytes)
            rc = self.L.imc_get_unique_id(buf)
            uid = buf.raw if rc == 0 else b""
            if store is not None and world_size > 1:
                store.set(key, uid)  # an empty id tells the other ranks to fail with us, not wait
            self._chk(rc, "ncclGetUniqueId")
        else:
            if store is None:
                raise RuntimeError("RcclCommunicator needs a c10d store to bootstrap rank > 0")
            store.wait([key])
            uid = store.get(key)
            if len(uid) != nbytes:
                raise RuntimeError("rank 0 could not create an RCCL unique id")
        h = C.c_void_p()
        self._chk(self.L.imc_comm_init(uid, world_size, rank, self.device.index or 0, 64, C.byref(h)),
                  "ncclCommInitRank")
        self.h = h
        self.stream = torch.cuda.ExternalStream(self.L.imc_comm_stream(h), device=self.device)

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.L.imc_last_error().decode()} (rc={rc})")

    def _cur(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def allreduce_(self, t, op="sum"):
        assert t.is_cuda and t.is_contiguous()
        if self.world_size == 1:
            return  # a one-rank all-reduce is the identity: skip the RCCL copy kernel
        self._chk(self.L.imc_allreduce(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], _OP[op], self._cur()),
                  "allreduce")
        # keep the tensor alive until the comm stream is done with it
        t.record_stream(self.stream)

    def broadcast_(self, t, root=0):
        assert t.is_cuda and t.is_contiguous()
        self._chk(self.L.imc_broadcast(self.h, t.data_ptr(), t.numel(), _DT[t.dtype], root, self._cur()),
                  "broadcast")
        t.record_stream(self.stream)
        self.join()

    def allgather(self, t):
        t = t.contiguous()
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self._chk(self.L.imc_allgather(self.h, t.data_ptr(), out.data_ptr(), t.numel(), _DT[t.dtype],
                                       self._cur()), "allgather")
        out.record_stream(self.stream)
        self.join()
        return out

    def depend_on(self, stream) -> None:
        if self.world_size > 1:  # the comm stream waits; the compute stream keeps going
            self._chk(self.L.imc_stream_join_from(self.h, stream.cuda_stream), "join_from")

    def join(self):
        self._chk(self.L.imc_stream_join_into(self.h, self._cur()), "join")

    def synchronize(self):
        self._chk(self.L.imc_synchronize(self.h), "sync")

    def healthy(self) -> bool:
        return self.L.imc_async_error(self.h) == 0

    def close(self):
        if getattr(self, "h", None):
            self.L.imc_comm_destroy(self.h)
            self.h = None


def _default_store():
    try:
        from torch.distributed.distributed_c10d import _get_default_store
        return _get_default_store()
    except Exception:
        return None


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
            # every rank fails the same ncclCommInitRank, so all of them fall back together
            warnings.warn(f"own RCCL communicator unavailable ({e}); using the c10d process group")
            return TorchCommunicator()
    if kind == "torch":
        return TorchCommunicator()
    return LocalCommunicator()
