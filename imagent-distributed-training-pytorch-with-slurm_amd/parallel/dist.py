"""Process-group bootstrap and teardown.

Reference: ``imagenet.py:267`` binds the device, ``imagenet.py:269-274`` calls
``init_process_group(init_method='env://', backend=backend)`` and prints the
backend; the reference never destroys the group. Here:

* ``backend='nccl'`` means the collectives run on RCCL (ROCm's NCCL). They go
  through our OWN RCCL communicator (:mod:`.comm`), so the c10d default group
  is only bootstrap plumbing (TCPStore rendezvous, barriers, the bench's
  elapsed-time max): it is created with the CPU-side ``gloo`` backend, and a
  c10d ``ProcessGroupNCCL`` is created lazily, only on the fallback path where
  the own communicator cannot start (:func:`.comm.make_communicator`). Every
  rank then holds exactly ONE RCCL communicator and no c10d NCCL streams: the
  same stream / hardware-queue layout as the single-GPU bench, which the
  stream-order study (``profiles/r50_b1024_comm_stream_study.md``) showed is
  worth 12-26 % img/s. ``IMAGENT_C10D_BACKEND=nccl`` restores an eager c10d
  NCCL default group (A/B).
* ``backend='gloo'`` runs the whole framework on CPU (tests, plumbing).
* a configurable timeout and a clean ``shutdown()``.
"""

from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from .launcher import Topology


class DistContext:
    """The live distributed state of this process."""

    def __init__(self, topo: Topology, backend: str, device: torch.device, initialized: bool,
                 c10d_backend: Optional[str] = None):
        self.topo = topo
        self.backend = backend            # the collective backend the job asked for (--backend)
        self.c10d_backend = c10d_backend  # the c10d default group's backend (None: no group)
        self.device = device
        self.initialized = initialized

    @property
    def rank(self) -> int:
        return self.topo.global_rank

    @property
    def world_size(self) -> int:
        return self.topo.world_size

    @property
    def is_master(self) -> bool:
        return self.topo.global_rank == 0

    def barrier(self) -> None:
        if self.initialized and self.world_size > 1:
            if self.c10d_backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def shutdown(self) -> None:
        if self.initialized and dist.is_initialized():
            try:
                dist.destroy_process_group()
            finally:
                self.initialized = False


def init_distributed(topo: Topology, backend: str = "nccl", timeout_s: float = 1800.0,
                     device: Optional[str] = None, verbose: bool = True) -> DistContext:
    """Bind the device and initialise the default process group.

    ``device``: ``None`` picks ``cuda:<local_rank>`` when a GPU is visible and
    the CPU otherwise (``nccl`` then falls back to ``gloo`` with a warning).
    A world of one skips the process group entirely unless
    ``IMAGENT_FORCE_PG=1`` (our communicator degenerates to a no-op).
    """
    if device is None:
        device = f"cuda:{topo.local_rank}" if torch.cuda.is_available() else "cpu"
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)   # imagenet.py:267
    if backend == "nccl" and dev.type != "cuda":
        backend = "gloo"

    topo.export_env()
    need_pg = topo.world_size > 1 or os.environ.get("IMAGENT_FORCE_PG") == "1"
    initialized = False
    c10d = c10d_backend(backend)
    if need_pg and not dist.is_initialized():
        if verbose:
            print("Initializing PyTorch distributed ...")
        kwargs = dict(init_method="env://", backend=c10d,
                      timeout=datetime.timedelta(seconds=timeout_s),
                      world_size=topo.world_size, rank=topo.global_rank)
        if c10d == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
        initialized = True
        if verbose:   # imagenet.py:274 prints the backend
            print(f"Backend: {backend}" + (f" (collectives on the own RCCL communicator, c10d bootstrap group: "
                                           f"{dist.get_backend()})" if dist.get_backend() != backend else ""))
    elif dist.is_initialized():
        initialized = True
        c10d = dist.get_backend()
    return DistContext(topo, backend, dev, initialized, c10d if initialized else None)


def c10d_backend(backend: str) -> str:
    """Backend of the c10d default group for a job that asked for ``backend``:
    ``nccl`` jobs bootstrap over ``gloo`` (their collectives use the own RCCL
    communicator; module docstring), unless ``IMAGENT_C10D_BACKEND`` says otherwise."""
    forced = os.environ.get("IMAGENT_C10D_BACKEND")
    if forced:
        return forced
    return "gloo" if backend == "nccl" else backend
