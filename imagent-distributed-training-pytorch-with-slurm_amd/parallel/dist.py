"""Process-group bootstrap and teardown.

Reference: ``imagenet.py:267`` binds the device, ``imagenet.py:269-274`` calls
``init_process_group(init_method='env://', backend=backend)`` and prints the
backend; the reference never destroys the group. Here:

* ``backend='nccl'`` is RCCL on ROCm (c10d ``ProcessGroupNCCL``); the gradient
  all-reduce itself goes through our own RCCL communicator
  (:mod:`.comm`), the c10d group is kept for rendezvous, barriers and
  object broadcasts.
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

    def __init__(self, topo: Topology, backend: str, device: torch.device, initialized: bool):
        self.topo = topo
        self.backend = backend
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
            if self.backend == "nccl":
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
    if need_pg and not dist.is_initialized():
        if verbose:
            print("Initializing PyTorch distributed ...")
        kwargs = dict(init_method="env://", backend=backend,
                      timeout=datetime.timedelta(seconds=timeout_s),
                      world_size=topo.world_size, rank=topo.global_rank)
        if backend == "nccl":
            kwargs["device_id"] = dev
        dist.init_process_group(**kwargs)
        initialized = True
        if verbose:
            print(f"Backend: {dist.get_backend()}")
    elif dist.is_initialized():
        initialized = True
    return DistContext(topo, backend, dev, initialized)
