"""Metric helpers.

* :class:`AverageMeter` (host timings), :func:`accuracy` / :func:`topk_hits`,
  :func:`reduce_tensor` and :func:`to_python_float` keep the reference's
  semantics (``imagenet.py:44-94``) and are what the engine uses for host
  timings, the torch-path accuracy counters and the cross-rank reduction.
* :class:`DeviceMetrics` is what the engine actually uses: a 4-float device
  accumulator ``[loss_sum, top1_hits, top5_hits, rows]`` filled by the fused
  softmax-xent kernel, all-reduced ONCE per logging interval / epoch instead
  of three scalar all-reduces + three ``.item()`` host syncs per step
  (``imagenet.py:137-147``). Averages are weighted by the
  true number of samples (quirk Q1 of the reference - ``input[0].size(0)``
  is the channel count, 3 - is fixed; :attr:`DeviceMetrics.ref_mean` keeps the
  reference's unweighted per-batch mean available for comparisons).
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import torch
import torch.nn.functional as F


class AverageMeter:
    """Running value / count-weighted mean (the reference's meter, imagenet.py:44-60).

    The engine keeps its host-side timings in these (``batch_time``,
    ``data_time`` in :meth:`Trainer.train_epoch`); the device-side loss and
    accuracy live in :class:`DeviceMetrics` instead (no per-step host sync)."""

    __slots__ = ("name", "val", "sum", "count")

    def __init__(self, name: str = ""):
        self.name = name
        self.reset()

    def reset(self) -> None:
        self.val, self.sum, self.count = 0.0, 0.0, 0

    def update(self, val: float, n: int = 1) -> None:
        self.val = float(val)
        self.sum += self.val * n
        self.count += n

    @property
    def avg(self) -> float:
        return self.sum / self.count if self.count else 0.0

    def __str__(self) -> str:
        return f"{self.name} {self.val:.4f} ({self.avg:.4f})"


def topk_hits(output: torch.Tensor, target: torch.Tensor, topk: Sequence[int] = (1,)) -> torch.Tensor:
    """Number of rows whose target is among the top-k logits, one count per k
    (device tensor, no host sync)."""
    with torch.no_grad():
        ranked = output.topk(min(max(topk), output.shape[1]), 1).indices
        hit = ranked == target.reshape(-1, 1)
        return torch.stack([hit[:, :k].any(1).float().sum() for k in topk])


def accuracy(output: torch.Tensor, target: torch.Tensor, topk: Tuple[int, ...] = (1,)) -> List[torch.Tensor]:
    """Precision@k in percent, one 1-element tensor per k (imagenet.py:63-79)."""
    hits = topk_hits(output, target, topk) * (100.0 / target.size(0))
    return [h.reshape(1) for h in hits]


def reduce_tensor(tensor: torch.Tensor, world_size: int, comm=None, op: str = "mean") -> torch.Tensor:
    """Cross-rank mean (imagenet.py:82-87) or sum of a copy of ``tensor``,
    through our communicator when given (else c10d)."""
    rt = tensor.clone()
    if world_size > 1:
        if comm is not None:
            comm.allreduce_(rt, "sum")
            comm.join()
        elif torch.distributed.is_initialized():
            torch.distributed.all_reduce(rt)
    if op == "mean":
        rt /= world_size
    return rt


def to_python_float(t) -> float:
    """Host float of a 1-element tensor or a plain number / sequence (imagenet.py:90-94)."""
    if hasattr(t, "item"):
        return float(t.item())
    return float(t[0]) if isinstance(t, (list, tuple)) else float(t)


class DeviceMetrics:
    """Device-side loss/top-1/top-5 accumulator, reduced across ranks on demand."""

    def __init__(self, device):
        self.buf = torch.zeros(4, dtype=torch.float32, device=device)
        self.batches = 0
        self._batch_means: List[torch.Tensor] = []

    def reset(self):
        self.buf.zero_()
        self.batches = 0

    def update_from_logits(self, logits: torch.Tensor, target: torch.Tensor, loss: torch.Tensor):
        """Torch-path update (the HIP path's xent kernel accumulates itself)."""
        with torch.no_grad():
            B = target.numel()
            h1, h5 = topk_hits(logits, target, (1, 5))
            self.buf += torch.stack([loss.detach().float() * B, h1, h5,
                                     torch.tensor(float(B), device=self.buf.device)])
        self.batches += 1

    def count_batch(self):
        self.batches += 1

    def reduced(self, comm=None) -> Tuple[float, float, float, float]:
        """(mean loss, top1 %, top5 %, samples) over all ranks. One collective."""
        ws = comm.world_size if comm is not None else 1
        loss, t1, t5, n = reduce_tensor(self.buf, ws, comm, op="sum").tolist()
        n = max(n, 1.0)
        return loss / n, 100.0 * t1 / n, 100.0 * t5 / n, n
